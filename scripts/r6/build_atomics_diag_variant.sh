#!/bin/bash
# Timing-only diagnostic (wrong leaf sums by construction, never a product build):
# the partition kernels' per-workgroup fold of the leaf-sum window adds into
# global memory from 1 workgroup in 16 only, to price the contention of 1024
# workgroups x ~189 device-scope 64-bit atomics on the same addresses.
# Output: h2omx/lib/variants/atomdiag/libh2omx_tree.so
set -e
cd "$(dirname "$0")/../.."
T=$(mktemp -d)
cp h2omx/csrc/*.h h2omx/csrc/tree_kernels.hip h2omx/csrc/sketch_kernels.hip $T/
python3 - "$T/tree_kernels.hip" <<'PY'
import sys
p = sys.argv[1]
s = open(p).read()
a = "        if (v && base + t / 3 < cap) atomicAdd(leaf_acc + 3 * base + t, v);"
assert s.count(a) == 1
s = s.replace(a, "        if (v && base + t / 3 < cap && (blockIdx.x & 15) == 0) atomicAdd(leaf_acc + 3 * base + t, v);")
open(p, "w").write(s)
PY
mkdir -p h2omx/lib/variants/atomdiag
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -munsafe-fp-atomics -I $T \
  -o h2omx/lib/variants/atomdiag/libh2omx_tree.so $T/tree_kernels.hip $T/sketch_kernels.hip
rm -rf $T
cd h2omx/lib/variants/atomdiag && for l in dense explain host metrics mlp p2p; do ln -sf ../../libh2omx_$l.so libh2omx_$l.so; done
ls -la libh2omx_tree.so
