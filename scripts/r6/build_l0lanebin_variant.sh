#!/bin/bash
# Timing-only diagnostic (wrong level-0 histograms by construction, never a
# product build): the level-0 lane-copy histogram atomics (COP 8) address bin
# (lane / 8) + 8 x (a code bit) instead of the row's code, i.e. every lane of
# a wave hits its own 64-bit word - bank-conflict-free - while the code loads
# stay live.  Prices the level-0 LDS bank conflicts (PMC: 49 % of LDS cycles).
# Output: h2omx/lib/variants/l0lanebin/libh2omx_tree.so
set -e
cd "$(dirname "$0")/../.."
T=$(mktemp -d)
cp h2omx/csrc/*.h h2omx/csrc/tree_kernels.hip h2omx/csrc/sketch_kernels.hip $T/
python3 - "$T/tree_kernels.hip" <<'PY'
import sys
p = sys.argv[1]
s = open(p).read()
a = "if (so[r] >= 0) atomicAdd(hb + (so[r] + ((cw[r >> 2] >> (8 * (r & 3))) & 0xff)) * COP, pk[r]);"
assert s.count(a) == 1
s = s.replace(a, "if (so[r] >= 0) atomicAdd(hb + (so[r] + (lane >> 3) + ((cw[r >> 2] >> (31 - (r & 3))) & 1u) * 8) * COP, pk[r]);")
open(p, "w").write(s)
PY
mkdir -p h2omx/lib/variants/l0lanebin
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -munsafe-fp-atomics -I $T \
  -o h2omx/lib/variants/l0lanebin/libh2omx_tree.so $T/tree_kernels.hip $T/sketch_kernels.hip
rm -rf $T
cd h2omx/lib/variants/l0lanebin && for l in dense explain host metrics mlp p2p; do ln -sf ../../libh2omx_$l.so libh2omx_$l.so; done
ls -la libh2omx_tree.so
