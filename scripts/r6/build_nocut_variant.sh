#!/bin/bash
# A/B build (not a product build): the UniformAdaptive candidate scan without
# the per-wave cut tables (ua_count's division form on every boundary, as
# before round 6).  Output: h2omx/lib/variants/nocut/libh2omx_tree.so
# (H2OMX_LIB_DIR=h2omx/lib/variants/nocut).
set -e
cd "$(dirname "$0")/../.."
T=$(mktemp -d)
cp h2omx/csrc/*.h h2omx/csrc/tree_kernels.hip h2omx/csrc/sketch_kernels.hip $T/
python3 - "$T/tree_kernels.hip" <<'PY'
import sys
p = sys.argv[1]
s = open(p).read()
a = "  if (mode == 1 && cut_tab != nullptr && nb <= 64) {"
assert s.count(a) == 1
s = s.replace(a, "  if (mode == 1 && cut_tab != nullptr && nb < 0) {")
open(p, "w").write(s)
PY
mkdir -p h2omx/lib/variants/nocut
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -munsafe-fp-atomics -I $T \
  -o h2omx/lib/variants/nocut/libh2omx_tree.so $T/tree_kernels.hip $T/sketch_kernels.hip
rm -rf $T
cd h2omx/lib/variants/nocut && for l in dense explain host metrics mlp p2p; do ln -sf ../../libh2omx_$l.so libh2omx_$l.so; done
ls -la libh2omx_tree.so
