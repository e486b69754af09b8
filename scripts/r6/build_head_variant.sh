#!/bin/bash
# A/B build: libh2omx_tree.so from the kernel sources of a commit (default
# HEAD), for comparing the working tree's kernels against it.  Output:
# h2omx/lib/variants/head/libh2omx_tree.so (H2OMX_LIB_DIR=h2omx/lib/variants/head).
# usage: build_head_variant.sh [REF]
set -e
cd "$(dirname "$0")/../.."
T=$(mktemp -d)
REF=${1:-HEAD}
for f in $(git ls-tree -r --name-only $REF h2omx/csrc | grep -E '\.(h|hip)$'); do git show $REF:$f > $T/$(basename $f); done
mkdir -p h2omx/lib/variants/head
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -munsafe-fp-atomics -I $T \
  -o h2omx/lib/variants/head/libh2omx_tree.so $T/tree_kernels.hip $T/sketch_kernels.hip
rm -rf $T
cd h2omx/lib/variants/head && for l in dense explain host metrics mlp p2p; do ln -sf ../../libh2omx_$l.so libh2omx_$l.so; done
ls -la libh2omx_tree.so
