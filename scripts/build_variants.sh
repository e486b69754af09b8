#!/bin/bash
# Build tree-kernel tuning variants: build_variants.sh NAME "-DFLAG=V ..." [NAME2 "FLAGS2" ...]
# Output: h2omx/lib/variants/NAME/libh2omx_tree.so (load with H2OMX_LIB_DIR=h2omx/lib/variants/NAME)
set -e
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  d=h2omx/lib/variants/$1; mkdir -p $d
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -munsafe-fp-atomics -I h2omx/csrc $2 \
    -o $d/libh2omx_tree.so h2omx/csrc/tree_kernels.hip 2>&1 | grep -E "error" || true
  ls $d/libh2omx_tree.so
  shift 2
done
