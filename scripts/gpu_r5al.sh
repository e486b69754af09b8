#!/bin/bash
# XGBoost Airlines-shape histogram knob sweep (LDS budget per workgroup, fused-routing depth, grid)
set -o pipefail
O=gpurun_out/r5al
mkdir -p $O
run() {
  tag=$1; shift
  env "$@" timeout -k 10 240 python bench.py --model xgboost-airlines --steps 20 --warmup 3 --fit-trees 0 --instrument-steps 0 > $O/xgb_$tag.json 2> $O/xgb_$tag.err || exit 1
}
run base H2OMX_HIST_LDS_KB=64
run lds96 H2OMX_HIST_LDS_KB=96
run lds128 H2OMX_HIST_LDS_KB=128
run fuse8 H2OMX_FUSE_MAX_PREV=8
run fuse16 H2OMX_FUSE_MAX_PREV=16
run wgs1024 H2OMX_HIST_WGS=1024
run wgs768 H2OMX_HIST_WGS=768
run base2 H2OMX_HIST_LDS_KB=64
run lds152 H2OMX_HIST_LDS_KB=152
