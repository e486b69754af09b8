#!/bin/bash
# fused MLP step A/B: load depth x tile shape
set -o pipefail
O=gpurun_out/r5e
mkdir -p $O
for D in 1 2 4 6; do
  for T in auto 1,1 1,2 2,2; do
    if [ "$T" = auto ]; then unset H2OMX_MLP_TILE; else export H2OMX_MLP_TILE=$T; fi
    H2OMX_MLP_DEPTH=$D timeout -k 10 120 python scripts/mlp_step_bench.py >> $O/ab.jsonl 2>> $O/ab.err || exit 1
  done
done
unset H2OMX_MLP_TILE
H2OMX_MLP_DEPTH=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_d1 -o p -- python scripts/mlp_step_bench.py > $O/prof_d1.log 2>&1 || exit 1
