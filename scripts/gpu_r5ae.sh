#!/bin/bash
# DL batch 8192: weight-gradient split-K target workgroups (256 = current, 512, 1024)
set -o pipefail
O=gpurun_out/r5ae2
mkdir -p $O
for rep in 1 2; do
  for w in 256 512 1024; do
    H2OMX_SPLITK_WGS=$w timeout -k 10 300 python bench.py --model dl-mlp --steps 100 --warmup 10 > $O/dl_w${w}_$rep.json 2> $O/dl_w${w}_$rep.err || exit 1
  done
done
