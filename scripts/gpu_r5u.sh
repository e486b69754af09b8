#!/bin/bash
# final partition: batched split-code gathers and fewer LDS leaf-sum copies (occupancy)
set -o pipefail
O=gpurun_out/r5u
mkdir -p $O
export PYTHONUNBUFFERED=1
H2OMX_PART_BATCH=1 H2OMX_PART_COPIES=8 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 \
  --timeout-method thread -m gpu tests/test_tree_gpu.py > $O/pytest_batch.log 2>&1 || exit 1
for rep in 1 2; do
  for cfg in "0 64" "1 64" "0 8" "0 16" "1 8" "1 16"; do
    set -- $cfg
    H2OMX_PART_BATCH=$1 H2OMX_PART_COPIES=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 3 \
      --fit-trees 0 > $O/bench_b$1_c$2_$rep.json 2> $O/bench_b$1_c$2_$rep.err || exit 1
  done
done
