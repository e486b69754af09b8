#!/bin/bash
# reduce_split with several workgroups per (slot, feature) row (ticketed combine): tests + A/B
set -o pipefail
O=gpurun_out/r5ad
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_tree_gpu.py tests/test_hist_adaptive.py tests/test_estimators_gpu.py tests/test_p2p_gpu.py \
  tests/test_multirank_gpu.py > $O/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  for k in 1 16; do
    H2OMX_RS_SPLITS=$k timeout -k 10 300 python bench.py --steps 20 --warmup 3 --fit-trees 0 > $O/bench_k${k}_$rep.json 2> $O/bench_k${k}_$rep.err || exit 1
    H2OMX_RS_SPLITS=$k timeout -k 10 300 python bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0 > $O/bench1375_k${k}_$rep.json 2> $O/bench1375_k${k}_$rep.err || exit 1
  done
done
