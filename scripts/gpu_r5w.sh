#!/bin/bash
# batched final partition (default now): tests; histogram code-load prefetch depth A/B
# (H2OMX_HB_PF 1 / 2 / 4 builds); XGBoost Airlines and AutoML 10M x 100 records
set -o pipefail
O=gpurun_out/r5w
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_tree_gpu.py tests/test_hist_adaptive.py tests/test_p2p_gpu.py > $O/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  for pf in 1 2 4; do
    if [ $pf = 1 ]; then LD=""; else LD="$PWD/h2omx/lib_pf$pf"; fi
    H2OMX_LIB_DIR=$LD timeout -k 10 300 python bench.py --steps 20 --warmup 3 --fit-trees 0 \
      > $O/bench_pf${pf}_$rep.json 2> $O/bench_pf${pf}_$rep.err || exit 1
  done
done
timeout -k 10 300 python bench.py --model xgboost-airlines --steps 10 --warmup 2 > $O/bench_xgb.json 2> $O/bench_xgb.err || exit 1
timeout -k 10 400 python scripts/automl_bench.py --rows 10000000 --cols 100 > $O/automl.json 2> $O/automl.err || exit 1
