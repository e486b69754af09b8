#!/bin/bash
# regression after pruning the lost A/B paths: tree / DL / P2P GPU suites + headline bench
set -o pipefail
O=gpurun_out/r5n
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_tree_gpu.py tests/test_dl_step_gpu.py tests/test_estimators_gpu.py tests/test_p2p_gpu.py \
  tests/test_multirank_gpu.py tests/test_tree_dp_gpu.py tests/test_dl_bf16.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench_n1.json 2> $O/bench_n1.err || exit 1
timeout -k 10 300 python bench.py --model dl-mlp --estimator-defaults --steps 400 --warmup 40 > $O/bench_dlest.json 2> $O/bench_dlest.err || exit 1
timeout -k 10 200 python scripts/gemm_x3_bench.py > $O/gemm_x3.txt 2>&1 || exit 1
