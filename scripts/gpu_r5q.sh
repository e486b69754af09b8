#!/bin/bash
# x3 data / weight gradients, fused level finalisation: tests, DL bench + kernel
# stats, GBM bench, GBM per-level PMC table
set -o pipefail
O=gpurun_out/r5q
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_dense_gpu.py tests/test_dl_step_gpu.py tests/test_tree_gpu.py tests/test_hist_adaptive.py \
  tests/test_estimators_gpu.py tests/test_p2p_gpu.py tests/test_tree_dp_gpu.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model dl-mlp --steps 100 --warmup 10 > $O/bench_dl.json 2> $O/bench_dl.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench_n1.json 2> $O/bench_n1.err || exit 1
export TMPDIR=/tmp
mkdir -p $O/prof_dl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dl -o run -- \
  python bench.py --model dl-mlp --steps 30 --warmup 5 > $O/prof_dl/bench.json 2> $O/prof_dl/bench.err || exit 1
./scripts/gpu_pmc_levels.sh r5q > $O/pmc.txt 2>&1 || exit 1
