#!/bin/bash
# after removing the slower variants: dense / DL tests, DL + GBM benches, GBM per-level PMC table
set -o pipefail
O=gpurun_out/r5r
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_dense_gpu.py tests/test_dl_step_gpu.py tests/test_tree_gpu.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model dl-mlp --steps 100 --warmup 10 > $O/bench_dl.json 2> $O/bench_dl.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench_n1.json 2> $O/bench_n1.err || exit 1
bash ./scripts/gpu_pmc_levels.sh r5r > $O/pmc.txt 2>&1 || exit 1
