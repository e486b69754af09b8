#!/bin/bash
# round 3, step 6: fp32 GEMM FULL pipeline (load-to-use one K-step), small-batch split-K
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3s6
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_dense_gpu.py tests/test_estimators_gpu.py -k "gemm or deeplearning" > $O/pytest_gemm.log 2>&1 || exit $?
timeout -k 10 200 python scripts/r3/gemm_bench.py > $O/gemm_bench.jsonl 2> $O/gemm_bench.err || exit $?
timeout -k 10 200 python bench.py --model dl-mlp --estimator-defaults --steps 300 --warmup 30 > $O/bench_dl_estdef.json 2> $O/bench_dl_estdef.err || exit $?
echo done
