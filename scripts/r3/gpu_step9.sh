#!/bin/bash
# round 3, step 9: FULL w64 GEMM as default + fused dact in the DL backward
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3s9
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_dense_gpu.py tests/test_estimators_gpu.py tests/test_dl_bf16.py -k "gemm or deeplearning or act_backward or bf16 or mlp" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --model dl-mlp --steps 30 --warmup 5 > $O/bench_dl_fp32.json 2> $O/bench_dl_fp32.err || exit $?
timeout -k 10 200 python bench.py --model dl-mlp --estimator-defaults --steps 300 --warmup 30 > $O/bench_dl_estdef.json 2> $O/bench_dl_estdef.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dl -o run -- python bench.py --model dl-mlp --steps 10 --warmup 3 > $O/prof_dl.log 2>&1 || exit $?
echo done
