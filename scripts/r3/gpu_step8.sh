#!/bin/bash
# round 3, step 8: interleaved FULL GEMM pipeline: tests, K sweep, microbench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3s8
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_dense_gpu.py -k "gemm" > $O/pytest_gemm.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ksweep -o run -- python scripts/r3/gemm_ksweep.py > $O/ksweep.log 2>&1 || exit $?
timeout -k 10 200 python scripts/r3/gemm_bench.py > $O/gemm_bench.jsonl 2> $O/gemm_bench.err || exit $?
echo done
