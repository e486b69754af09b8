#!/bin/bash
# round 3, step 4: monotone constraints + DRF OOB on the GPU, tree regression, bench;
# fp32 GEMM with 64 x 64 wave tiles (tests + microbench)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3s4
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_dense_gpu.py -k "gemm" > $O/pytest_gemm.log 2>&1 || exit $?
timeout -k 10 200 python scripts/r3/gemm_bench.py > $O/gemm_bench.jsonl 2> $O/gemm_bench.err || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_monotone.py tests/test_drf_oob.py tests/test_tree_gpu.py -m gpu > $O/pytest.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
echo done
