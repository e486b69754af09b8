#!/bin/bash
# split-K reduce with float4 columns and loads in flight: dense / DL GPU tests, DL bench, kernel stats
set -o pipefail
O=gpurun_out/r5ai
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dense_gpu.py tests/test_dl_step_gpu.py tests/test_estimators_gpu.py > $O/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --model dl-mlp --steps 100 --warmup 10 > $O/dl_$rep.json 2> $O/dl_$rep.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o dl -- python3 $GRAFT_REPO_ROOT/bench.py --model dl-mlp --steps 30 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
