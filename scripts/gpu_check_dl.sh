#!/bin/bash
# tree / estimator GPU tests, GBM fit stages, DL fp32 kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_tree_gpu.py tests/test_estimators_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/tree_tests.log 2>&1 || { tail -30 gpurun_out/tree_tests.log; exit 1; }
tail -2 gpurun_out/tree_tests.log
timeout -k 10 300 python3 scripts/gbm_fit_stages.py > gpurun_out/fit_stages.txt 2>&1 || { tail -5 gpurun_out/fit_stages.txt; exit 1; }
tail -6 gpurun_out/fit_stages.txt
OUT=gpurun_out/dlprof
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --model dl-mlp --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
python3 scripts/prof_summary.py $OUT > $OUT/summary.txt 2>&1
head -70 $OUT/summary.txt
