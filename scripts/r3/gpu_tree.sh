#!/bin/bash
# Tree engine iteration: tree GPU tests, GBM headline bench, one-step kernel timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=${1:-tree}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_tree_gpu.py tests/test_estimators_gpu.py tests/test_multirank_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$TAG/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --fit-trees 0 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/bench.json')); print('gbm', round(d['ms_per_step'],4), 'ms/step auc', d['train_auc'], d.get('phase_us_per_tree'))"
OUT=gpurun_out/$TAG/prof; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-auc --fit-trees 0 --instrument-steps 0 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 scripts/prof_summary.py "$OUT" > $OUT/summary.txt; sed -n '/one step/,$p' $OUT/summary.txt
