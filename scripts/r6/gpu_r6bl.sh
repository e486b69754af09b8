#!/bin/bash
# r6bl: 16 KB segmented-histogram budget as the default: tree GPU tests, DRF depth 20 (3 reps), AutoML
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6bl
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tree_gpu.py tests/test_hist_adaptive.py -p no:cacheprovider > $O/pytest.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python3 scripts/drf_deep_ab.py 10000000 new > $O/drf_new_$r.jsonl 2>> $O/err.log || exit 1
done
timeout -k 10 600 python3 scripts/automl_bench.py --rows 10000000 --cols 100 > $O/automl.json 2> $O/automl.err || exit 1
