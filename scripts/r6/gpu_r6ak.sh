#!/bin/bash
# r6ak: deep-tree forest downloaded per tree by a helper thread: tree GPU tests, then DRF depth 20
# A/B vs the same build gathering h (ASYNC_DOWNLOAD=0), 3 reps interleaved, + level table of the new build
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6ak
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tree_gpu.py tests/test_hist_adaptive.py > $O/pytest.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python3 scripts/drf_deep_ab.py 10000000 new > $O/drf_new_$r.jsonl 2>> $O/err.log || exit 1
  timeout -k 10 300 python3 scripts/r6/bench_ab.py h2omx.models.tree.boost:GpuBooster.ASYNC_DOWNLOAD=0 -- scripts/drf_deep_ab.py 10000000 head > $O/drf_head_$r.jsonl 2>> $O/err.log || exit 1
done
timeout -k 10 600 python3 scripts/automl_bench.py --rows 10000000 --cols 100 > $O/automl.json 2> $O/automl.err || exit 1
