#!/bin/bash
# r6ba: out-of-bag walk on a side stream overlapping the last partition (BAG_OVERLAP) vs after it, DRF depth 20,
# 3 reps interleaved, + bag tests
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6ba
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tree_gpu.py -k "bag or async or mean or deep" > $O/pytest.log 2>&1 || exit 1
E=h2omx.models.tree.engine:HipTreeBuilder
for r in 1 2 3; do
  timeout -k 10 300 python3 scripts/drf_deep_ab.py 10000000 new > $O/drf_new_$r.jsonl 2>> $O/err.log || exit 1
  timeout -k 10 300 python3 scripts/r6/bench_ab.py $E.BAG_OVERLAP=0 -- scripts/drf_deep_ab.py 10000000 head > $O/drf_head_$r.jsonl 2>> $O/err.log || exit 1
done
