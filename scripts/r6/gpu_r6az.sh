#!/bin/bash
# r6az: out-of-bag walk loading the 16-byte node header only; DRF depth 20 (3 reps), compared with r6at / r6ax
# + kernel stats
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6az
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tree_gpu.py -k "bag or async or mean or deep or rowmajor" > $O/pytest.log 2>&1 || exit 1
E=h2omx.models.tree.engine:HipTreeBuilder
for r in 1 2 3; do
  timeout -k 10 300 python3 scripts/drf_deep_ab.py 10000000 new > $O/drf_new_$r.jsonl 2>> $O/err.log || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o drf -- python3 $GRAFT_REPO_ROOT/scripts/drf_deep_ab.py 10000000 prof > /dev/null 2> $O/prof.err || exit 1
cd $GRAFT_REPO_ROOT
python3 scripts/level_breakdown.py $O/prof/drf_kernel_trace.csv 20 > $O/levels.txt 2>&1 || true
