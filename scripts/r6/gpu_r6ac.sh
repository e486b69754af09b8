#!/bin/bash
# r6ac: segmented kernels find their chunk's node by a wave 64-ary search instead of a serial binary search
# vs the committed kernels: seg-engine tests, DRF depth 20 A/B, level table
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6ac
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_gpu.py tests/test_hist_adaptive.py tests/test_tree_dp_gpu.py tests/test_estimators_gpu.py -m gpu > $O/pytest.log 2>&1 || exit 1
H=$GRAFT_REPO_ROOT/h2omx/lib/variants/head
for r in 1 2 3; do
  timeout -k 10 300 python3 scripts/drf_deep_ab.py 10000000 new > $O/drf_new_$r.jsonl 2>> $O/err.log || exit 1
  H2OMX_LIB_DIR=$H timeout -k 10 300 python3 scripts/drf_deep_ab.py 10000000 head > $O/drf_head_$r.jsonl 2>> $O/err.log || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drf -o drf -- python3 $GRAFT_REPO_ROOT/scripts/drf_deep_ab.py 10000000 newp > /dev/null 2> $O/drf_prof.err || exit 1
cd $GRAFT_REPO_ROOT
python3 scripts/level_breakdown.py $O/drf/drf_kernel_trace.csv 20 > $O/drf_levels.txt 2>&1 || true
