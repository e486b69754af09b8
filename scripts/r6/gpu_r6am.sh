#!/bin/bash
# r6am: per-tree forest download through a pinned stage: tree GPU tests, then DRF depth 20
# A/B vs the same build gathering h (DOWNLOAD_PINNED=0), 3 reps interleaved, + level table of the new build
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6am
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tree_gpu.py -k "async or mean_leaves or rowmajor" > $O/pytest.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python3 scripts/drf_deep_ab.py 10000000 new > $O/drf_new_$r.jsonl 2>> $O/err.log || exit 1
  timeout -k 10 300 python3 scripts/r6/bench_ab.py h2omx.models.tree.boost:GpuBooster.DOWNLOAD_PINNED=0 -- scripts/drf_deep_ab.py 10000000 head > $O/drf_head_$r.jsonl 2>> $O/err.log || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o drf -- python3 $GRAFT_REPO_ROOT/scripts/drf_deep_ab.py 10000000 prof > /dev/null 2> $O/prof.err || exit 1
cd $GRAFT_REPO_ROOT
python3 scripts/level_breakdown.py $O/prof/drf_kernel_trace.csv 20 > $O/levels.txt 2>&1 || true
