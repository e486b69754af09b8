#!/bin/bash
# r6ah: DRF depth 20 - segmented (in-bag rows only) histograms from shallower levels (HipTreeBuilder.SCAN_SLOTS),
# 3 reps interleaved + level table of SCAN_SLOTS=1
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6ah
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
E=h2omx.models.tree.engine:HipTreeBuilder
for r in 1 2 3; do
  for s in 1 0 16; do
    timeout -k 10 300 python3 scripts/r6/bench_ab.py $E.SCAN_SLOTS=$s -- scripts/drf_deep_ab.py 10000000 ss$s > $O/drf_ss${s}_$r.jsonl 2>> $O/err.log || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o drf -- python3 $GRAFT_REPO_ROOT/scripts/r6/bench_ab.py $E.SCAN_SLOTS=1 -- scripts/drf_deep_ab.py 10000000 prof > /dev/null 2> $O/prof.err || exit 1
cd $GRAFT_REPO_ROOT
python3 scripts/level_breakdown.py $O/prof/drf_kernel_trace.csv 20 > $O/levels.txt 2>&1 || true
