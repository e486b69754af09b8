#!/bin/bash
# r6ap: DRF depth 20 with DIRECT_WAVE_ROWS 512: direct levels from more nodes, segmented-histogram chunking,
# 3 reps interleaved + level table of the default
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6ap
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
E=h2omx.models.tree.engine:HipTreeBuilder
for r in 1 2 3; do
  for cfg in "base" "DIRECT_MIN_NODES=2048" "SEG_TARGET_CHUNKS=2048" "SEG_TARGET_CHUNKS=512"; do
    a=""; [ "$cfg" != base ] && a="$E.$cfg"
    timeout -k 10 300 python3 scripts/r6/bench_ab.py $a -- scripts/drf_deep_ab.py 10000000 $cfg > $O/drf_${cfg}_$r.jsonl 2>> $O/err.log || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o drf -- python3 $GRAFT_REPO_ROOT/scripts/drf_deep_ab.py 10000000 prof > /dev/null 2> $O/prof.err || exit 1
cd $GRAFT_REPO_ROOT
python3 scripts/level_breakdown.py $O/prof/drf_kernel_trace.csv 20 > $O/levels.txt 2>&1 || true
