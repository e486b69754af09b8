#!/bin/bash
# r6bh: DRF depth 20 segmented-histogram LDS budget and row-chunk cap,
# 3 reps interleaved
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6bh
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
E=h2omx.models.tree.engine:HipTreeBuilder
for r in 1 2 3; do
  for cfg in "base" "SEG_LDS_BUDGET=32768" "SEG_LDS_BUDGET=98304" "ROWS_CAP=131072" "ROWS_CAP=524288"; do
    a=""; [ "$cfg" != base ] && a="$E.$cfg"
    timeout -k 10 300 python3 scripts/r6/bench_ab.py $a -- scripts/drf_deep_ab.py 10000000 $cfg > $O/drf_${cfg}_$r.jsonl 2>> $O/err.log || exit 1
  done
done
