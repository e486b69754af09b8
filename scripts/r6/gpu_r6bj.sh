#!/bin/bash
# r6bj: DRF depth 20 segmented-histogram LDS budget below 16 KB,
# 3 reps interleaved
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6bj
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
E=h2omx.models.tree.engine:HipTreeBuilder
for r in 1 2 3; do
  for cfg in "SEG_LDS_BUDGET=16384" "SEG_LDS_BUDGET=12288" "SEG_LDS_BUDGET=8192" "SEG_LDS_BUDGET=4096"; do
    a=""; [ "$cfg" != base ] && a="$E.$cfg"
    timeout -k 10 300 python3 scripts/r6/bench_ab.py $a -- scripts/drf_deep_ab.py 10000000 $cfg > $O/drf_${cfg}_$r.jsonl 2>> $O/err.log || exit 1
  done
done
