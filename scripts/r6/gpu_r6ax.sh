#!/bin/bash
# r6ax: DRF depth 20 readback / close / partition thresholds on the final kernels,
# 3 reps interleaved
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6ax
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
E=h2omx.models.tree.engine:HipTreeBuilder
for r in 1 2 3; do
  for cfg in "base" "SYNC_NODE_CAP=2048" "CLOSE_SINGLE_BLOCK=1024" "CLOSE_SINGLE_BLOCK=4096" "PART_WAVE_NODES=4096"; do
    a=""; [ "$cfg" != base ] && a="$E.$cfg"
    timeout -k 10 300 python3 scripts/r6/bench_ab.py $a -- scripts/drf_deep_ab.py 10000000 $cfg > $O/drf_${cfg}_$r.jsonl 2>> $O/err.log || exit 1
  done
done
