#!/bin/bash
# r6bb: 1.375M-row shard (11M / 8) and its loopback-8 sequence - partition grid / histogram workgroup targets,
# 3 reps interleaved
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6bb
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
E=h2omx.models.tree.engine:HipTreeBuilder
S="--rows 1375000 --steps 50 --warmup 5 --fit-trees 0"
for r in 1 2 3; do
  for cfg in "base" "PART_BLOCKS=512" "PART_BLOCKS=256" "TARGET_WGS=256" "TARGET_WGS=1024"; do
    a=""; [ "$cfg" != base ] && a="$E.$cfg"
    timeout -k 10 300 python3 scripts/r6/bench_ab.py $a -- $S > $O/shard_${cfg}_$r.json 2>> $O/err.log || exit 1
  done
done
