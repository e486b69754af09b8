#!/bin/bash
# r6aa: single-rank level finalisation folded into the reduce + split launch (FUSE_FIN_LOCAL) re-measured on
# the round-6 kernels: 1.375M shard and 11M headline, 3 reps interleaved
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6aa
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
E=h2omx.models.tree.engine:HipTreeBuilder
S="--rows 1375000 --steps 50 --warmup 5 --fit-trees 0"
for r in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 300 python3 scripts/r6/bench_ab.py $E.FUSE_FIN_LOCAL=$v -- $S > $O/shard_ff${v}_$r.json 2>> $O/err.log || exit 1
    timeout -k 10 300 python3 scripts/r6/bench_ab.py $E.FUSE_FIN_LOCAL=$v -- --fit-trees 0 > $O/n1_ff${v}_$r.json 2>> $O/err.log || exit 1
  done
done
