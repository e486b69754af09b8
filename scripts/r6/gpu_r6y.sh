#!/bin/bash
# r6y: small-shard histogram grids re-measured on the round-6 kernels (SMALL_SHARD / N_CUS), 1.375M shard
# and loopback-8, 3 reps interleaved
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6y
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
E=h2omx.models.tree.engine:HipTreeBuilder
S="--rows 1375000 --steps 50 --warmup 5 --fit-trees 0"
for r in 1 2 3; do
  for arm in "base $E.SMALL_SHARD=1" "ncu128 $E.N_CUS=128" "noss $E.SMALL_SHARD=0"; do
    set -- $arm
    timeout -k 10 300 python3 scripts/r6/bench_ab.py $2 -- $S > $O/shard_$1_$r.json 2>> $O/err.log || exit 1
    timeout -k 10 300 python3 scripts/r6/bench_ab.py $2 -- $S --loopback-ranks 8 > $O/loop8_$1_$r.json 2>> $O/err.log || exit 1
  done
done
