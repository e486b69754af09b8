#!/bin/bash
# r6z: wider small-shard grids (N_CUS 512: more feature groups; TARGET_WGS 1024: more workgroups per group),
# 1.375M shard + loopback-8 (+ the 11M headline for TARGET_WGS), 3 reps interleaved
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6z
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
E=h2omx.models.tree.engine:HipTreeBuilder
S="--rows 1375000 --steps 50 --warmup 5 --fit-trees 0"
for r in 1 2 3; do
  for arm in "base $E.SMALL_SHARD=1" "ncu512 $E.N_CUS=512" "tw1024 $E.TARGET_WGS=1024"; do
    set -- $arm
    timeout -k 10 300 python3 scripts/r6/bench_ab.py $2 -- $S > $O/shard_$1_$r.json 2>> $O/err.log || exit 1
    timeout -k 10 300 python3 scripts/r6/bench_ab.py $2 -- $S --loopback-ranks 8 > $O/loop8_$1_$r.json 2>> $O/err.log || exit 1
  done
  timeout -k 10 300 python3 scripts/r6/bench_ab.py $E.SMALL_SHARD=1 -- --fit-trees 0 > $O/n1_base_$r.json 2>> $O/err.log || exit 1
  timeout -k 10 300 python3 scripts/r6/bench_ab.py $E.TARGET_WGS=1024 -- --fit-trees 0 > $O/n1_tw1024_$r.json 2>> $O/err.log || exit 1
done
