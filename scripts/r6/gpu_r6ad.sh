#!/bin/bash
# r6ad: level 4 routes its rows inside its histogram kernel (FUSE_MAX_PREV 8: no separate routing partition)
# vs 4, on the round-6 kernels: tree tests with the switch, GBM headline / shard / XGBoost, 3 reps interleaved
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6ad
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
E=h2omx.models.tree.engine:HipTreeBuilder
S="--rows 1375000 --steps 50 --warmup 5 --fit-trees 0"
for r in 1 2 3; do
  for v in 8 4; do
    timeout -k 10 300 python3 scripts/r6/bench_ab.py $E.FUSE_MAX_PREV=$v -- --fit-trees 0 > $O/n1_fp${v}_$r.json 2>> $O/err.log || exit 1
    timeout -k 10 300 python3 scripts/r6/bench_ab.py $E.FUSE_MAX_PREV=$v -- $S > $O/shard_fp${v}_$r.json 2>> $O/err.log || exit 1
    timeout -k 10 300 python3 scripts/r6/bench_ab.py $E.FUSE_MAX_PREV=$v -- --model xgboost-airlines --steps 20 --warmup 3 > $O/xgb_fp${v}_$r.json 2>> $O/err.log || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gbm8 -o gbm -- python3 $GRAFT_REPO_ROOT/scripts/r6/bench_ab.py $E.FUSE_MAX_PREV=8 -- --steps 20 --warmup 3 --instrument-steps 0 --no-auc --fit-trees 0 > /dev/null 2> $O/gbm8_prof.err || exit 1
