#!/bin/bash
# r6a: per-kernel trace of the 1.375M-row shard (1 rank) vs the 8-rank loopback proxy
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6a
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0 --instrument-steps 0 --no-auc"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/shard -o shard -- $B > $O/shard.json 2> $O/shard.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/loop8 -o loop8 -- $B --loopback-ranks 8 > $O/loop8.json 2> $O/loop8.err || exit 1
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0 --loopback-ranks 8 > $O/loop8_$r.json 2>> $O/plain.err || exit 1
  timeout -k 10 300 python3 bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0 > $O/shard_$r.json 2>> $O/plain.err || exit 1
done
