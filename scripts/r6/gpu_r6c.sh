#!/bin/bash
# r6c: loopback-8 (reduce-scatter + write-through) x3 vs the timing-only fenced variant x3,
# 1.375M shard x3, headline N=1 x3, kernel traces of loopback-8 and of the 11M headline
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6c
mkdir -p $O
cd $GRAFT_REPO_ROOT
B="python3 bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0"
for r in 1 2 3; do
  timeout -k 10 300 $B --loopback-ranks 8 > $O/loop8_$r.json 2>> $O/plain.err || exit 1
  H2OMX_LIB_DIR=h2omx/lib/variants/fenced timeout -k 10 300 $B --loopback-ranks 8 > $O/loop8_fenced_$r.json 2>> $O/plain.err || exit 1
  timeout -k 10 300 $B > $O/shard_$r.json 2>> $O/plain.err || exit 1
  timeout -k 10 300 python3 bench.py > $O/n1_$r.json 2>> $O/plain.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/loop8 -o loop8 -- python3 $GRAFT_REPO_ROOT/bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0 --instrument-steps 0 --no-auc --loopback-ranks 8 > $O/loop8.json 2> $O/loop8.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/n1 -o n1 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --fit-trees 0 --instrument-steps 0 --no-auc > $O/n1.json 2> $O/n1.err || exit 1
