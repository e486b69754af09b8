#!/bin/bash
# loopback-8 proxy repeatability (1.375M rows, the 8-rank launch sequence on one GPU), 3 reps + the single-rank shard
set -o pipefail
O=gpurun_out/r5bf
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0 --loopback-ranks 8 > $O/loop8_$rep.json 2> $O/loop8_$rep.err || exit 1
done
timeout -k 10 300 python bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0 > $O/shard.json 2> $O/shard.err || exit 1
