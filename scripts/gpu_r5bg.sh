#!/bin/bash
# loopback-8 A/B on one box: current tree (new) vs the tree package of a3a28c1 (old = before the edge preloading)
set -o pipefail
O=gpurun_out/r5bg
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0 --loopback-ranks 8 > $O/new_$rep.json 2> $O/new_$rep.err || exit 1
  (cd ab_old && timeout -k 10 300 python bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0 --loopback-ranks 8 > ../$O/old_$rep.json 2> ../$O/old_$rep.err) || exit 1
done
