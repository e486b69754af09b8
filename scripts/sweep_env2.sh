#!/bin/bash
# env-var sweep of the GBM bench with extra bench arguments (BENCH_ARGS):
# one line per config in gpurun_out/sweep_$SWEEP_TAG.txt
out=gpurun_out/sweep_${SWEEP_TAG:-x}.txt
: > $out
for cfg in "$@"; do
  tag=${cfg%%:*}; vars=${cfg#*:}
  [ "$vars" = "$cfg" ] && vars=""
  line=$(env $(echo "$vars" | tr ',' ' ') timeout -k 10 120 python3 bench.py --steps 40 --warmup 4 --fit-trees 0 $BENCH_ARGS 2>/dev/null | tail -1) || { echo "$tag FAILED" >> $out; exit 1; }
  echo "$tag $vars $(echo "$line" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), round(d["train_auc"],6))')" >> $out
done
cat $out
