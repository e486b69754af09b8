#!/bin/bash
# env-var sweep of the headline GBM bench: one line per config in gpurun_out/sweep.txt
out=gpurun_out/sweep.txt
: > $out
run() {
  local tag="$1"; shift
  local line
  line=$(env "$@" timeout -k 10 120 python bench.py --steps 30 --fit-trees 0 2>/dev/null | tail -1) || { echo "$tag FAILED" >> $out; return 1; }
  echo "$tag $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), round(d["train_auc"],6))')" >> $out
}
for cfg in "$@"; do
  # cfg: tag=base or tag:VAR=val,VAR=val
  tag=${cfg%%:*}; vars=${cfg#*:}
  [ "$vars" = "$cfg" ] && vars=""
  run "$tag" $(echo "$vars" | tr ',' ' ') H2OMX_SWEEP=1 || exit 1
done
