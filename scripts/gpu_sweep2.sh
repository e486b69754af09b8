#!/bin/bash
# bench sweep of an env knob: gpu_sweep2.sh VAR v1 v2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python -m h2omx.build > gpurun_out/build.log 2>&1 || exit 1
VAR=$1; shift
for v in "$@"; do
  env $VAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-auc > gpurun_out/sw_$v.json 2> gpurun_out/sw_$v.err || { tail -5 gpurun_out/sw_$v.err; exit 1; }
  echo "$VAR=$v $(python3 -c "import json;print(json.load(open('gpurun_out/sw_$v.json'))['ms_per_step'])")"
done
