#!/bin/bash
# Sweep hist-build launch configurations (LDS budget KB, threads, rows/lane, target WGs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python -m h2omx.build > gpurun_out/build.log 2>&1 || exit 1
OUT=gpurun_out/sweep_${1:-a}.txt
: > $OUT
for cfg in "64 512 16 512" "96 512 16 512" "128 1024 16 256" "150 1024 16 256" "64 512 8 512" "64 256 16 1024" "128 1024 16 512"; do
  set -- $cfg
  r=$(H2OMX_HIST_LDS_KB=$1 H2OMX_HIST_THREADS=$2 H2OMX_HIST_ROWS=$3 H2OMX_HIST_WGS=$4 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-auc 2>/dev/null) || { echo "cfg $cfg FAILED" | tee -a $OUT; exit 1; }
  ms=$(echo "$r" | python3 -c "import json,sys; print(round(json.loads(sys.stdin.read())['ms_per_step'],3))")
  echo "lds=$1KB threads=$2 rows=$3 wgs=$4 ms_per_step=$ms" | tee -a $OUT
done
