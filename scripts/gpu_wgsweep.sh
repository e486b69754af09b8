#!/bin/bash
# Histogram grid sweep + timeline (GBM HIGGS 11M depth 5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m h2omx.build > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
for W in ${WGS:-256 512 1024}; do
  H2OMX_HIST_WGS=$W timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-auc > gpurun_out/wg.json 2> gpurun_out/wg.err || { tail -5 gpurun_out/wg.err; exit 1; }
  echo "WGS=$W $(python3 -c "import json; d=json.load(open('gpurun_out/wg.json')); print(d['ms_per_step'])")"
done
OUT=gpurun_out/prof_wg
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-auc > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 scripts/prof_summary.py "$OUT" > $OUT/summary.txt; sed -n '/one step/,$p' $OUT/summary.txt
