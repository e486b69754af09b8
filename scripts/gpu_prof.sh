#!/bin/bash
# Kernel timeline of one GBM step.  Usage: gpu_prof.sh TAG [bench args...]; env passes through.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-auc "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 scripts/prof_summary.py "$OUT" > $OUT/summary.txt; sed -n '/one step/,$p' $OUT/summary.txt
