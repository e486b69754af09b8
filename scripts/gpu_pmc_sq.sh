#!/bin/bash
# Per-dispatch SQ instruction-mix / stall counters of one GBM step.
# Usage: gpu_pmc_sq.sh TAG "COUNTERS" ["COUNTERS2" ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
i=0
for set in "$@"; do
  i=$((i+1))
  OUT=gpurun_out/pmc_${TAG}_$i
  mkdir -p $OUT
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-auc > $OUT/bench.json 2> $OUT/bench.err || { echo "pmc set $i failed"; tail -5 $OUT/bench.err; exit 1; }
  python3 scripts/pmc_dispatch.py $OUT 26 hist_build partition boost > $OUT/dispatch.txt
  cat $OUT/dispatch.txt
done
