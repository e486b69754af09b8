#!/bin/bash
# Hardware counters of the GBM step (each counter set in its own rocprofv3 run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc}
python -m h2omx.build > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
i=0
for set in "SQ_INSTS_LDS_ATOMIC SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "FETCH_SIZE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "LdsBankConflict LdsUtil MemUnitStalled OccupancyPercent"; do
  i=$((i+1))
  OUT=gpurun_out/${TAG}_$i
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-auc > $OUT/bench.json 2> $OUT/bench.err || { echo "pmc set $i failed"; tail -5 $OUT/bench.err; exit 1; }
  python3 scripts/pmc_summary.py $OUT > $OUT/summary.txt
  cat $OUT/summary.txt | head -14
done
