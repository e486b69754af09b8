#!/bin/bash
# GLM / K-Means kernel time + MFMA counters at the AutoML shape (10M x 100).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dpmc
export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/dense_pmc_run.py 5 > gpurun_out/dpmc/timing.json 2> gpurun_out/dpmc/timing.err || { tail -5 gpurun_out/dpmc/timing.err; exit 1; }
cat gpurun_out/dpmc/timing.json
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dpmc/trace -o run -- python3 scripts/dense_pmc_run.py 3 > /dev/null 2> gpurun_out/dpmc/trace.err || { tail -5 gpurun_out/dpmc/trace.err; exit 1; }
i=0
for set in "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU_MFMA_F32" \
           "FETCH_SIZE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS"; do
  i=$((i+1)); OUT=gpurun_out/dpmc/pmc$i; mkdir -p $OUT
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT -o run -- python3 scripts/dense_pmc_run.py 2 > /dev/null 2> $OUT/err || { echo "pmc $i failed"; tail -5 $OUT/err; exit 1; }
  python3 scripts/pmc_summary.py $OUT > $OUT/summary.txt; head -8 $OUT/summary.txt
done
