#!/bin/bash
# Per-dispatch memory / LDS counters of one GBM step (HIGGS 11M x 28, depth 5).
# Usage: gpu_pmc_levels.sh TAG   (env passes through to bench.py, e.g. H2OMX_HIST_CMP=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-lv}
i=0
for set in "FETCH_SIZE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "WRITE_SIZE SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  OUT=gpurun_out/pmc_${TAG}_$i
  mkdir -p $OUT
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-auc > $OUT/bench.json 2> $OUT/bench.err || { echo "pmc set $i failed"; tail -5 $OUT/bench.err; exit 1; }
  python3 scripts/pmc_dispatch.py $OUT 26 > $OUT/dispatch.txt
  cat $OUT/dispatch.txt
done
