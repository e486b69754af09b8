#!/bin/bash
# Per-dispatch memory / LDS counters of one GBM tree (HIGGS 11M x 28, depth 5),
# eager dispatches (no graph), two counter passes merged into one level table.
# Usage: gpu_pmc_levels.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-lv}
i=0
dirs=""
for set in "FETCH_SIZE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "WRITE_SIZE SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  OUT=gpurun_out/pmc_${TAG}_$i
  mkdir -p $OUT
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $OUT -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-auc --tree-graph 0 --fit-trees 0 --instrument-steps 0 > $OUT/bench.json 2> $OUT/bench.err || { echo "pmc set $i failed"; tail -5 $OUT/bench.err; exit 1; }
  dirs="$dirs $OUT"
done
python3 scripts/pmc_levels_table.py $dirs > gpurun_out/pmc_${TAG}_table.txt
cat gpurun_out/pmc_${TAG}_table.txt
