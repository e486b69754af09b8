#!/bin/bash
# PMC of the fused MLP step kernels (one counter set per run)
set -o pipefail
O=gpurun_out/r5g
mkdir -p $O
export REPLAYS=3
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_MFMA_F32 SQ_WAVES" \
           "FETCH_SIZE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/pmc$i -o run -- python3 scripts/mlp_step_bench.py > $O/pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -5 $O/pmc$i.log; exit 1; }
  python3 scripts/pmc_summary.py $O/pmc$i > $O/pmc$i.txt
done
