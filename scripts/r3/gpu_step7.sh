#!/bin/bash
# round 3, step 7: fp32 GEMM K sweep (kernel trace) + counters of the FULL kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3s7
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ksweep -o run -- python scripts/r3/gemm_ksweep.py > $O/ksweep.log 2>&1 || exit $?
i=0
for set in "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY"; do
  i=$((i+1)); OUT=$O/pmc$i; mkdir -p $OUT
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $OUT -o run -- python3 scripts/r3/gemm_pmc_run.py 1 1 > /dev/null 2> $OUT/err || { echo "pmc $i failed"; tail -5 $OUT/err; exit 1; }
  python3 scripts/pmc_summary.py $OUT > $OUT/summary.txt || exit 1
done
echo done
