#!/bin/bash
# r6i: counters of the DRF depth-20 kernels (what bounds the direct levels:
# issue / memory wait / LDS / L2 / translation), the GBM per-level PMC table for
# round 6, XGBoost Airlines-shape x3 with the leaf-sum replicas
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6i
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --model xgboost-airlines --steps 20 --warmup 3 > $O/xgb_$r.json 2>> $O/err.log || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
D="python3 $GRAFT_REPO_ROOT/scripts/r6/drf_pmc_run.py 10000000 2"
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU --output-format csv -d $O/drf_p1 -o run -- $D > $O/drf_p1.json 2> $O/drf_p1.err || exit 1
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/drf_p2 -o run -- $D > $O/drf_p2.json 2> $O/drf_p2.err || exit 1
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES FETCH_SIZE --output-format csv -d $O/drf_p3 -o run -- $D > $O/drf_p3.json 2> $O/drf_p3.err || exit 1
if grep -q "TCP_UTCL1_TRANSLATION_MISS" $O/counters.txt; then
  timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --output-format csv -d $O/drf_p4 -o run -- $D > $O/drf_p4.json 2> $O/drf_p4.err || exit 1
fi
cd $GRAFT_REPO_ROOT
python3 scripts/r6/pmc_by_kernel.py $O/drf_p1 $O/drf_p2 $O/drf_p3 $O/drf_p4 > $O/drf_pmc_table.txt 2>&1 || true
bash scripts/gpu_pmc_levels.sh r6i > $O/pmc_levels.log 2>&1 || exit 1
cp gpurun_out/pmc_r6i_table.txt $O/ 2>/dev/null || true
