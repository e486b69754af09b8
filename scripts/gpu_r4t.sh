# round 4: GLM split kernel counters (where do 15k cycles per 32-row chunk go?),
# K-Means NA-free timing, DL estimator weight-gradient side stream A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4t
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/r4t/counters.txt 2>&1 || true
timeout -k 10 120 python3 scripts/dense_pmc_run.py 5 na_free > gpurun_out/r4t/dense_nafree.json 2> gpurun_out/r4t/dense_nafree.err &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4t/trace -o run -- python3 scripts/dense_pmc_run.py 3 na_free > /dev/null 2> gpurun_out/r4t/trace.err &&
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES"; do
  i=$((i+1)); OUT=gpurun_out/r4t/pmc$i; mkdir -p $OUT
  timeout -s KILL 60 rocprofv3 --pmc $set --output-format csv -d $OUT -o run -- python3 scripts/dense_pmc_run.py 2 na_free > /dev/null 2> $OUT/err || { echo "pmc $i failed"; tail -5 $OUT/err; exit 1; }
  python3 scripts/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; head -6 $OUT/summary.txt
done
for sd in 0 1; do
  H2OMX_DL_SIDE=$sd timeout -k 10 300 python3 bench.py --model dl-mlp --estimator-defaults --steps 400 --warmup 40 > gpurun_out/r4t/dlest_side$sd.json 2> gpurun_out/r4t/dlest_side$sd.err || exit 1
done
