# round 4: pipelined GLM split kernel (tests + timing vs fp32 MFMA), DL side-stream A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4u
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_dense_gpu.py -x -q -k "glm" --timeout 120 --timeout-method thread > gpurun_out/r4u/pytest_glm.log 2>&1 &&
for g in f32 split; do
  H2OMX_GLM_GRAM=$g timeout -k 10 120 python3 scripts/dense_pmc_run.py 5 na_free glm > gpurun_out/r4u/glm_$g.json 2> gpurun_out/r4u/glm_$g.err || exit 1
done &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4u/trace -o run -- python3 scripts/dense_pmc_run.py 3 na_free > /dev/null 2> gpurun_out/r4u/trace.err &&
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/r4u/pmc -o run -- python3 scripts/dense_pmc_run.py 2 na_free glm > /dev/null 2> gpurun_out/r4u/pmc.err &&
python3 scripts/pmc_summary.py gpurun_out/r4u/pmc > gpurun_out/r4u/pmc_summary.txt 2>&1 &&
for sd in 0 1; do
  H2OMX_DL_SIDE=$sd timeout -k 10 300 python3 bench.py --model dl-mlp --estimator-defaults --steps 400 --warmup 40 > gpurun_out/r4u/dlest_side$sd.json 2> gpurun_out/r4u/dlest_side$sd.err || exit 1
done
