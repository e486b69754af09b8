# round 4: GLM split kernel prefetch depth A/B (1 vs 2 chunks ahead) + tests, DL side-stream test
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4v
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_dense_gpu.py tests/test_estimators_gpu.py -x -q -k "glm or side_stream" --timeout 120 --timeout-method thread > gpurun_out/r4v/pytest.log 2>&1 &&
for pd in 1 2; do
  H2OMX_GLM_PD=$pd timeout -k 10 120 python3 scripts/dense_pmc_run.py 5 na_free glm > gpurun_out/r4v/glm_pd$pd.json 2> gpurun_out/r4v/glm_pd$pd.err || exit 1
done &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4v/trace -o run -- python3 scripts/dense_pmc_run.py 3 na_free glm > /dev/null 2> gpurun_out/r4v/trace.err &&
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/r4v/pmc -o run -- python3 scripts/dense_pmc_run.py 2 na_free glm > /dev/null 2> gpurun_out/r4v/pmc.err &&
python3 scripts/pmc_summary.py gpurun_out/r4v/pmc > gpurun_out/r4v/pmc_summary.txt 2>&1
