# round 4: GLM / K-Means final: tests, end-to-end pass timing, kernel trace, counters
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4y
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_dense_gpu.py tests/test_estimators_gpu.py tests/test_glm_families.py tests/test_glm_solvers.py -x -q -k "glm or GLM or kmeans or KMeans" --timeout 120 --timeout-method thread > gpurun_out/r4y/pytest.log 2>&1 &&
timeout -k 10 120 python3 scripts/dense_pmc_run.py 5 na_free > gpurun_out/r4y/dense.json 2> gpurun_out/r4y/dense.err &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4y/trace -o run -- python3 scripts/dense_pmc_run.py 3 na_free > /dev/null 2> gpurun_out/r4y/trace.err &&
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/r4y/pmc -o run -- python3 scripts/dense_pmc_run.py 2 na_free > /dev/null 2> gpurun_out/r4y/pmc.err &&
python3 scripts/pmc_summary.py gpurun_out/r4y/pmc > gpurun_out/r4y/pmc_summary.txt 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --output-format csv -d gpurun_out/r4y/pmc2 -o run -- python3 scripts/dense_pmc_run.py 2 na_free > /dev/null 2> gpurun_out/r4y/pmc2.err &&
python3 scripts/pmc_summary.py gpurun_out/r4y/pmc2 > gpurun_out/r4y/pmc2_summary.txt 2>&1
