# round 4: GLM split kernel, LDS-DMA staging A/B (H2OMX_GLM_GLDS=0/1) + tests
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4x
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_dense_gpu.py -x -q -k "glm" --timeout 120 --timeout-method thread > gpurun_out/r4x/pytest.log 2>&1 &&
for g in 0 1; do
  H2OMX_GLM_GLDS=$g timeout -k 10 120 python3 scripts/dense_pmc_run.py 5 na_free glm > gpurun_out/r4x/glm_glds$g.json 2> gpurun_out/r4x/glm_glds$g.err || exit 1
done &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4x/trace -o run -- python3 scripts/dense_pmc_run.py 3 na_free glm > /dev/null 2> gpurun_out/r4x/trace.err
