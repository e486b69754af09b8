# round 4: GLM split kernel wave-unit count A/B (H2OMX_GLM_UNITS)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4al
export TMPDIR=/tmp
for u in 2048 1024 1536 4096 2048; do
  H2OMX_GLM_UNITS=$u timeout -k 10 120 python3 scripts/dense_pmc_run.py 10 na_free glm > gpurun_out/r4al/glm_u$u.json 2> gpurun_out/r4al/glm_u$u.err || exit 1
  echo "units=$u $(cat gpurun_out/r4al/glm_u$u.json)" >> gpurun_out/r4al/sweep.txt
done
