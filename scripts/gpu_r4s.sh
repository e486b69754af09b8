# round 4: GLM split-bf16 Gram and K-Means MFMA-sum tests + dense timing A/B (old kernels vs new), then the full GPU
# suite, DL estimator-default bench and the XGBoost row-major compaction A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4s
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_dense_gpu.py -x -q -k "glm or kmeans" --timeout 120 --timeout-method thread > gpurun_out/r4s/pytest_glm.log 2>&1 &&
for g in f32 split; do
  km=0; [ $g = split ] && km=1
  H2OMX_KM_MFMA=$km H2OMX_GLM_GRAM=$g timeout -k 10 200 python3 scripts/dense_pmc_run.py 5 > gpurun_out/r4s/dense_$g.json 2> gpurun_out/r4s/dense_$g.err || exit 1
done &&
timeout -k 10 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4s/pytest_full.log 2>&1 &&
timeout -k 10 300 python3 bench.py --model dl-mlp --estimator-defaults --steps 400 --warmup 40 > gpurun_out/r4s/dlest.json 2> gpurun_out/r4s/dlest.err &&
for rm in 0 1; do
  H2OMX_HIST_RM=$rm timeout -k 10 200 python3 bench.py --model xgboost-airlines --steps 20 --warmup 3 > gpurun_out/r4s/xgb_rm$rm.json 2> gpurun_out/r4s/xgb_rm$rm.err || exit 1
done
tail -3 gpurun_out/r4s/pytest_full.log
