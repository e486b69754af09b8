# round 4: full GPU test suite, DL estimator-default bench, XGBoost row-major compaction A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4r
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4r/pytest_full.log 2>&1 &&
timeout -k 10 300 python3 bench.py --model dl-mlp --estimator-defaults --steps 400 --warmup 40 > gpurun_out/r4r/dlest.json 2> gpurun_out/r4r/dlest.err &&
for rm in 0 1; do
  H2OMX_HIST_RM=$rm timeout -k 10 200 python3 bench.py --model xgboost-airlines --steps 20 --warmup 3 > gpurun_out/r4r/xgb_rm$rm.json 2> gpurun_out/r4r/xgb_rm$rm.err || exit 1
done
tail -3 gpurun_out/r4r/pytest_full.log
