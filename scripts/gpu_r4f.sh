# round 4: data-parallel direct levels test, XGBoost Airlines-shape and DL benches
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4f
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_tree_dp_gpu.py tests/test_tree_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4f/pytest.log 2>&1 &&
timeout -k 10 300 python3 bench.py --model xgboost-airlines --steps 20 --warmup 3 > gpurun_out/r4f/xgb.json 2> gpurun_out/r4f/xgb.err &&
timeout -k 10 300 python3 bench.py --model dl-mlp --steps 50 --warmup 10 > gpurun_out/r4f/dl.json 2> gpurun_out/r4f/dl.err &&
timeout -k 10 300 python3 bench.py --model dl-mlp --estimator-defaults --steps 200 --warmup 20 > gpurun_out/r4f/dl_est.json 2> gpurun_out/r4f/dl_est.err
