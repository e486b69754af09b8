# round 4: byte labels (H2OMX_Y8), int16 leaf ids for boost_update, 16-deep reduce_split loads:
# tests, A/B, 11M timeline, XGBoost
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4m
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_tree_gpu.py tests/test_p2p_gpu.py tests/test_bench_contract.py tests/test_monotone.py tests/test_categorical_splits.py tests/test_tree_dp_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4m/pytest.log 2>&1 &&
SWEEP_TAG=r4m_11m BENCH_ARGS="" bash scripts/sweep_env2.sh base y80:H2OMX_Y8=0 base2 &&
SWEEP_TAG=r4m_1375k BENCH_ARGS="--rows 1375000" bash scripts/sweep_env2.sh base y80:H2OMX_Y8=0 &&
timeout -k 10 200 python3 bench.py --model xgboost-airlines --steps 20 --warmup 3 > gpurun_out/r4m/xgb.json 2> gpurun_out/r4m/xgb.err &&
bash scripts/gpu_prof.sh r4m_11m --instrument-steps 0 --fit-trees 0
