# round 4: level 0 reading the packed rows boost_update quantised (H2OMX_PK_IN_BOOST) - tests, A/B, timeline
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4i
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_tree_gpu.py tests/test_p2p_gpu.py tests/test_bench_contract.py tests/test_monotone.py tests/test_categorical_splits.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r4i/pytest.log 2>&1 &&
for pk in 1 0; do
  H2OMX_PK_IN_BOOST=$pk timeout -k 10 200 python3 bench.py --steps 40 --warmup 4 > gpurun_out/r4i/b11m_pk$pk.json 2> gpurun_out/r4i/b11m_pk$pk.err || exit 1
  H2OMX_PK_IN_BOOST=$pk timeout -k 10 200 python3 bench.py --steps 40 --warmup 4 --rows 1375000 > gpurun_out/r4i/b1375k_pk$pk.json 2> gpurun_out/r4i/b1375k_pk$pk.err || exit 1
  H2OMX_PK_IN_BOOST=$pk timeout -k 10 200 python3 bench.py --model xgboost-airlines --steps 20 --warmup 3 > gpurun_out/r4i/xgb_pk$pk.json 2> gpurun_out/r4i/xgb_pk$pk.err || exit 1
done &&
bash scripts/gpu_prof.sh r4i_11m --instrument-steps 0 --fit-trees 0
[ $? -eq 0 ] && for sm in 1 0; do
  H2OMX_GEMM_LIB_SMALL=$sm timeout -k 10 300 python3 bench.py --model dl-mlp --estimator-defaults --steps 200 --warmup 20 > gpurun_out/r4i/dlest_small$sm.json 2> gpurun_out/r4i/dlest_small$sm.err || exit 1
done
