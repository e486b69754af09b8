# round-4 GPU check: new paths (P2P all-reduce, one-graph 2-rank GBM, Newton monotone
# bounds, GLM solvers, categorical group splits), the tree kernel suite, then the bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4a
T="python -u -m pytest -x -v --timeout 280 --timeout-method thread"
timeout -k 10 600 $T tests/test_p2p_gpu.py tests/test_bench_contract.py -m gpu > gpurun_out/r4a/p2p.log 2>&1 &&
timeout -k 10 600 $T tests/test_categorical_splits.py tests/test_monotone.py tests/test_glm_solvers.py tests/test_tree_gpu.py -m gpu > gpurun_out/r4a/trees.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r4a/bench_gbm.json 2> gpurun_out/r4a/bench_gbm.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --rows 1375000 --fit-trees 0 > gpurun_out/r4a/bench_gbm_1375k.json 2> gpurun_out/r4a/bench_gbm_1375k.err
