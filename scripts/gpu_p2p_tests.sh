# round-4 GPU check: P2P all-reduce, 2-rank one-graph GBM, monotone (Newton bounds), GLM solvers
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_p2p_gpu.py tests/test_bench_contract.py -m gpu > gpurun_out/p2p_tests.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_monotone.py tests/test_glm_solvers.py -m gpu > gpurun_out/mono_glm_tests.log 2>&1
