# round 4: fold-ADADELTA with a block-uniform fold test: DL tests + estimator bench + timeline
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4ah
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_estimators_gpu.py tests/test_dl_bf16.py -x -q -k "deeplearning or dl or DL" --timeout 120 --timeout-method thread > gpurun_out/r4ah/pytest.log 2>&1 &&
timeout -k 10 300 python3 bench.py --model dl-mlp --estimator-defaults --steps 400 --warmup 40 > gpurun_out/r4ah/dlest.json 2> gpurun_out/r4ah/dlest.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4ah/dlprof -o run -- python3 bench.py --model dl-mlp --estimator-defaults --steps 200 --warmup 20 > /dev/null 2> gpurun_out/r4ah/dlprof.err &&
python3 scripts/prof_summary.py gpurun_out/r4ah/dlprof adadelta > gpurun_out/r4ah/dl_summary.txt 2>&1
