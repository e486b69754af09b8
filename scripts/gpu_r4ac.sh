# round 4 closing run: full GPU suite, the four headline benches, AutoML 10M x 100
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4ac
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4ac/pytest_full.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/r4ac/bench_gbm.json 2> gpurun_out/r4ac/bench_gbm.err &&
timeout -k 10 300 python3 bench.py --model xgboost-airlines --steps 20 --warmup 3 > gpurun_out/r4ac/bench_xgb.json 2> gpurun_out/r4ac/bench_xgb.err &&
timeout -k 10 300 python3 bench.py --model dl-mlp --steps 100 --warmup 10 > gpurun_out/r4ac/bench_dl.json 2> gpurun_out/r4ac/bench_dl.err &&
timeout -k 10 300 python3 bench.py --model dl-mlp --estimator-defaults --steps 400 --warmup 40 > gpurun_out/r4ac/bench_dlest.json 2> gpurun_out/r4ac/bench_dlest.err &&
timeout -k 10 600 python3 scripts/automl_bench.py --rows 10000000 --cols 100 > gpurun_out/r4ac/automl.json 2> gpurun_out/r4ac/automl.err
tail -3 gpurun_out/r4ac/pytest_full.log
