# round 4: level_close fixes (segmented engine) - tests, DRF 10M x 100 timing + level table, AutoML, headline x3
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4n
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_tree_gpu.py tests/test_tree_dp_gpu.py tests/test_estimators_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4n/pytest.log 2>&1 &&
timeout -k 10 300 python3 scripts/deep_tree_prof.py 10000000 drf > gpurun_out/r4n/drf.txt 2>&1 &&
mkdir -p gpurun_out/r4n/prof && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4n/prof -o run -- \
  python3 scripts/deep_tree_prof.py 10000000 drf > gpurun_out/r4n/prof.txt 2>&1 &&
python3 scripts/level_breakdown.py gpurun_out/r4n/prof/run_kernel_trace.csv 20 > gpurun_out/r4n/levels.txt && rm -f gpurun_out/r4n/prof/run_kernel_trace.csv &&
timeout -k 10 600 python3 scripts/automl_bench.py --rows 10000000 --cols 100 > gpurun_out/r4n/automl.json 2> gpurun_out/r4n/automl.err &&
SWEEP_TAG=r4n_11m BENCH_ARGS="" bash scripts/sweep_env2.sh a b c &&
SWEEP_TAG=r4n_1375k BENCH_ARGS="--rows 1375000" bash scripts/sweep_env2.sh a b
