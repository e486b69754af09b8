# round 4: DL estimator-default step (gradient folds in ADADELTA): tests, bench, timeline (hipBLASLt small GEMMs,
# 8-step graph replays, the group's mini-batches gathered once)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4ae
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_estimators_gpu.py tests/test_dl_bf16.py -x -q -k "deeplearning or dl or DL" --timeout 120 --timeout-method thread > gpurun_out/r4ae/pytest.log 2>&1 &&
timeout -k 10 300 python3 bench.py --model dl-mlp --estimator-defaults --steps 400 --warmup 40 > gpurun_out/r4ae/dlest.json 2> gpurun_out/r4ae/dlest.err &&
OUT=gpurun_out/r4ae/dlprof &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --model dl-mlp --estimator-defaults --steps 200 --warmup 20 > /dev/null 2> gpurun_out/r4ae/dlprof.err &&
python3 scripts/prof_summary.py $OUT adadelta > gpurun_out/r4ae/dl_summary.txt 2>&1
