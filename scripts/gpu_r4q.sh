# round 4: grouped DL graph replays - tests, estimator-default bench A/B, step timeline
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4q
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_estimators_gpu.py tests/test_dl_bf16.py tests/test_dl_model_averaging.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4q/pytest.log 2>&1 &&
for g in 4 1 8; do
  H2OMX_DL_GRAPH_STEPS=$g timeout -k 10 300 python3 bench.py --model dl-mlp --estimator-defaults --steps 400 --warmup 40 > gpurun_out/r4q/dlest_g$g.json 2> gpurun_out/r4q/dlest_g$g.err || exit 1
done &&
mkdir -p gpurun_out/prof_r4q_dlest &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4q_dlest -o run -- \
  python3 bench.py --model dl-mlp --estimator-defaults --steps 100 --warmup 20 > gpurun_out/prof_r4q_dlest/bench.json 2> gpurun_out/prof_r4q_dlest/bench.err &&
python3 scripts/prof_summary.py gpurun_out/prof_r4q_dlest adadelta > gpurun_out/prof_r4q_dlest/summary.txt &&
rm -f gpurun_out/prof_r4q_dlest/run_kernel_trace.csv; sed -n '/one step/,$p' gpurun_out/prof_r4q_dlest/summary.txt | head -50
