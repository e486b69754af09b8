# round 4: precision-pin GPU part (portable data, 11M x 28, 50 trees), host data checksums,
# DL fp32 library-GEMM A/B + estimator-default timeline, XGBoost Airlines-shape timeline
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4h gpurun_out/prec11m
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/precision_parity.py --part gpu --out gpurun_out/prec11m --rows 11000000 --trees 50 > gpurun_out/r4h/prec_gpu.log 2>&1 &&
timeout -k 10 300 python3 scripts/data_checksum.py > gpurun_out/r4h/checksum_box.json 2> gpurun_out/r4h/checksum.err &&
timeout -k 10 300 python3 -u -m pytest tests/test_dense_gpu.py tests/test_dl_bf16.py tests/test_dl_model_averaging.py tests/test_estimators_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r4h/pytest.log 2>&1 &&
for lib in 1 0; do
  H2OMX_GEMM_LIB=$lib timeout -k 10 300 python3 bench.py --model dl-mlp --steps 50 --warmup 10 > gpurun_out/r4h/dl_lib$lib.json 2> gpurun_out/r4h/dl_lib$lib.err || exit 1
done &&
mkdir -p gpurun_out/prof_r4h_dlest &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4h_dlest -o run -- \
  python3 bench.py --model dl-mlp --estimator-defaults --steps 100 --warmup 20 > gpurun_out/prof_r4h_dlest/bench.json 2> gpurun_out/prof_r4h_dlest/bench.err &&
python3 scripts/prof_summary.py gpurun_out/prof_r4h_dlest adadelta > gpurun_out/prof_r4h_dlest/summary.txt &&
rm -f gpurun_out/prof_r4h_dlest/*/run_kernel_trace.csv gpurun_out/prof_r4h_dlest/run_kernel_trace.csv &&
bash scripts/gpu_prof.sh r4h_xgb --model xgboost-airlines --instrument-steps 0 --fit-trees 0
