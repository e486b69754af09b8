# round 4: host data checksums (precision pin), DL fp32 with hipBLASLt forward GEMMs A/B,
# estimator-default DL step timeline
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4g
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/data_checksum.py > gpurun_out/r4g/checksum_box.json 2> gpurun_out/r4g/checksum.err &&
timeout -k 10 300 python3 -u -m pytest tests/test_dense_gpu.py tests/test_dl_bf16.py tests/test_dl_model_averaging.py tests/test_estimators_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r4g/pytest.log 2>&1 ;
for lib in 1 0; do
  H2OMX_GEMM_LIB=$lib timeout -k 10 300 python3 bench.py --model dl-mlp --steps 50 --warmup 10 > gpurun_out/r4g/dl_lib$lib.json 2> gpurun_out/r4g/dl_lib$lib.err || exit 1
done &&
mkdir -p gpurun_out/prof_r4g_dlest &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4g_dlest -o run -- \
  python3 bench.py --model dl-mlp --estimator-defaults --steps 200 --warmup 20 > gpurun_out/prof_r4g_dlest/bench.json 2> gpurun_out/prof_r4g_dlest/bench.err &&
python3 scripts/prof_summary.py gpurun_out/prof_r4g_dlest adadelta > gpurun_out/prof_r4g_dlest/summary.txt
