# round 4: cooperative row moves (H2OMX_MOVE_ROWS) - direct-level tests, DRF A/B + level table;
# AutoML 10M x 100 end to end; 1.375M-row histogram knob sweep
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4l
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_tree_gpu.py -x -q -m gpu -k "direct or segmented or graph" --timeout 300 --timeout-method thread > gpurun_out/r4l/pytest.log 2>&1 &&
for mv in 0 direct seg; do
  H2OMX_MOVE_ROWS=$mv timeout -k 10 300 python3 scripts/deep_tree_prof.py 10000000 drf > gpurun_out/r4l/drf_move_$mv.txt 2>&1 || exit 1
done &&
mkdir -p gpurun_out/r4l/prof && H2OMX_MOVE_ROWS=direct timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4l/prof -o run -- \
  python3 scripts/deep_tree_prof.py 10000000 drf > gpurun_out/r4l/prof.txt 2>&1 &&
python3 scripts/level_breakdown.py gpurun_out/r4l/prof/run_kernel_trace.csv 20 > gpurun_out/r4l/levels_move_direct.txt && rm -f gpurun_out/r4l/prof/run_kernel_trace.csv &&
timeout -k 10 600 python3 scripts/automl_bench.py --rows 10000000 --cols 100 > gpurun_out/r4l/automl.json 2> gpurun_out/r4l/automl.err &&
SWEEP_TAG=r4l_1375k BENCH_ARGS="--rows 1375000" bash scripts/sweep_env2.sh base small0:H2OMX_HIST_SMALL=0 mg2:H2OMX_HIST_MIN_GROUPS=2 wgs256:H2OMX_HIST_WGS=256 wgs1024:H2OMX_HIST_WGS=1024 lds96:H2OMX_HIST_LDS_KB=96 l0c4:H2OMX_HIST_L0_COPIES=4
cat gpurun_out/r4l/drf_move_*.txt | grep DRF
