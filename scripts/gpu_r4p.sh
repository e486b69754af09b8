# round 4: code rows moved once at the first direct level (H2OMX_MOVE_ROWS=once) - tests, DRF A/B + level table
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4p
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_tree_gpu.py -x -q -m gpu -k "direct or segmented" --timeout 300 --timeout-method thread > gpurun_out/r4p/pytest.log 2>&1 &&
for mv in 0 once; do
  H2OMX_MOVE_ROWS=$mv timeout -k 10 300 python3 scripts/deep_tree_prof.py 10000000 drf > gpurun_out/r4p/drf_move_$mv.txt 2>&1 || exit 1
done &&
mkdir -p gpurun_out/r4p/prof && H2OMX_MOVE_ROWS=once timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4p/prof -o run -- \
  python3 scripts/deep_tree_prof.py 10000000 drf > gpurun_out/r4p/prof.txt 2>&1 &&
python3 scripts/level_breakdown.py gpurun_out/r4p/prof/run_kernel_trace.csv 20 > gpurun_out/r4p/levels_once.txt && rm -f gpurun_out/r4p/prof/run_kernel_trace.csv
tail -12 gpurun_out/r4p/levels_once.txt; grep DRF gpurun_out/r4p/drf_move_*.txt
