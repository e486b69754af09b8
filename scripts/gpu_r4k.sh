# round 4: int16 node ids (H2OMX_NID16), final partition re-deriving (g, h) (H2OMX_REGRAD),
# code rows moved with their segments in deep trees (H2OMX_MOVE_ROWS): tests, A/B, DRF level table
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4k
export TMPDIR=/tmp
H2OMX_REGRAD=1 timeout -k 10 900 python3 -u -m pytest tests/test_tree_gpu.py tests/test_p2p_gpu.py tests/test_bench_contract.py tests/test_tree_dp_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4k/pytest.log 2>&1 &&
SWEEP_TAG=r4k_11m BENCH_ARGS="" bash scripts/sweep_env2.sh base nid0:H2OMX_NID16=0 rg1:H2OMX_REGRAD=1 both:H2OMX_REGRAD=1 &&
SWEEP_TAG=r4k_1375k BENCH_ARGS="--rows 1375000" bash scripts/sweep_env2.sh base nid0:H2OMX_NID16=0 rg1:H2OMX_REGRAD=1 &&
for mv in 0 direct seg; do
  H2OMX_MOVE_ROWS=$mv timeout -k 10 300 python3 scripts/deep_tree_prof.py 10000000 drf > gpurun_out/r4k/drf_move_$mv.txt 2>&1 || exit 1
done &&
mkdir -p gpurun_out/r4k/prof && H2OMX_MOVE_ROWS=direct timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4k/prof -o run -- \
  python3 scripts/deep_tree_prof.py 10000000 drf > gpurun_out/r4k/prof.txt 2>&1 &&
python3 scripts/level_breakdown.py gpurun_out/r4k/prof/run_kernel_trace.csv 20 > gpurun_out/r4k/levels_move_direct.txt; rm -f gpurun_out/r4k/prof/run_kernel_trace.csv; tail -25 gpurun_out/r4k/levels_move_direct.txt; cat gpurun_out/r4k/drf_move_*.txt | grep DRF
