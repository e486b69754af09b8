# round 4: final partition re-derives (g, h) (H2OMX_REGRAD) + code rows moved with their
# segments in deep trees (H2OMX_MOVE_ROWS): tests, GBM A/B, DRF 10M x 100 depth-20 A/B + level table
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4k
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_tree_gpu.py tests/test_p2p_gpu.py tests/test_bench_contract.py tests/test_tree_dp_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4k/pytest.log 2>&1 &&
for rg in 1 0; do
  H2OMX_REGRAD=$rg timeout -k 10 200 python3 bench.py --steps 40 --warmup 4 > gpurun_out/r4k/b11m_rg$rg.json 2> gpurun_out/r4k/b11m_rg$rg.err || exit 1
  H2OMX_REGRAD=$rg timeout -k 10 200 python3 bench.py --steps 40 --warmup 4 --rows 1375000 > gpurun_out/r4k/b1375k_rg$rg.json 2> gpurun_out/r4k/b1375k_rg$rg.err || exit 1
done &&
for mv in 0 direct seg; do
  H2OMX_MOVE_ROWS=$mv timeout -k 10 300 python3 scripts/deep_tree_prof.py 10000000 drf > gpurun_out/r4k/drf_move_$mv.txt 2>&1 || exit 1
done &&
mkdir -p gpurun_out/r4k/prof && H2OMX_MOVE_ROWS=direct timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4k/prof -o run -- \
  python3 scripts/deep_tree_prof.py 10000000 drf > gpurun_out/r4k/prof.txt 2>&1 &&
python3 scripts/level_breakdown.py gpurun_out/r4k/prof/run_kernel_trace.csv 20 > gpurun_out/r4k/levels_move_direct.txt; rm -f gpurun_out/r4k/prof/run_kernel_trace.csv; tail -25 gpurun_out/r4k/levels_move_direct.txt; cat gpurun_out/r4k/drf_move_*.txt | grep DRF
