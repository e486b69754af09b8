# DRF depth 20 10M x 100: direct levels with segment-order code rows (timing experiment) vs default
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4j
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/deep_tree_prof.py 10000000 drf > gpurun_out/r4j/drf_default.txt 2>&1 &&
H2OMX_DBG_SEQ_ROWS=1 timeout -k 10 300 python3 scripts/deep_tree_prof.py 10000000 drf > gpurun_out/r4j/drf_seq.txt 2>&1 &&
mkdir -p gpurun_out/r4j/prof && H2OMX_DBG_SEQ_ROWS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4j/prof -o run -- \
  python3 scripts/deep_tree_prof.py 10000000 drf > gpurun_out/r4j/prof.txt 2>&1 &&
python3 scripts/level_breakdown.py gpurun_out/r4j/prof/run_kernel_trace.csv 20 > gpurun_out/r4j/levels_seq.txt; rm -f gpurun_out/r4j/prof/run_kernel_trace.csv; cat gpurun_out/r4j/*.txt | tail -40
