#!/bin/bash
# round 3, step 2: row-major compacted histograms - bit-identity, bench, kernel timeline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3s2
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_tree_gpu.py tests/test_multirank_gpu.py -k "row_major or graph_replay or gbm_bernoulli or two_ranks or pk32" > gpurun_out/r3s2/pytest_tree.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_contract.py -m gpu > gpurun_out/r3s2/pytest_bench.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r3s2/bench_rm.json 2> gpurun_out/r3s2/bench_rm.err || exit $?
H2OMX_HIST_RM=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r3s2/bench_norm.json 2> gpurun_out/r3s2/bench_norm.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3s2/prof -o run -- python bench.py --steps 10 --warmup 3 --fit-trees 0 --instrument-steps 0 > gpurun_out/r3s2/prof.log 2>&1 || exit $?
echo done
