#!/bin/bash
# round 3, step 3: RM kernel pipelining - bit-identity, bench A/B, per-kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3s3
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_tree_gpu.py -k "row_major or graph_replay" > $O/pytest_tree.log 2>&1 || exit $?
H2OMX_HIST_RM=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_rm.json 2> $O/bench_rm.err || exit $?
H2OMX_HIST_RM=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_norm.json 2> $O/bench_norm.err || exit $?
H2OMX_HIST_RM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_rm -o run -- python bench.py --steps 10 --warmup 3 --fit-trees 0 --instrument-steps 0 > $O/prof_rm.log 2>&1 || exit $?
H2OMX_HIST_RM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_norm -o run -- python bench.py --steps 10 --warmup 3 --fit-trees 0 --instrument-steps 0 > $O/prof_norm.log 2>&1 || exit $?
echo done
