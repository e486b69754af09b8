#!/bin/bash
# First GPU validation: build, GPU numerics tests, smoke, short bench + profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m h2omx.build > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; cat gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke 2>&1 | tail -5 || exit 1
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_r1a.json 2> gpurun_out/bench_r1a.err
rc=$?
cat gpurun_out/bench_r1a.json; tail -5 gpurun_out/bench_r1a.err
exit $rc
