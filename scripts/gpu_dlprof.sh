#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m h2omx.build > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests/test_estimators_gpu.py -x -q > gpurun_out/pt_est.log 2>&1; tail -3 gpurun_out/pt_est.log
OUT=gpurun_out/prof_dl
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --model dl-mlp --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 scripts/prof_summary.py "$OUT" | head -40
