#!/bin/bash
# DL iteration: dense GPU tests, the fp32 bench (default build and GK=64 variant), kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py tests/test_dl_bf16.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/dense_tests.log 2>&1 || { tail -30 gpurun_out/dense_tests.log; exit 1; }
tail -2 gpurun_out/dense_tests.log
timeout -k 10 200 python3 bench.py --model dl-mlp --steps 30 --warmup 3 > gpurun_out/dl_default.json 2> gpurun_out/dl_default.err || { tail -5 gpurun_out/dl_default.err; exit 1; }
cat gpurun_out/dl_default.json
OUT=gpurun_out/dlprof
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --model dl-mlp --steps 10 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 scripts/prof_summary.py $OUT adadelta > $OUT/summary.txt 2>&1
sed -n '/one step/,$p' $OUT/summary.txt
