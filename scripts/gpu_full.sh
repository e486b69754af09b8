#!/bin/bash
# Full validation: all GPU tests, smoke, the three BASELINE benches, DL + GBM kernel profiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-full}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu_$TAG.log | head; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
for M in gbm-higgs xgboost-airlines dl-mlp; do
  timeout -k 10 600 python bench.py --model $M --steps 30 --warmup 3 > gpurun_out/bench_${TAG}_$M.json 2> gpurun_out/bench_${TAG}_$M.err || { tail -20 gpurun_out/bench_${TAG}_$M.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$M.json')); print('$M', round(d['ms_per_step'],4), 'ms/step', d['value'])"
done
for M in gbm-higgs dl-mlp; do
  OUT=gpurun_out/prof_${TAG}_$M; mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 bench.py --model $M --steps 5 --warmup 1 --no-auc > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
  python3 scripts/prof_summary.py "$OUT" > $OUT/summary.txt
done
