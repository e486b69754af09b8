#!/bin/bash
# Round-2 checkpoint: full GPU test suite, smoke, the three benches, AutoML 10M x 100 on one GPU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2b}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu_$TAG.log | head; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
for M in gbm-higgs xgboost-airlines dl-mlp; do
  timeout -k 10 600 python bench.py --model $M --steps 30 --warmup 3 > gpurun_out/bench_${TAG}_$M.json 2> gpurun_out/bench_${TAG}_$M.err || { tail -20 gpurun_out/bench_${TAG}_$M.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$M.json')); print('$M', round(d['ms_per_step'],4), 'ms/step', d['value'], d.get('fit_rows_per_s'))"
done
timeout -k 10 600 python3 scripts/automl_bench.py --rows 10000000 --cols 100 > gpurun_out/automl_$TAG.json 2> gpurun_out/automl_$TAG.err || { tail -20 gpurun_out/automl_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/automl_$TAG.json')); print('automl wall', d['automl_wall_s'], d['model_run_ms'])"
