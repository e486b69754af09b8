#!/bin/bash
# A/B: selected GPU tests + bench under two env settings.  Usage: gpu_ab.sh TAG "ENV_A" "ENV_B" [pytest -k expr]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; A=$2; B=$3; K=${4:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_$TAG.log | head -20; exit $rc; }
fi
for V in A B; do
  E=${!V}
  env $E timeout -k 10 300 python bench.py --steps 30 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench_${TAG}_$V.json 2> gpurun_out/bench_${TAG}_$V.err || { tail -20 gpurun_out/bench_${TAG}_$V.err; exit 1; }
  echo "$V [$E]: $(python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_${TAG}_$V.json')); print(round(d['ms_per_step'],4), 'ms/step auc', d.get('train_auc'))")"
done
