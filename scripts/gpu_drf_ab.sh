#!/bin/bash
# DRF depth 20 on 10M x 100: GPU tree tests, then wall time with env A vs env B
# (scripts/deep_tree_prof.py).  Usage: gpu_drf_ab.sh TAG "ENV_A" "ENV_B"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; A=$2; B=$3
timeout -k 10 600 python -u -m pytest tests/test_tree_gpu.py tests/test_estimators_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_$TAG.log | head -20; exit $rc; }
for V in A B; do
  E=${!V}
  env $E timeout -k 10 300 python3 scripts/deep_tree_prof.py 10000000 drf > gpurun_out/drf_${TAG}_$V.txt 2>&1 || { tail -5 gpurun_out/drf_${TAG}_$V.txt; exit 1; }
  echo "$V [$E]"; grep "DRF" gpurun_out/drf_${TAG}_$V.txt
done
