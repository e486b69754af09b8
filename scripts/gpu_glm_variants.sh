#!/bin/bash
# GLM IRLS kernel variants (h2omx/lib/variants/<name>, H2OMX_LIB_DIR) on 10M x 100:
# GLM GPU tests per variant, then plain + lambda-search fit wall times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for V in "$@"; do
  if [ "$V" = default ]; then unset H2OMX_LIB_DIR; else export H2OMX_LIB_DIR=h2omx/lib/variants/$V; fi
  timeout -k 10 300 python -u -m pytest tests -m gpu -k "glm or GLM" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_glmv_$V.log 2>&1 || { echo "$V tests FAILED"; tail -5 gpurun_out/pytest_glmv_$V.log; exit 1; }
  timeout -k 10 300 python3 scripts/deep_tree_prof.py 10000000 glm > gpurun_out/glmv_$V.txt 2>&1 || { tail -5 gpurun_out/glmv_$V.txt; exit 1; }
  echo "== $V: $(tail -1 gpurun_out/pytest_glmv_$V.log)"; grep GLM gpurun_out/glmv_$V.txt
done
