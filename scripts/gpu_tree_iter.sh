#!/bin/bash
# tree-engine iteration: the tree GPU tests, then the DRF 10M x 100 depth-20 profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_tree_gpu.py -x -q --timeout 120 --timeout-method thread \
  ${TREE_TEST_K:+-k "$TREE_TEST_K"} > gpurun_out/tree_tests.log 2>&1 || { tail -30 gpurun_out/tree_tests.log; exit 1; }
tail -3 gpurun_out/tree_tests.log
bash scripts/gpu_drf10m.sh
