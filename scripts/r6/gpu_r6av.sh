#!/bin/bash
# r6av: in-bag root segment across class counts (multinomial DRF / GBM)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6av
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_tree_gpu.py -k "bag_compact" > $O/pytest.log 2>&1 || exit 1
