#!/bin/bash
# ECODES decoupled from histogram batching: deep-tree tests (the direct-level equivalence test twice), DRF depth 20
set -o pipefail
O=gpurun_out/r5ac
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_tree_gpu.py tests/test_tree_dp_gpu.py tests/test_hist_adaptive.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_tree_gpu.py -k direct_deep_levels > $O/pytest_direct_rerun.log 2>&1 || exit 1
timeout -k 10 300 python scripts/drf_deep_ab.py 10000000 ecodes_decoupled > $O/drf.jsonl 2> $O/drf.err || exit 1
