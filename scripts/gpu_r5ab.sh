#!/bin/bash
# DRF depth 20: one-wave-per-node LDS budget 8 / 10 / 16 KB (10+ keeps the 10 eligible 63-bin features in one batch with ECODES)
set -o pipefail
O=gpurun_out/r5ab
mkdir -p $O
for kb in 8 10 16; do
  H2OMX_DIRECT_WAVE_KB=$kb timeout -k 10 300 python scripts/drf_deep_ab.py 10000000 kb$kb >> $O/drf.jsonl 2> $O/drf_kb$kb.err || exit 1
done
H2OMX_DIRECT_WAVE_KB=10 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_tree_gpu.py tests/test_tree_dp_gpu.py tests/test_hist_adaptive.py > $O/pytest_kb10.log 2>&1 || exit 1
