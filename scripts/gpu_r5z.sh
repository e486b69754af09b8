#!/bin/bash
# AutoML 10M x 100 with the deep-tree fine-grid cap; GPU estimator tests
set -o pipefail
O=gpurun_out/r5z
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_hist_adaptive.py tests/test_estimators_gpu.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 400 python scripts/automl_bench.py --rows 10000000 --cols 100 > $O/automl.json 2> $O/automl.err || exit 1
