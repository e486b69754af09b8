#!/bin/bash
# forest kept on the device for the first predictions after a fit: tree / estimator GPU tests, DRF CV profile, AutoML
set -o pipefail
O=gpurun_out/r5bb
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_gpu.py tests/test_estimators_gpu.py tests/test_hist_adaptive.py tests/test_categorical_splits.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 400 python scripts/drf_fit_prof.py 50 3 > $O/prof.txt 2>&1 || exit 1
timeout -k 10 400 python scripts/automl_bench.py --rows 10000000 --cols 100 > $O/automl.json 2> $O/automl.err || exit 1
