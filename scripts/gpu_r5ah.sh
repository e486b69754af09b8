#!/bin/bash
# DL GPU tests on the x3 data-gradient route
set -o pipefail
O=gpurun_out/r5ah
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dl_step_gpu.py tests/test_dl_bf16.py tests/test_estimators_gpu.py tests/test_dense_gpu.py > $O/pytest.log 2>&1
