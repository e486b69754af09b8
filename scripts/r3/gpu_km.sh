#!/bin/bash
# K-Means wave kernel: tests, 10M x 100 timing, kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/km
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py tests/test_estimators_gpu.py -k "kmeans" -x -v --timeout 120 --timeout-method thread > gpurun_out/km/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/km/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/km/pytest.log | head -20; exit $rc; }
timeout -k 10 120 python scripts/r3/km_bench.py > gpurun_out/km/bench.json 2> gpurun_out/km/bench.err || { tail -20 gpurun_out/km/bench.err; exit 1; }
cat gpurun_out/km/bench.json
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/km/prof -o run -- python3 scripts/r3/km_bench.py > gpurun_out/km/prof.out 2>&1 || { tail -5 gpurun_out/km/prof.out; exit 1; }
find gpurun_out/km/prof -name "*kernel_stats.csv" -exec head -8 {} \;
