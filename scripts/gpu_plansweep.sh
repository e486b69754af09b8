#!/bin/bash
# Histogram plan sweep (GBM HIGGS 11M depth 5): deep-plan switch point and LDS budgets.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m h2omx.build > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
run() {
  env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-auc > gpurun_out/ps.json 2> gpurun_out/ps.err || { tail -5 gpurun_out/ps.err; exit 1; }
  echo "$* $(python3 -c "import json; print(json.load(open('gpurun_out/ps.json'))['ms_per_step'])")"
}
run H2OMX_HIST_DEEP_MIN_GROUPS=4
run H2OMX_HIST_DEEP_MIN_GROUPS=2
run H2OMX_HIST_DEEP_MIN_GROUPS=2 H2OMX_HIST_DEEP_LDS_KB=156
run H2OMX_HIST_DEEP_MIN_GROUPS=4 H2OMX_HIST_DEEP_LDS_KB=156
run H2OMX_HIST_LDS_KB=56
run H2OMX_HIST_WGS=1024
run H2OMX_HIST_WGS=256
