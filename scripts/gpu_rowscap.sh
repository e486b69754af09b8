#!/bin/bash
# Rows-per-workgroup cap sweep (GBM HIGGS 11M depth 5): speed and AUC.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m h2omx.build > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
for RC in ${RCS:-32768 65536 131072 262144}; do
  H2OMX_ROWS_CAP=$RC timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/rc.json 2> gpurun_out/rc.err || { tail -5 gpurun_out/rc.err; exit 1; }
  echo "RC=$RC $(python3 -c "import json; d=json.load(open('gpurun_out/rc.json')); print(d['ms_per_step'], d['train_auc'])")"
done
