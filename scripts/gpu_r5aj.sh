#!/bin/bash
# kernel timelines of the GBM headline and the XGBoost Airlines-shape bench (current tree)
set -o pipefail
O=gpurun_out/r5aj
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/gbm -o gbm -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/$O/gbm.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/xgb -o xgb -- python3 $GRAFT_REPO_ROOT/bench.py --model xgboost-airlines --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/$O/xgb.log 2>&1
