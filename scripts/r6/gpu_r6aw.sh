#!/bin/bash
# r6aw: the segmented engine (segmented histograms from level 1 since r6ah) on the shallow headline configs:
# XGBoost Airlines-shape depth 6 and GBM HIGGS depth 5, scan (auto) vs seg, 3 reps interleaved
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6aw
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --model xgboost-airlines --steps 20 --warmup 3 > $O/xgb_auto_$r.json 2>> $O/err.log || exit 1
  H2OMX_TREE_ENGINE=seg timeout -k 10 300 python3 bench.py --model xgboost-airlines --steps 20 --warmup 3 > $O/xgb_seg_$r.json 2>> $O/err.log || exit 1
  timeout -k 10 300 python3 bench.py > $O/gbm_auto_$r.json 2>> $O/err.log || exit 1
  H2OMX_TREE_ENGINE=seg timeout -k 10 300 python3 bench.py > $O/gbm_seg_$r.json 2>> $O/err.log || exit 1
done
