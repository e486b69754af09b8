#!/bin/bash
# r6m: level-0 copy kernel with sliced low-cardinality features - bit-identity test,
# XGBoost Airlines-shape and GBM HIGGS-shape A/B against the HEAD kernels (3 reps interleaved)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6m
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_gpu.py -k "level0_copies or graph_replay or gbm_bernoulli" -m gpu > $O/pytest.log 2>&1 || exit 1
H=$GRAFT_REPO_ROOT/h2omx/lib/variants/head
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --model xgboost-airlines --steps 20 --warmup 3 > $O/xgb_new_$r.json 2>> $O/err.log || exit 1
  H2OMX_LIB_DIR=$H timeout -k 10 300 python3 bench.py --model xgboost-airlines --steps 20 --warmup 3 > $O/xgb_head_$r.json 2>> $O/err.log || exit 1
  timeout -k 10 300 python3 bench.py --fit-trees 0 > $O/gbm_new_$r.json 2>> $O/err.log || exit 1
  H2OMX_LIB_DIR=$H timeout -k 10 300 python3 bench.py --fit-trees 0 > $O/gbm_head_$r.json 2>> $O/err.log || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/xgb_new -o xgb -- python3 $GRAFT_REPO_ROOT/bench.py --model xgboost-airlines --steps 10 --warmup 2 --instrument-steps 0 --no-auc > /dev/null 2> $O/xgb_prof.err || exit 1
H2OMX_LIB_DIR=$H timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/xgb_head -o xgb -- python3 $GRAFT_REPO_ROOT/bench.py --model xgboost-airlines --steps 10 --warmup 2 --instrument-steps 0 --no-auc > /dev/null 2> $O/xgb_prof_head.err || exit 1
