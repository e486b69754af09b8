#!/bin/bash
# r6f: new fused-finalisation test + P2P tests after the loopback slot fix, loopback-8 x3,
# DRF depth 20 (10M x 100, 10 trees) per-level kernel table, XGBoost Airlines-shape kernel stats
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6f
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_tree_gpu.py -k "level_finalisation or graph_replay" > $O/pytest_tree.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_p2p_gpu.py -m gpu > $O/pytest_p2p.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0 --loopback-ranks 8 > $O/loop8_$r.json 2>> $O/err.log || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drf -o drf -- python3 $GRAFT_REPO_ROOT/scripts/drf_deep_ab.py 10000000 r6f > $O/drf.jsonl 2> $O/drf.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/xgb -o xgb -- python3 $GRAFT_REPO_ROOT/bench.py --model xgboost-airlines --steps 10 --warmup 2 --instrument-steps 0 --no-auc > $O/xgb.json 2> $O/xgb.err || exit 1
cd $GRAFT_REPO_ROOT
python3 scripts/level_breakdown.py $O/drf/drf_kernel_trace.csv 20 > $O/drf_levels.txt 2>&1 || true
