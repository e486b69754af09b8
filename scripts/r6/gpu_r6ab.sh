#!/bin/bash
# r6ab: per-node split records kept in LDS between the arg-max and the finalisation (node_best_finalize) vs the
# committed kernels: tree tests, 1.375M shard / loopback-8 / 11M headline, 3 reps interleaved
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6ab
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_gpu.py tests/test_p2p_gpu.py tests/test_monotone.py tests/test_hist_adaptive.py -m gpu > $O/pytest.log 2>&1 || exit 1
H=$GRAFT_REPO_ROOT/h2omx/lib/variants/head
S="--rows 1375000 --steps 50 --warmup 5 --fit-trees 0"
for r in 1 2 3; do
  for arm in new head; do
    if [ $arm = head ]; then export H2OMX_LIB_DIR=$H; else unset H2OMX_LIB_DIR; fi
    timeout -k 10 300 python3 bench.py $S > $O/shard_${arm}_$r.json 2>> $O/err.log || exit 1
    timeout -k 10 300 python3 bench.py $S --loopback-ranks 8 > $O/loop8_${arm}_$r.json 2>> $O/err.log || exit 1
    timeout -k 10 300 python3 bench.py --fit-trees 0 > $O/n1_${arm}_$r.json 2>> $O/err.log || exit 1
  done
done
