#!/bin/bash
# r6e: level finalisation folded into the reduce launch (FUSE_FIN): tree / P2P / multi-rank tests,
# A/B on the headline, the shard and loopback-8 (3 reps each, interleaved)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6e
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_tree_gpu.py tests/test_p2p_gpu.py tests/test_multirank_gpu.py tests/test_tree_dp_gpu.py tests/test_hist_adaptive.py tests/test_monotone.py tests/test_categorical_splits.py -m gpu > $O/pytest.log 2>&1 || exit 1
AB="python3 scripts/r6/bench_ab.py h2omx.models.tree.engine:HipTreeBuilder.FUSE_FIN"
S="--rows 1375000 --steps 50 --warmup 5 --fit-trees 0"
for r in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 300 $AB=$v -- $S > $O/shard_fin${v}_$r.json 2>> $O/err.log || exit 1
    timeout -k 10 300 $AB=$v -- $S --loopback-ranks 8 > $O/loop8_fin${v}_$r.json 2>> $O/err.log || exit 1
    timeout -k 10 300 $AB=$v -- --fit-trees 0 > $O/n1_fin${v}_$r.json 2>> $O/err.log || exit 1
  done
done
