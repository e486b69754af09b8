#!/bin/bash
# r6h: leaf-sum replicas (LEAF_REPS) + DRF eligible codes on packed wave levels:
# tree / seg-engine / P2P / multi-rank / monotone tests, A/B of LEAF_REPS 16 vs 1 (3 reps, interleaved),
# DRF depth 20 timing + per-level table
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6h
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_tree_gpu.py tests/test_p2p_gpu.py tests/test_multirank_gpu.py tests/test_tree_dp_gpu.py tests/test_hist_adaptive.py tests/test_monotone.py tests/test_estimators_gpu.py -m gpu > $O/pytest.log 2>&1 || exit 1
AB="python3 scripts/r6/bench_ab.py h2omx.models.tree.engine:HipTreeBuilder.LEAF_REPS"
S="--rows 1375000 --steps 50 --warmup 5 --fit-trees 0"
for r in 1 2 3; do
  for v in 16 1; do
    timeout -k 10 300 $AB=$v -- --fit-trees 0 > $O/n1_reps${v}_$r.json 2>> $O/err.log || exit 1
    timeout -k 10 300 $AB=$v -- $S > $O/shard_reps${v}_$r.json 2>> $O/err.log || exit 1
    timeout -k 10 300 $AB=$v -- $S --loopback-ranks 8 > $O/loop8_reps${v}_$r.json 2>> $O/err.log || exit 1
  done
done
timeout -k 10 300 python3 scripts/drf_deep_ab.py 10000000 r6h > $O/drf.jsonl 2> $O/drf.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drf -o drf -- python3 $GRAFT_REPO_ROOT/scripts/drf_deep_ab.py 10000000 r6hp > $O/drf_prof.jsonl 2> $O/drf_prof.err || exit 1
cd $GRAFT_REPO_ROOT
python3 scripts/level_breakdown.py $O/drf/drf_kernel_trace.csv 20 > $O/drf_levels.txt 2>&1 || true
