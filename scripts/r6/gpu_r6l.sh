#!/bin/bash
# r6l: DRF deep levels - lane-best split scans (one wave arg-max per node, packed single
# prefix sum), early pinned node-count readback, column-major planes (COLMAJOR_EVERY 6 / 0 / 3):
# GPU tree tests, DRF depth 20 A/B (3 reps interleaved), level table, AutoML 10M x 100
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6l
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_gpu.py tests/test_hist_adaptive.py tests/test_tree_dp_gpu.py tests/test_estimators_gpu.py -m gpu > $O/pytest.log 2>&1 || exit 1
AB="python3 scripts/r6/bench_ab.py h2omx.models.tree.engine:HipTreeBuilder.COLMAJOR_EVERY"
for r in 1 2 3; do
  for v in 6 0 3; do
    timeout -k 10 300 $AB=$v -- scripts/drf_deep_ab.py 10000000 cm$v > $O/drf_cm${v}_$r.jsonl 2>> $O/err.log || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drf6 -o drf -- python3 $GRAFT_REPO_ROOT/scripts/drf_deep_ab.py 10000000 cm6p > $O/drf6_prof.jsonl 2> $O/drf6_prof.err || exit 1
cd $GRAFT_REPO_ROOT
python3 scripts/level_breakdown.py $O/drf6/drf_kernel_trace.csv 20 > $O/drf6_levels.txt 2>&1 || true
timeout -k 10 600 python3 scripts/automl_bench.py --rows 10000000 > $O/automl.json 2> $O/automl.err || exit 1
