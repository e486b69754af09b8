#!/bin/bash
# r6k: column-major planes on the row-chunk direct levels only (COLMAJOR_EVERY 3 / 6 / 0),
# 4x4-block transpose; bit-identity tests; DRF depth 20 A/B (3 reps interleaved); level table
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6k
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_gpu.py tests/test_hist_adaptive.py tests/test_tree_dp_gpu.py -m gpu > $O/pytest.log 2>&1 || exit 1
AB="python3 scripts/r6/bench_ab.py h2omx.models.tree.engine:HipTreeBuilder.COLMAJOR_EVERY"
for r in 1 2 3; do
  for v in 3 0 6; do
    timeout -k 10 300 $AB=$v -- scripts/drf_deep_ab.py 10000000 cm$v > $O/drf_cm${v}_$r.jsonl 2>> $O/err.log || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drf3 -o drf -- python3 $GRAFT_REPO_ROOT/scripts/r6/bench_ab.py h2omx.models.tree.engine:HipTreeBuilder.COLMAJOR_EVERY=3 -- scripts/drf_deep_ab.py 10000000 cm3p > $O/drf3_prof.jsonl 2> $O/drf3_prof.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drf6 -o drf -- python3 $GRAFT_REPO_ROOT/scripts/r6/bench_ab.py h2omx.models.tree.engine:HipTreeBuilder.COLMAJOR_EVERY=6 -- scripts/drf_deep_ab.py 10000000 cm6p > $O/drf6_prof.jsonl 2> $O/drf6_prof.err || exit 1
cd $GRAFT_REPO_ROOT
python3 scripts/level_breakdown.py $O/drf3/drf_kernel_trace.csv 20 > $O/drf3_levels.txt 2>&1 || true
python3 scripts/level_breakdown.py $O/drf6/drf_kernel_trace.csv 20 > $O/drf6_levels.txt 2>&1 || true
# level-0 LDS bank-conflict price: conflict-free timing-only variant vs product (kernel traces, 2 each)
cd /tmp
for r in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gbm_base$r -o gbm -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --instrument-steps 0 --no-auc --fit-trees 0 > $O/gbm_base$r.json 2> $O/gbm_base$r.err || exit 1
  H2OMX_LIB_DIR=$GRAFT_REPO_ROOT/h2omx/lib/variants/l0lanebin timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gbm_lanebin$r -o gbm -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --instrument-steps 0 --no-auc --fit-trees 0 > $O/gbm_lanebin$r.json 2> $O/gbm_lanebin$r.err || exit 1
done
