#!/bin/bash
# r6j: DRF deep levels - per-wave UniformAdaptive cut tables (vs the division form,
# variants/nocut) and column-major segment code planes (HipTreeBuilder.COLMAJOR_EVERY):
# bit-identity tests, DRF depth 20 A/B (3 reps interleaved), per-level kernel table
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6j
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_gpu.py tests/test_hist_adaptive.py -k "direct_deep_levels or uniform_adaptive or trees_match_cpu" -m gpu > $O/pytest.log 2>&1 || exit 1
AB="python3 scripts/r6/bench_ab.py h2omx.models.tree.engine:HipTreeBuilder.COLMAJOR_EVERY"
for r in 1 2 3; do
  timeout -k 10 300 $AB=0 -- scripts/drf_deep_ab.py 10000000 cut_cm0 > $O/drf_cut_cm0_$r.jsonl 2>> $O/err.log || exit 1
  H2OMX_LIB_DIR=$GRAFT_REPO_ROOT/h2omx/lib/variants/nocut timeout -k 10 300 $AB=0 -- scripts/drf_deep_ab.py 10000000 nocut_cm0 > $O/drf_nocut_cm0_$r.jsonl 2>> $O/err.log || exit 1
  timeout -k 10 300 $AB=3 -- scripts/drf_deep_ab.py 10000000 cut_cm3 > $O/drf_cut_cm3_$r.jsonl 2>> $O/err.log || exit 1
  timeout -k 10 300 $AB=2 -- scripts/drf_deep_ab.py 10000000 cut_cm2 > $O/drf_cut_cm2_$r.jsonl 2>> $O/err.log || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drf -o drf -- python3 $GRAFT_REPO_ROOT/scripts/r6/bench_ab.py h2omx.models.tree.engine:HipTreeBuilder.COLMAJOR_EVERY=0 -- scripts/drf_deep_ab.py 10000000 cutp > $O/drf_prof.jsonl 2> $O/drf_prof.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drf3 -o drf -- python3 $GRAFT_REPO_ROOT/scripts/r6/bench_ab.py h2omx.models.tree.engine:HipTreeBuilder.COLMAJOR_EVERY=3 -- scripts/drf_deep_ab.py 10000000 cut_cm3p > $O/drf3_prof.jsonl 2> $O/drf3_prof.err || exit 1
cd $GRAFT_REPO_ROOT
python3 scripts/level_breakdown.py $O/drf/drf_kernel_trace.csv 20 > $O/drf_levels.txt 2>&1 || true
python3 scripts/level_breakdown.py $O/drf3/drf_kernel_trace.csv 20 > $O/drf3_levels.txt 2>&1 || true
