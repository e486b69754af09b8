#!/bin/bash
# r6v: line-aligned row-major code rows with the transpose's odd LDS row pitch (BinnedMatrix.ROW_ALIGN 1 vs 0):
# seg-engine tests, DRF depth 20 A/B (3 reps interleaved), level table, AutoML
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6v
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_gpu.py tests/test_hist_adaptive.py tests/test_tree_dp_gpu.py tests/test_estimators_gpu.py -m gpu > $O/pytest.log 2>&1 || exit 1
AB="python3 scripts/r6/bench_ab.py h2omx.models.tree.binning:BinnedMatrix.ROW_ALIGN"
for r in 1 2 3; do
  timeout -k 10 300 $AB=1 -- scripts/drf_deep_ab.py 10000000 al1 > $O/drf_al1_$r.jsonl 2>> $O/err.log || exit 1
  timeout -k 10 300 $AB=0 -- scripts/drf_deep_ab.py 10000000 al0 > $O/drf_al0_$r.jsonl 2>> $O/err.log || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drf -o drf -- python3 $GRAFT_REPO_ROOT/scripts/drf_deep_ab.py 10000000 al1p > /dev/null 2> $O/drf_prof.err || exit 1
cd $GRAFT_REPO_ROOT
python3 scripts/level_breakdown.py $O/drf/drf_kernel_trace.csv 20 > $O/drf_levels.txt 2>&1 || true
timeout -k 10 600 python3 scripts/automl_bench.py --rows 10000000 > $O/automl.json 2> $O/automl.err || exit 1
