#!/bin/bash
# r6bk: feature-group identity test; the 255-bin DRF grid with the 64 KB vs 16 KB segmented-histogram budget
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6bk
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tree_gpu.py -k "feature_groups or bag_compact_matches" -p no:cacheprovider > $O/pytest.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 scripts/r6/drf_fine255.py 65536 > $O/drf255_64k_$r.jsonl 2>> $O/err.log || exit 1
  timeout -k 10 300 python3 scripts/r6/drf_fine255.py 16384 > $O/drf255_16k_$r.jsonl 2>> $O/err.log || exit 1
done
