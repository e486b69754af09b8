#!/bin/bash
# per-node histogram rule: fine edges loaded before the range reductions: tree GPU tests (bit-identity), DRF depth 20, GBM headline + shard
set -o pipefail
O=gpurun_out/r5bd
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tree_gpu.py tests/test_tree_dp_gpu.py tests/test_hist_adaptive.py tests/test_interaction.py tests/test_categorical_splits.py tests/test_p2p_gpu.py tests/test_multirank_gpu.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python scripts/drf_deep_ab.py 10000000 edges > $O/drf.jsonl 2> $O/drf.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/drf -o drf -- python3 $GRAFT_REPO_ROOT/scripts/drf_deep_ab.py > $GRAFT_REPO_ROOT/$O/drf_prof.log 2>&1
