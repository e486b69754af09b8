#!/bin/bash
# after reverting the edge preloading: tree / P2P GPU tests, loopback-8 and shard, DRF depth 20
set -o pipefail
O=gpurun_out/r5bh
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tree_gpu.py tests/test_tree_dp_gpu.py tests/test_hist_adaptive.py tests/test_p2p_gpu.py tests/test_multirank_gpu.py tests/test_estimators_gpu.py > $O/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0 --loopback-ranks 8 > $O/loop8_$rep.json 2> $O/loop8_$rep.err || exit 1
done
timeout -k 10 300 python bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0 > $O/shard.json 2> $O/shard.err || exit 1
timeout -k 10 300 python scripts/drf_deep_ab.py 10000000 reverted > $O/drf.jsonl 2> $O/drf.err || exit 1
