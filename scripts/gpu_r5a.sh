#!/bin/bash
# round 5: fused N-rank level (reduce_split_p2p / leaf_finalize_p2p), P2P fault
# propagation, loopback strong-scaling proxy; N=1 headline unchanged
set -o pipefail
O=gpurun_out/r5a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_p2p_gpu.py tests/test_multirank_gpu.py tests/test_tree_dp_gpu.py > $O/pytest_p2p.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench_n1.json 2> $O/bench_n1.err &&
timeout -k 10 300 python bench.py --rows 1375000 --steps 40 --warmup 5 --fit-trees 0 > $O/bench_1375k.json 2> $O/bench_1375k.err &&
for K in fine coarse uncached; do
  H2OMX_P2P_SYM=$K timeout -k 10 300 python bench.py --rows 1375000 --loopback-ranks 8 --steps 40 --warmup 5 \
    > $O/bench_loop8_$K.json 2> $O/bench_loop8_$K.err || exit 1
done
