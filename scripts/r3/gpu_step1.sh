#!/bin/bash
# round 3, step 1: graph replay / strong-scaling tests + bench with per-tree instrumentation
set -o pipefail
mkdir -p gpurun_out/r3s1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_tree_gpu.py -k "graph_replay or gbm_bernoulli or fused_routing" > gpurun_out/r3s1/pytest_tree.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_bench_contract.py -m gpu > gpurun_out/r3s1/pytest_bench.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r3s1/bench_graph.json 2> gpurun_out/r3s1/bench_graph.err || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --tree-graph 0 > gpurun_out/r3s1/bench_eager.json 2> gpurun_out/r3s1/bench_eager.err || exit $?
echo done
