#!/bin/bash
# x3 data-gradient GEMM: numerics tests, then the DL batch-8192 A/B (x3 dact on / off)
set -o pipefail
O=gpurun_out/r5ag
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dense_gpu.py -k "x3 or dact" tests/test_dl_step_gpu.py > $O/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  for d in 1 0; do
    timeout -k 10 300 python scripts/dl_dact_ab.py $d --model dl-mlp --steps 100 --warmup 10 > $O/dl_d${d}_$rep.json 2> $O/dl_d${d}_$rep.err || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o dl -- python3 $GRAFT_REPO_ROOT/bench.py --model dl-mlp --steps 30 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
