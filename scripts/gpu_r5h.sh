#!/bin/bash
# LDS-staged fused MLP step vs register-direct; numerics; timeline
set -o pipefail
O=gpurun_out/r5h
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_dl_step_gpu.py > $O/pytest_dl_step.log 2>&1 || exit 1
for D in 100 2; do for T in auto 1,2 2,2 1,1; do
  if [ "$T" = auto ]; then unset H2OMX_MLP_TILE; else export H2OMX_MLP_TILE=$T; fi
  H2OMX_MLP_DEPTH=$D timeout -k 10 120 python scripts/mlp_step_bench.py >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done; done
unset H2OMX_MLP_TILE
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python scripts/mlp_step_bench.py > $O/prof.log 2>&1 || exit 1
