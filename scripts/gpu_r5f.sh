#!/bin/bash
# fused MLP step A/B: k-group rotation x padded strides x depth; numerics
set -o pipefail
O=gpurun_out/r5f
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_dl_step_gpu.py > $O/pytest_dl_step.log 2>&1 || exit 1
for D in 2 4; do for R in 0 1; do for P in 0 1; do
  H2OMX_MLP_DEPTH=$D H2OMX_MLP_ROT=$R H2OMX_MLP_PAD=$P timeout -k 10 120 python scripts/mlp_step_bench.py | \
    sed "s/}$/, \"rot\": $R, \"pad\": $P}/" >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done; done; done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python scripts/mlp_step_bench.py > $O/prof.log 2>&1 || exit 1
