#!/bin/bash
set -o pipefail
O=gpurun_out/${R5TAG:-r5j}
mkdir -p $O
export PYTHONUNBUFFERED=1
B=./bench_micro/mlp_phase_micro
{
for mode in 2 4 8; do
  $B 256 512 512 1 2 $mode
  $B 256 512 64 1 2 $mode
  $B 16 32 512 1 2 $mode
  $B 256 512 1024 1 2 $mode
  $B 8192 512 512 2 2 $mode
done
} > $O/micro.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_dl_step_gpu.py > $O/pytest_dl_step.log 2>&1 || exit 1
for D in 4 8; do
  H2OMX_MLP_DEPTH=$D timeout -k 10 120 python scripts/mlp_step_bench.py >> $O/ab.jsonl 2>> $O/ab.err || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python scripts/mlp_step_bench.py > $O/prof.log 2>&1 || exit 1
