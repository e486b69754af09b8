#!/bin/bash
set -o pipefail
O=gpurun_out/r5m
mkdir -p $O
B=./bench_micro/mlp_phase_micro
{
for mode in 2 4; do
  for K in 16 32 64 128 256 512 1024; do $B 16 32 $K 1 2 $mode; done
  $B 256 512 512 1 2 $mode
  $B 256 512 512 2 2 $mode
  $B 256 512 512 1 1 $mode
done
} > $O/micro.txt 2>&1
