#!/bin/bash
# x3 GEMM variants (issue order / LDS double buffer) vs hipBLASLt
set -o pipefail
O=gpurun_out/r5o
mkdir -p $O
timeout -k 10 200 python scripts/gemm_x3_bench.py > $O/gemm_x3.txt 2>&1 || exit 1
