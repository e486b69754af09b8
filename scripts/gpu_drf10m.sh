#!/bin/bash
# DRF depth 20 on the AutoML shape (10M x 100): wall time with and without the
# direct deep-level engine, then a kernel trace of the direct run for the per-level table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/drf10m
mkdir -p $OUT
H2OMX_DIRECT_MIN_NODES=0 timeout -k 10 300 python3 scripts/deep_tree_prof.py 10000000 drf > $OUT/subtract.txt 2>&1 || { tail -5 $OUT/subtract.txt; exit 1; }
cat $OUT/subtract.txt
timeout -k 10 300 python3 scripts/deep_tree_prof.py 10000000 drf > $OUT/direct.txt 2>&1 || { tail -5 $OUT/direct.txt; exit 1; }
cat $OUT/direct.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 scripts/deep_tree_prof.py 10000000 drf > $OUT/prof.txt 2>&1 || { tail -5 $OUT/prof.txt; exit 1; }
python3 scripts/level_breakdown.py $(ls $OUT/prof/*/run_kernel_trace.csv $OUT/prof/run_kernel_trace.csv 2>/dev/null | tail -1) 20 > $OUT/levels.txt
cat $OUT/levels.txt
