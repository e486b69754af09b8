#!/bin/bash
# r6al: kernel trace of the DRF depth-20 fit on the current tree (per-tree walls, gaps, fit prologue)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6al
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof -o drf -- python3 $GRAFT_REPO_ROOT/scripts/drf_deep_ab.py 10000000 prof > $O/drf.jsonl 2> $O/prof.err || exit 1
cd $GRAFT_REPO_ROOT
python3 scripts/level_breakdown.py $O/prof/drf_kernel_trace.csv 20 > $O/levels.txt 2>&1 || true
