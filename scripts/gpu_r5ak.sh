#!/bin/bash
# DRF depth 20 (10 trees, 10M x 100) kernel trace: GPU busy vs idle per tree
set -o pipefail
O=gpurun_out/r5ak
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/drf -o drf -- python3 $GRAFT_REPO_ROOT/scripts/drf_deep_ab.py > $GRAFT_REPO_ROOT/$O/drf.log 2>&1
