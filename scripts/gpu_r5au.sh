#!/bin/bash
# diagnostic (timing only, not kept): seg_direct_wave_kernel scanning every feature twice
set -o pipefail
O=gpurun_out/r5au
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/drf -o drf -- python3 $GRAFT_REPO_ROOT/scripts/drf_deep_ab.py > $GRAFT_REPO_ROOT/$O/drf_prof.log 2>&1
