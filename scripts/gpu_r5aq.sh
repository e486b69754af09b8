#!/bin/bash
# direct deep-level kernels forced to 5 waves per SIMD (with register spills): DRF depth-20 timing
set -o pipefail
O=gpurun_out/r5aq
mkdir -p $O
timeout -k 10 300 python scripts/drf_deep_ab.py 10000000 wpe5 > $O/drf.jsonl 2> $O/drf.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/drf -o drf -- python3 $GRAFT_REPO_ROOT/scripts/drf_deep_ab.py > $GRAFT_REPO_ROOT/$O/drf_prof.log 2>&1
