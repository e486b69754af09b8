#!/bin/bash
# round 3: precision pin at the headline resolution (11M rows, 50 trees) - GPU half
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prec11m
mkdir -p $O
timeout -k 10 600 python -u scripts/precision_parity.py --part gpu --out $O --rows 11000000 > $O/gpu.log 2>&1 || exit $?
timeout -k 10 200 python bench.py > gpurun_out/bench_default_r3.json 2> gpurun_out/bench_default_r3.err || exit $?
echo done
