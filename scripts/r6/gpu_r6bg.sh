#!/bin/bash
# r6bg: DRF depth 20 with the 255-bin fine grid (explicit nbins_top_level) on the final pipeline
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6bg
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
for r in 1 2; do
  timeout -k 10 300 python3 scripts/r6/drf_fine255.py > $O/drf255_$r.jsonl 2>> $O/err.log || exit 1
done
