#!/bin/bash
# DRF depth 20 on 10M x 100: direct (eligible-feature) levels from a lower node count.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/drf_direct; mkdir -p $OUT
export TMPDIR=/tmp
for M in "$@"; do
  echo "== H2OMX_DIRECT_MIN_NODES=$M"
  H2OMX_DIRECT_MIN_NODES=$M timeout -k 10 300 python3 scripts/deep_tree_prof.py 10000000 drf > $OUT/m$M.txt 2>&1 || { tail -5 $OUT/m$M.txt; exit 1; }
  grep "DRF" $OUT/m$M.txt | cut -c1-200
done
