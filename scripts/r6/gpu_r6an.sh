#!/bin/bash
# r6an: DRF depth 20 path switches re-swept on the current kernels (direct-from nodes, wave rows per node,
# host node-count readback cap), 3 reps interleaved
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6an
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
E=h2omx.models.tree.engine:HipTreeBuilder
for r in 1 2 3; do
  for cfg in "base" "DIRECT_WAVE_ROWS=128" "DIRECT_WAVE_ROWS=512" "DIRECT_MIN_NODES=512" "SYNC_NODE_CAP=16384" "PART_WAVE_NODES=512"; do
    a=""; [ "$cfg" != base ] && a="$E.$cfg"
    timeout -k 10 300 python3 scripts/r6/bench_ab.py $a -- scripts/drf_deep_ab.py 10000000 $cfg > $O/drf_${cfg}_$r.jsonl 2>> $O/err.log || exit 1
  done
done
