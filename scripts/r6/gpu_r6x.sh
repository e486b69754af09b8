#!/bin/bash
# r6x: direct (eligible-feature) levels from earlier depths with column-major planes (DIRECT_MIN_NODES x
# COLMAJOR_EVERY), DRF depth 20, 2 reps per arm + level table of the best guess
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6x
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
E=h2omx.models.tree.engine:HipTreeBuilder
for r in 1 2; do
  for cfg in "1024 6" "256 6" "32 6" "32 4" "2 6"; do
    set -- $cfg
    timeout -k 10 300 python3 scripts/r6/bench_ab.py $E.DIRECT_MIN_NODES=$1 $E.COLMAJOR_EVERY=$2 -- scripts/drf_deep_ab.py 10000000 dm$1_cm$2 > $O/drf_dm$1_cm$2_$r.jsonl 2>> $O/err.log || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dm32 -o drf -- python3 $GRAFT_REPO_ROOT/scripts/r6/bench_ab.py $E.DIRECT_MIN_NODES=32 -- scripts/drf_deep_ab.py 10000000 dm32p > /dev/null 2> $O/dm32_prof.err || exit 1
cd $GRAFT_REPO_ROOT
python3 scripts/level_breakdown.py $O/dm32/drf_kernel_trace.csv 20 > $O/dm32_levels.txt 2>&1 || true
