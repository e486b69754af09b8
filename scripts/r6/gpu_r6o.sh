#!/bin/bash
# r6o: DRF depth-20 path-switch sweep on the round-6 kernels (3 reps interleaved):
# wave-chunk partition from level 0 (PART_WAVE_NODES 1) and direct levels from 512 nodes
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6o
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
E=h2omx.models.tree.engine:HipTreeBuilder
for r in 1 2 3; do
  timeout -k 10 300 python3 scripts/r6/bench_ab.py $E.COLMAJOR_EVERY=6 -- scripts/drf_deep_ab.py 10000000 base > $O/drf_base_$r.jsonl 2>> $O/err.log || exit 1
  timeout -k 10 300 python3 scripts/r6/bench_ab.py $E.PART_WAVE_NODES=1 -- scripts/drf_deep_ab.py 10000000 pw1 > $O/drf_pw1_$r.jsonl 2>> $O/err.log || exit 1
  timeout -k 10 300 python3 scripts/r6/bench_ab.py $E.PART_WAVE_NODES=256 -- scripts/drf_deep_ab.py 10000000 pw256 > $O/drf_pw256_$r.jsonl 2>> $O/err.log || exit 1
  timeout -k 10 300 python3 scripts/r6/bench_ab.py $E.DIRECT_MIN_NODES=512 -- scripts/drf_deep_ab.py 10000000 dm512 > $O/drf_dm512_$r.jsonl 2>> $O/err.log || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pw1 -o drf -- python3 $GRAFT_REPO_ROOT/scripts/r6/bench_ab.py $E.PART_WAVE_NODES=1 -- scripts/drf_deep_ab.py 10000000 pw1p > /dev/null 2> $O/pw1_prof.err || exit 1
cd $GRAFT_REPO_ROOT
python3 scripts/level_breakdown.py $O/pw1/drf_kernel_trace.csv 20 > $O/pw1_levels.txt 2>&1 || true
