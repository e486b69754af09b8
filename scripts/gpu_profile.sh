#!/bin/bash
# Kernel-level profile of the headline bench (rocprofv3 kernel trace + stats).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${1:-bench}
mkdir -p $OUT
shift || true
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --steps 5 --warmup 1 "$@" > $OUT/bench.json 2> $OUT/bench.err
rc=$?
cat $OUT/bench.json
find $OUT -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -40 {}'
exit $rc
