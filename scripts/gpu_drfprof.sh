#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m h2omx.build > gpurun_out/build.log 2>&1 || exit 1
OUT=gpurun_out/prof_drf
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 scripts/drf_time.py auto > $OUT/out.txt 2> $OUT/err.txt || { tail -5 $OUT/err.txt; exit 1; }
cat $OUT/out.txt
python3 scripts/prof_summary.py "$OUT" | head -18
