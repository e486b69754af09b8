#!/bin/bash
# DRF depth 20 on 10M x 100 under rocprofv3 --stats, env A vs env B: per-kernel totals.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; A=$2; B=$3
for V in A B; do
  E=${!V}
  OUT=gpurun_out/drfprof_${TAG}_$V; mkdir -p $OUT
  export $E
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 scripts/deep_tree_prof.py 10000000 drf > $OUT/out.txt 2>&1 || { tail -5 $OUT/out.txt; exit 1; }
  echo "== $V [$E]"; grep DRF $OUT/out.txt
  python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for x in list(csv.DictReader(open(f)))[:8]:
    print(f"{x['Name'][:60]:60s} calls={x['Calls']:>6s} tot={float(x['TotalDurationNs'])/1e6:8.2f}ms")
PY
done
