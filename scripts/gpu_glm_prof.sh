#!/bin/bash
# GLM binomial (plain and lambda search) on 10M x 100: wall time + kernel totals.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/glmprof; mkdir -p $OUT
timeout -k 10 300 python3 scripts/deep_tree_prof.py 10000000 glm > $OUT/plain.txt 2>&1 || { tail -5 $OUT/plain.txt; exit 1; }
cat $OUT/plain.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 scripts/deep_tree_prof.py 10000000 glm > $OUT/prof.txt 2>&1 || { tail -5 $OUT/prof.txt; exit 1; }
python3 - "$OUT/prof" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
print("total kernel ms", sum(float(x['TotalDurationNs']) for x in rows) / 1e6)
for x in rows[:14]:
    print(f"{x['Name'][:60]:60s} calls={x['Calls']:>6s} avg={float(x['AverageNs'])/1e3:8.1f}us tot={float(x['TotalDurationNs'])/1e6:8.2f}ms")
PY
