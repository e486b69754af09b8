#!/bin/bash
# Iteration loop on the GPU box: GPU tests, bench, kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-iter}
ls h2omx/lib/libh2omx_tree.so >/dev/null 2>&1 || { python -m h2omx.build > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; cat gpurun_out/build.log; exit 1; }; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
grep -E "passed|failed|PASSED|FAILED|Error" gpurun_out/pytest_gpu_$TAG.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-auc > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 scripts/prof_summary.py "$OUT"; exit 0
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
r = list(csv.DictReader(open(f)))
for x in r[:14]:
    print(f"{x['Name'][:70]:70s} calls={x['Calls']:>5s} avg={float(x['AverageNs'])/1e3:9.1f}us tot={float(x['TotalDurationNs'])/1e6:8.2f}ms {float(x['Percentage']):5.1f}%")
PY
