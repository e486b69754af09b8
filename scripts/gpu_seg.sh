#!/bin/bash
# A/B of the segmented vs scan tree engines: parity tests, bench, profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-seg}
python -m h2omx.build > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; cat gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_tree_gpu.py -x -q > gpurun_out/pytest_tree_$TAG.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_tree_$TAG.log
[ $rc -eq 0 ] || exit $rc
for eng in seg scan; do
  H2OMX_TREE_ENGINE=$eng timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_${TAG}_$eng.json 2> gpurun_out/bench_${TAG}_$eng.err || { tail -20 gpurun_out/bench_${TAG}_$eng.err; exit 1; }
  echo "$eng: $(cat gpurun_out/bench_${TAG}_$eng.json)"
done
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-auc > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 scripts/prof_summary.py "$OUT"
