#!/bin/bash
# One bench model under rocprofv3 --kernel-trace --stats: bench JSON + kernel summary / step timeline.
# Usage: gpu_prof_model.sh TAG MODEL [extra bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; M=$2; shift 2
timeout -k 10 600 python bench.py --model $M --steps 20 --warmup 3 "$@" > gpurun_out/bench_${TAG}_$M.json 2> gpurun_out/bench_${TAG}_$M.err || { tail -20 gpurun_out/bench_${TAG}_$M.err; exit 1; }
cat gpurun_out/bench_${TAG}_$M.json
OUT=gpurun_out/prof_${TAG}_$M; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --model $M --steps 5 --warmup 1 --no-auc "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 scripts/prof_summary.py "$OUT" > $OUT/summary.txt
cat $OUT/summary.txt
