#!/bin/bash
# A/B of env switches on the GBM headline: bench + one-step timeline per variant.
# Usage: [BENCH_ARGS="--model ..."] gpu_ab.sh TAG "ENV=.. ENV=.." "ENV=.." ...   (empty string = defaults)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=$1; shift
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
i=0
for V in "$@"; do
  i=$((i+1)); O=gpurun_out/$TAG/v$i; mkdir -p $O
  echo "== v$i: ${V:-defaults}"
  env $V timeout -k 10 300 python bench.py $BENCH_ARGS --steps 30 --warmup 3 --fit-trees 0 --instrument-steps 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench.json')); print('  ms/step', round(d['ms_per_step'],4), 'auc', d['train_auc'])"
  env $V timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py $BENCH_ARGS --steps 5 --warmup 1 --no-auc --fit-trees 0 --instrument-steps 0 > $O/prof.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
  python3 scripts/prof_summary.py "$O/prof" > $O/summary.txt; grep -E "one step|partition|hist_build|kernel-busy" $O/summary.txt | sed -n '/one step/,$p' | head -14
done
