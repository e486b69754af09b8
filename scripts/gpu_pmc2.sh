#!/bin/bash
# per-dispatch counters for one kernel: gpu_pmc2.sh TAG KERNEL "counter set 1" "counter set 2" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; KN=$2; shift 2
python -m h2omx.build > gpurun_out/build.log 2>&1 || exit 1
i=0
for set in "$@"; do
  i=$((i+1)); OUT=gpurun_out/${TAG}_$i; mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-auc > $OUT/bench.json 2> $OUT/bench.err || { echo "set $i failed"; tail -3 $OUT/bench.err; exit 1; }
  python3 scripts/pmc_kernel.py $OUT $KN
done
