#!/bin/bash
# Partition grid sweep + current kernel timeline (GBM HIGGS 11M depth 5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m h2omx.build > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
timeout -k 10 300 python -m pytest tests/test_tree_gpu.py -x -q > gpurun_out/tt.log 2>&1 || { tail -20 gpurun_out/tt.log; exit 1; }
tail -1 gpurun_out/tt.log
for PB in ${PBS:-512 1024 2048 4096}; do
  H2OMX_PART_BLOCKS=$PB timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-auc > gpurun_out/pb_$PB.json 2> gpurun_out/pb_$PB.err || { tail -5 gpurun_out/pb_$PB.err; exit 1; }
  echo "PB=$PB $(python3 -c "import json,sys; d=json.load(open('gpurun_out/pb_$PB.json')); print(d['ms_per_step'])")"
done
OUT=gpurun_out/prof_pb
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-auc > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 scripts/prof_summary.py "$OUT" > $OUT/summary.txt; head -60 $OUT/summary.txt
