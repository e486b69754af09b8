#!/bin/bash
# what bounds the GBM histogram kernels: issue / wait counters per dispatch of one tree
set -o pipefail
O=gpurun_out/r5t
mkdir -p $O
export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAVES SQ_INST_CYCLES_VMEM_RD"; do
  i=$((i+1))
  mkdir -p $O/p$i
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-auc --tree-graph 0 --fit-trees 0 --instrument-steps 0 > $O/p$i/bench.json 2> $O/p$i/bench.err || { tail -5 $O/p$i/bench.err; exit 1; }
  python3 scripts/pmc_dispatch.py $O/p$i 22 > $O/p$i/dispatch.txt
done
