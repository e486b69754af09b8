#!/bin/bash
# histogram lane copies: level 0 8 (current) vs 16 (conflict-free 16-lane groups);
# routed level 1 without / with 16 copies
set -o pipefail
O=gpurun_out/r5s
mkdir -p $O
export PYTHONUNBUFFERED=1
H2OMX_HIST_L0_COPIES=16 H2OMX_HIST_ROUTE_COPIES=16 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 \
  --timeout-method thread -m gpu tests/test_tree_gpu.py > $O/pytest_cop16.log 2>&1 || exit 1
for rep in 1 2; do
  for cfg in "8 0" "16 0" "16 16" "8 8"; do
    set -- $cfg
    H2OMX_HIST_L0_COPIES=$1 H2OMX_HIST_ROUTE_COPIES=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 3 \
      --fit-trees 0 > $O/bench_l0c$1_rc$2_$rep.json 2> $O/bench_l0c$1_rc$2_$rep.err || exit 1
  done
done
export TMPDIR=/tmp
mkdir -p $O/pmc16
H2OMX_HIST_L0_COPIES=16 H2OMX_HIST_ROUTE_COPIES=16 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE SQ_LDS_IDX_ACTIVE \
  SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD --output-format csv -d $O/pmc16 -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-auc --tree-graph 0 --fit-trees 0 --instrument-steps 0 > $O/pmc16/bench.json 2> $O/pmc16/bench.err || exit 1
python3 scripts/pmc_levels_table.py $O/pmc16 > $O/pmc16_table.txt
