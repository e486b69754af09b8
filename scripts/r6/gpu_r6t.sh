#!/bin/bash
# r6t: row-chunk direct kernel with scalar feature offsets + prefetched rows vs without (variants/head
# = the same tree with the fast path disabled): DRF depth 20 A/B (3 reps interleaved), level tables;
# counters of the direct kernels after the round-6 changes
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6t
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
H=$GRAFT_REPO_ROOT/h2omx/lib/variants/head
for r in 1 2 3; do
  timeout -k 10 300 python3 scripts/drf_deep_ab.py 10000000 new > $O/drf_new_$r.jsonl 2>> $O/err.log || exit 1
  H2OMX_LIB_DIR=$H timeout -k 10 300 python3 scripts/drf_deep_ab.py 10000000 head > $O/drf_head_$r.jsonl 2>> $O/err.log || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drf -o drf -- python3 $GRAFT_REPO_ROOT/scripts/drf_deep_ab.py 10000000 newp > /dev/null 2> $O/drf_prof.err || exit 1
H2OMX_LIB_DIR=$H timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drfh -o drf -- python3 $GRAFT_REPO_ROOT/scripts/drf_deep_ab.py 10000000 headp > /dev/null 2> $O/drfh_prof.err || exit 1
D="python3 $GRAFT_REPO_ROOT/scripts/r6/drf_pmc_run.py 10000000 2"
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU --output-format csv -d $O/pmc1 -o run -- $D > $O/pmc1.json 2> $O/pmc1.err || exit 1
cd $GRAFT_REPO_ROOT
python3 scripts/level_breakdown.py $O/drf/drf_kernel_trace.csv 20 > $O/drf_levels.txt 2>&1 || true
python3 scripts/level_breakdown.py $O/drfh/drf_kernel_trace.csv 20 > $O/drfh_levels.txt 2>&1 || true
python3 scripts/r6/pmc_by_kernel.py $O/pmc1 > $O/pmc_table.txt 2>&1 || true
