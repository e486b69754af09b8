#!/bin/bash
# round 3, step 5: fp32 GEMM variants (tests, microbench, MFMA counters)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3s5
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_dense_gpu.py tests/test_estimators_gpu.py -k "gemm or deeplearning" > $O/pytest_gemm.log 2>&1 || exit $?
timeout -k 10 200 python scripts/r3/gemm_bench.py > $O/gemm_bench.jsonl 2> $O/gemm_bench.err || exit $?
i=0
for cfg in "1 0" "1 1" "2 1"; do
  for set in "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS" \
             "FETCH_SIZE SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"; do
    i=$((i+1)); OUT=$O/pmc$i; mkdir -p $OUT
    echo "$cfg | $set" > $OUT/cfg.txt
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $OUT -o run -- python3 scripts/r3/gemm_pmc_run.py $cfg > /dev/null 2> $OUT/err || { echo "pmc $i failed"; tail -5 $OUT/err; exit 1; }
    python3 scripts/pmc_summary.py $OUT > $OUT/summary.txt || exit 1
  done
done
timeout -k 10 200 python bench.py --model dl-mlp --steps 30 --warmup 5 > $O/bench_dl_fp32.json 2> $O/bench_dl_fp32.err || exit $?
timeout -k 10 200 python bench.py --model dl-mlp --estimator-defaults --steps 300 --warmup 30 > $O/bench_dl_estdef.json 2> $O/bench_dl_estdef.err || exit $?
echo done
