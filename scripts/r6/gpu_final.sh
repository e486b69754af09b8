#!/bin/bash
# round-6 final validation on one MI355X: whole GPU suite, smoke, then every headline config
# (3 fresh processes for the tree benchmarks), DL, GLM / K-Means passes, DRF depth 20, AutoML
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6final
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
S="--rows 1375000 --steps 50 --warmup 5 --fit-trees 0"
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py > $O/bench_default_$r.json 2> $O/bench_default_$r.err || exit 1
  timeout -k 10 300 python3 bench.py $S > $O/bench_1375k_$r.json 2> $O/bench_1375k_$r.err || exit 1
  timeout -k 10 300 python3 bench.py $S --loopback-ranks 8 > $O/bench_loop8_$r.json 2> $O/bench_loop8_$r.err || exit 1
  timeout -k 10 300 python3 bench.py --model xgboost-airlines --steps 20 --warmup 3 > $O/bench_xgb_$r.json 2> $O/bench_xgb_$r.err || exit 1
done
timeout -k 10 300 python3 bench.py --model dl-mlp --steps 100 --warmup 10 > $O/bench_dl.json 2> $O/bench_dl.err || exit 1
timeout -k 10 300 python3 bench.py --model dl-mlp --estimator-defaults --steps 400 --warmup 40 > $O/bench_dlest.json 2> $O/bench_dlest.err || exit 1
timeout -k 10 300 python3 scripts/dense_pmc_run.py 20 na_free > $O/dense.json 2> $O/dense.err || exit 1
timeout -k 10 300 python3 scripts/drf_deep_ab.py 10000000 final > $O/drf.jsonl 2> $O/drf.err || exit 1
timeout -k 10 600 python3 scripts/automl_bench.py --rows 10000000 --cols 100 > $O/automl.json 2> $O/automl.err || exit 1
