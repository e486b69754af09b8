#!/bin/bash
# round-5 final validation: whole GPU suite, smoke, headline + strong-scaling shard + loopback proxy, DL, XGBoost
set -o pipefail
O=gpurun_out/r5be
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 300 python bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0 > $O/bench_1375k.json 2> $O/bench_1375k.err || exit 1
timeout -k 10 300 python bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0 --loopback-ranks 8 > $O/bench_loop8.json 2> $O/bench_loop8.err || exit 1
timeout -k 10 300 python bench.py --model dl-mlp --steps 100 --warmup 10 > $O/bench_dl.json 2> $O/bench_dl.err || exit 1
timeout -k 10 300 python bench.py --model dl-mlp --estimator-defaults --steps 400 --warmup 40 > $O/bench_dlest.json 2> $O/bench_dlest.err || exit 1
timeout -k 10 300 python bench.py --model xgboost-airlines --steps 10 --warmup 2 > $O/bench_xgb.json 2> $O/bench_xgb.err || exit 1
timeout -k 10 300 python scripts/drf_deep_ab.py 10000000 final > $O/drf.jsonl 2> $O/drf.err || exit 1
timeout -k 10 400 python scripts/automl_bench.py --rows 10000000 --cols 100 > $O/automl.json 2> $O/automl.err || exit 1
