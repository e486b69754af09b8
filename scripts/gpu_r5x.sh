#!/bin/bash
# per-node histogram rule cost on the AutoML shapes; AutoML 10M x 100 with sample-based ranges
set -o pipefail
O=gpurun_out/r5x
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python scripts/hist_rule_ab.py 10000000 > $O/hist_rule_ab.jsonl 2> $O/hist_rule_ab.err || exit 1
timeout -k 10 400 python scripts/automl_bench.py --rows 10000000 --cols 100 > $O/automl.json 2> $O/automl.err || exit 1
