#!/bin/bash
set -o pipefail
O=gpurun_out/r5y
mkdir -p $O
timeout -k 10 600 python scripts/hist_rule_ab.py 10000000 > $O/hist_rule_ab.jsonl 2> $O/hist_rule_ab.err || exit 1
