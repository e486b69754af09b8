#!/bin/bash
# r6last3: sanity on the committed tree - full GPU test suite (no -x: every failure listed), smoke(), default bench
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6last3
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 300 python3 scripts/drf_deep_ab.py 10000000 last > $O/drf.jsonl 2> $O/drf.err || exit 1
