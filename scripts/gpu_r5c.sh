#!/bin/bash
# round 5: fused small-batch DL step (csrc/mlp_kernels.hip) numerics + bench + timeline
set -o pipefail
O=gpurun_out/${R5TAG:-r5c}
mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_dl_step_gpu.py > $O/pytest_dl_step.log 2>&1
rc=$?
timeout -k 10 300 python bench.py --model dl-mlp --estimator-defaults --steps 400 --warmup 40 > $O/bench_dlest.json 2> $O/bench_dlest.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dlest -o prof -- python bench.py --model dl-mlp --estimator-defaults --steps 200 --warmup 20 > $O/prof_dlest.log 2>&1 || exit 1
exit $rc
