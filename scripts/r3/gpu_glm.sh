#!/bin/bash
# round 3: GLM wave-unit IRLS kernel - correctness, timing at 10M x 100, kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3glm
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dense_gpu.py \
  -k "glm" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 200 python scripts/dense_pmc_run.py 5 > $O/timing_wave.json 2> $O/timing_wave.err || exit $?
H2OMX_GLM_WAVE=0 timeout -k 10 200 python scripts/dense_pmc_run.py 5 > $O/timing_wg.json 2> $O/timing_wg.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python scripts/dense_pmc_run.py 3 > $O/prof.log 2>&1 || exit $?
echo done
