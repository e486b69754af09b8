#!/bin/bash
# r6d: whole GPU suite (new DL sync-gradient P2P test included) + smoke after the r6 changes
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6d
mkdir -p $O
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_dl_sync_p2p_gpu.py > $O/pytest_dlsync.log 2>&1 || exit 1
timeout -k 10 1100 python -u -m pytest -q --timeout 240 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
rc=$?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
exit $rc
