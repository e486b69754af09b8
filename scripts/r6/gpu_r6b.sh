#!/bin/bash
# r6b: push-based reduce-scatter N-rank level + write-through protocol: P2P / multi-rank tests,
# loopback-8 x3 (new) and x3 (timing-only fenced variant), kernel trace
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6b
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_p2p_gpu.py tests/test_multirank_gpu.py tests/test_tree_dp_gpu.py -m gpu > $O/pytest.log 2>&1 || exit 1
B="python3 bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0 --loopback-ranks 8"
for r in 1 2 3; do
  timeout -k 10 300 $B > $O/loop8_$r.json 2>> $O/plain.err || exit 1
  H2OMX_LIB_DIR=h2omx/lib/variants/fenced timeout -k 10 300 $B > $O/loop8_fenced_$r.json 2>> $O/plain.err || exit 1
done
timeout -k 10 300 python3 bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0 > $O/shard.json 2>> $O/plain.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/loop8 -o loop8 -- python3 $GRAFT_REPO_ROOT/bench.py --rows 1375000 --steps 50 --warmup 5 --fit-trees 0 --instrument-steps 0 --no-auc --loopback-ranks 8 > $O/loop8.json 2> $O/loop8.err || exit 1
