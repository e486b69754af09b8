#!/bin/bash
# r6g (timing diagnostic): partition kernels with 1/16 of the leaf-sum global atomics vs the product build
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --fit-trees 0 --instrument-steps 0 --no-auc"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/base -o base -- $B > $O/base.json 2> $O/base.err || exit 1
H2OMX_LIB_DIR=$GRAFT_REPO_ROOT/h2omx/lib/variants/atomdiag timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/diag -o diag -- $B > $O/diag.json 2> $O/diag.err || exit 1
