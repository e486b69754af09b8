#!/usr/bin/env python3
"""A/B of the hidden-layer data-gradient route in the batch-8192 DL bench:
argv[1] = 1 (x3 GEMM on W^T, ops.dense.X3_DACT) or 0 (fp32 MFMA gemm_dact);
the rest goes to bench.py."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    from h2omx.ops import dense as OD

    OD.X3_DACT = sys.argv[1] == "1"
    import bench

    sys.exit(bench.main(sys.argv[2:]))
