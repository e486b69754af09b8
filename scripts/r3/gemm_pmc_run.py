"""One fp32 GEMM (DL forward shape 8192 x 512 x 512, NT, bias + ReLU),
repeated, for rocprofv3 --pmc passes.  argv: tile full"""
import sys

import torch

sys.path.insert(0, ".")
from h2omx.backend import dense as D  # noqa: E402
from h2omx.ops import dense as OD  # noqa: E402

tile, full = int(sys.argv[1]), int(sys.argv[2])
dev = torch.device("cuda", 0)
A = torch.randn(8192, 512, device=dev)
B = torch.randn(512, 512, device=dev)
bias = torch.randn(512, device=dev)
C = torch.empty(8192, 512, device=dev)
OD.set_gemm_tile(tile)
OD.set_gemm_full(full)
for _ in range(20):
    D.gemm(A, B, bias, 1, False, True, out=C)
torch.cuda.synchronize()
print("ok")
