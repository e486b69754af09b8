"""K sweep of the fp32 NT GEMM (M=8192, N=512) for the FULL w64 kernels,
gemm64 and hipBLASLt: separates the per-K-step loop cost from the fixed
prologue / epilogue cost.  Times come from the kernel trace (run under
rocprofv3 --kernel-trace); this script only issues the launches."""
import sys

import torch

sys.path.insert(0, ".")
from h2omx.backend import dense as D  # noqa: E402
from h2omx.ops import dense as OD  # noqa: E402

dev = torch.device("cuda", 0)
for K in (128, 256, 512, 1024, 2048):
    A = torch.randn(8192, K, device=dev)
    B = torch.randn(512, K, device=dev)
    bias = torch.randn(512, device=dev)
    C = torch.empty(8192, 512, device=dev)
    for tile in (0, 1, 2):
        OD.set_gemm_tile(tile)
        for _ in range(20):
            D.gemm(A, B, bias, 1, False, True, out=C)
    OD.set_gemm_tile(0)
    for _ in range(20):
        torch.addmm(bias, A, B.T)
    torch.cuda.synchronize()
print("ok")
