"""One bf16 forward GEMM shape, repeated (for rocprofv3 --pmc passes)."""
import sys

import torch

sys.path.insert(0, ".")
from h2omx.ops import dense as D  # noqa: E402

dev = torch.device("cuda", 0)
M, N, K = 8192, 512, 512
A = torch.randn(M, K, device=dev).to(torch.bfloat16)
B = torch.randn(N, K, device=dev).to(torch.bfloat16)
bias = torch.randn(N, device=dev)
cb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
cbt = torch.empty(N, M, dtype=torch.bfloat16, device=dev)
for _ in range(20):
    D.gemm_bf16_nt(A, B, M, N, K, bias=bias, act=1, out_bf16=cb, out_bf16_t=cbt)
torch.cuda.synchronize()
print("ok")
