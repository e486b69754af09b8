"""Fixed-cost probe of gemm_bf16_nt: K sweep x epilogue outputs (variant 2)."""
import sys

import torch

sys.path.insert(0, ".")
from h2omx.ops import dense as D, dense_lib  # noqa: E402

dev = torch.device("cuda", 0)
lib = dense_lib()
lib.h2omx_gemm_bf16_variant(2)


def t(fn, reps=100):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / reps


M, N = 8192, 512
for K in (8, 64, 128, 256, 512):
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = torch.randn(N, K, device=dev).to(torch.bfloat16)
    cf = torch.empty(M, N, device=dev)
    cb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    cbt = torch.empty(N, M, dtype=torch.bfloat16, device=dev)
    r = {"f32": t(lambda: D.gemm_bf16_nt(A, B, M, N, K, out_f32=cf)),
         "bf16": t(lambda: D.gemm_bf16_nt(A, B, M, N, K, out_bf16=cb)),
         "bf16T": t(lambda: D.gemm_bf16_nt(A, B, M, N, K, out_bf16_t=cbt)),
         "both": t(lambda: D.gemm_bf16_nt(A, B, M, N, K, out_bf16=cb, out_bf16_t=cbt))}
    # host-side cost of one wrapper call (no GPU wait)
    import time
    torch.cuda.synchronize()
    h0 = time.perf_counter()
    for _ in range(200):
        D.gemm_bf16_nt(A, B, M, N, K, out_bf16=cb)
    h1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"K={K}: " + "  ".join(f"{k} {v:.1f}us" for k, v in r.items()) + f"  host/call {(h1 - h0) / 200 * 1e6:.1f}us",
          flush=True)
