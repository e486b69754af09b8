"""Microbenchmark of ops.dense.gemm_bf16_nt tile variants (HIP-event timed)."""
import sys

import torch

sys.path.insert(0, ".")
from h2omx.ops import dense as D, dense_lib  # noqa: E402

dev = torch.device("cuda", 0)
lib = dense_lib()


def t(fn, reps=50):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / reps


for (M, N, K, S, kind) in [(8192, 512, 512, 1, "fwd"), (8192, 512, 208, 1, "fwd"), (8192, 2, 512, 1, "fwd"),
                           (8192, 512, 512, 1, "dx"), (512, 513, 8192, 12, "dw"), (512, 513, 8192, 4, "dw"),
                           (8192, 512, 2048, 1, "fwd"), (32768, 512, 512, 1, "fwd")]:
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = torch.randn(N, K, device=dev).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    ld = (N + 7) // 8 * 8
    cb = torch.empty(M, ld, dtype=torch.bfloat16, device=dev)
    cbt = torch.empty(N, M, dtype=torch.bfloat16, device=dev)
    ym = torch.randn(M, ld, device=dev).to(torch.bfloat16)
    cf = torch.empty(M, N, device=dev)
    fl = 2 * M * N * K
    r = {}
    for v in (0, 1, 2):
        lib.h2omx_gemm_bf16_variant(v)
        if kind == "fwd":
            fn = lambda: D.gemm_bf16_nt(A, B, M, N, K, bias=bias, act=1, out_bf16=cb, out_bf16_t=cbt)
        elif kind == "dx":
            fn = lambda: D.gemm_bf16_nt(A, B, M, N, K, ymask=ym, mask_act=1, out_bf16=cb, out_bf16_t=cbt)
        else:
            fn = lambda: D.gemm_bf16_nt(A, B, M, N, K, out_f32=cf, splitk=S)
        r[f"v{v}"] = t(fn)
    lib.h2omx_gemm_bf16_variant(-1)
    r["torch.mm"] = t(lambda: torch.mm(A, B.T))
    print(f"{kind} M={M} N={N} K={K} S={S}: " + "  ".join(f"{k} {v:.1f}us ({fl / v / 1e6:.0f} TF)"
                                                          for k, v in r.items()), flush=True)
