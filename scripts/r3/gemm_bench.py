"""fp32 GEMM timings at the DL-MLP shapes (8192 x 512 x 512 forward / dH /
weight gradient) for every tile mode of ops.dense.set_gemm_tile, plus
torch.matmul (hipBLASLt) as a yardstick.  Prints one JSON line per case."""
import json
import sys

import torch

sys.path.insert(0, ".")
from h2omx.backend import dense as D  # noqa: E402
from h2omx.ops import dense as OD  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1000.0


dev = torch.device("cuda", 0)
torch.manual_seed(0)
cases = [("fwd_nt", 8192, 512, 512, False, True), ("fwd_nt_k200", 8192, 512, 200, False, True),
         ("dH_nn", 8192, 512, 512, False, False), ("wgrad_tn", 512, 512, 8192, True, False),
         ("wgrad_tn_200", 512, 200, 8192, True, False)]
for name, M, N, K, ta, tb in cases:
    A = torch.randn((K, M) if ta else (M, K), device=dev)
    B = torch.randn((N, K) if tb else (K, N), device=dev)
    bias = None if ta else torch.randn(N, device=dev)
    act = 0 if ta else 1
    res = {"case": name, "M": M, "N": N, "K": K}
    for tile, full in ((0, 1), (64, 1), (1, 0), (2, 0), (1, 1), (2, 1)):
        OD.set_gemm_tile(tile)
        OD.set_gemm_full(full)
        us = timeit(lambda: D.gemm(A, B, bias, act, ta, tb))
        key = f"tile{tile}" + ("_full" if full and tile in (1, 2) else "")
        res[f"{key}_us"] = round(us, 2)
        res[f"{key}_tflops"] = round(2 * M * N * K / us / 1e6, 1)
    OD.set_gemm_tile(0)
    OD.set_gemm_full(1)
    Aop = A.T if ta else A
    Bop = B.T if tb else B
    torch.backends.cuda.matmul.allow_tf32 = False
    res["torch_us"] = round(timeit(lambda: Aop @ Bop), 2)
    print(json.dumps(res), flush=True)
Y = torch.randn((8192, 512), device=dev).clamp_min(0)
dZ = torch.randn((8192, 512), device=dev)
W = torch.randn((512, 512), device=dev)
for tile in (1, 2):
    for full in (0, 1):
        OD.set_gemm_full(full)
        us = timeit(lambda: OD.gemm_dact(dZ, W, Y, 1, tile=tile))
        print(json.dumps({"case": f"dact_tile{tile}_full{full}", "us": round(us, 2)}), flush=True)
OD.set_gemm_full(1)
us = timeit(lambda: D.act_backward_bias(Y, D.gemm(dZ, W), 1))
print(json.dumps({"case": "gemm+act_backward_bias(tile0)", "us": round(us, 2)}), flush=True)
