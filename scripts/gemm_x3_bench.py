#!/usr/bin/env python3
"""fp32 GEMM C = A B^T (+ bias, ReLU) on MI355X: hipBLASLt (torch.addmm) vs the
own fp32 MFMA kernel (gemm_w64, ops.dense.gemm_fp32) vs the x3 bf16-split
kernel (ops.mlp.gemm_x3) and what ops.dense.gemm routes the shape to.  Accuracy vs float64; one JSON line
per shape."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2omx.ops import dense as OD  # noqa: E402
from h2omx.ops.mlp import gemm_x3  # noqa: E402

dev = torch.device("cuda", 0)


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return 1000.0 * e0.elapsed_time(e1) / reps


for M, N, K in ((8192, 512, 512), (8192, 512, 200), (8192, 2048, 2048), (256, 512, 512), (65536, 512, 512)):
    torch.manual_seed(0)
    A = torch.randn((M, K), device=dev)
    B = torch.randn((N, K), device=dev) * 0.05
    b = torch.randn((N,), device=dev)
    ref = torch.relu(A.double() @ B.double().T + b.double())
    out = {"M": M, "N": N, "K": K}
    for name, fn in (("hipblaslt", lambda: torch._addmm_activation(b, A, B.T)),
                     ("own_fp32_mfma", lambda: OD.gemm_fp32(A, B, bias=b, act=1, tb=True)),
                     ("x3", lambda: gemm_x3(A, B, b, 1)), ("routed", lambda: OD.gemm(A, B, bias=b, act=1, tb=True))):
        C = fn()
        err = ((C.double() - ref).abs().max() / ref.abs().max()).item()
        us = timeit(fn)
        out[name] = {"us": round(us, 2), "tflops": round(2 * M * N * K / us / 1e6, 1), "max_rel_err": err}
    print(json.dumps(out), flush=True)
