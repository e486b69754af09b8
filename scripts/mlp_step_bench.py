#!/usr/bin/env python3
"""Time the fused small-batch MLP step (ops/mlp.py) alone: 200-512x4-2 ReLU,
256-row batches, 8 steps per HIP-graph replay (as the trainer runs it).
Prints one JSON line; run under rocprofv3 for per-kernel times."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2omx.models.deeplearning import _Net  # noqa: E402
from h2omx.ops.mlp import FusedMlpStep  # noqa: E402

dev = torch.device("cuda", 0)
sizes = [int(v) for v in os.environ.get("SIZES", "200,512,512,512,512,2").split(",")]
M = int(os.environ.get("M", "256"))
net = _Net(sizes, 1, dev, torch.Generator().manual_seed(0))
E1, E2 = torch.zeros_like(net.flat), torch.zeros_like(net.flat)
st = FusedMlpStep(net, 1, M, E1, E2, 0.99, 1e-8, 0.0)
X = torch.randn((8 * M, sizes[0]), device=dev)
Y = torch.randint(0, sizes[-1], (8 * M,), device=dev, dtype=torch.int32)
for i in range(8):
    st.step(X[i * M:(i + 1) * M], Y[i * M:(i + 1) * M])
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for i in range(8):
        st.step(X[i * M:(i + 1) * M], Y[i * M:(i + 1) * M])
for _ in range(5):
    g.replay()
torch.cuda.synchronize()
R = int(os.environ.get("REPLAYS", "50"))
t0 = time.perf_counter()
for _ in range(R):
    g.replay()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / (8 * R)
print(json.dumps({"us_per_step": 1e6 * dt, "samples_per_s": M / dt, "launches": st.launches,
                  "tile": os.environ.get("H2OMX_MLP_TILE", "auto"), "depth": os.environ.get("H2OMX_MLP_DEPTH", "8")}))
