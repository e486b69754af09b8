#!/usr/bin/env python3
"""Per-feature checksums of the HIGGS-shape synthetic data and its cut points
(compute_edges on the host CPU), to compare the data / edges two machines
generate from the same seed (precision-pin investigation)."""
import hashlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2omx.frame.synthetic import higgs_like  # noqa: E402
from h2omx.models.tree import compute_edges  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 11_000_000
X, y = higgs_like(rows, seed=1, device=torch.device("cpu"))
e, nv, nbt = compute_edges(X, 255)
out = {"rows": rows,
       "x": [hashlib.sha1(X[f].numpy().tobytes()).hexdigest()[:12] for f in range(X.shape[0])],
       "y": hashlib.sha1(y.numpy().tobytes()).hexdigest()[:12],
       "edges": [hashlib.sha1(np.ascontiguousarray(e[f]).tobytes()).hexdigest()[:12] for f in range(e.shape[0])],
       "cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": ")}
print(json.dumps(out))
