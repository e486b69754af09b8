"""GLM IRLS pass (10M x 100, p = 100 + intercept, binomial) and K-Means Lloyd
pass (10M x 100, k = 10) at the AutoML shape, repeated, for rocprofv3
(--kernel-trace for time, --pmc for MFMA counters).  Prints achieved TFLOP/s
from HIP-event timing: GLM Gram 2 * n * (p+2)^2 / 2 (upper tiles), K-Means
distances 2 * n * k * d."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from h2omx.ops import dense as D  # noqa: E402

dev = torch.device("cuda", 0)
n, p, k = 10_000_000, 100, 10
g = torch.Generator(device=dev).manual_seed(1)
X = torch.randn((p, n), device=dev, generator=g)
beta = np.zeros((1, p + 1))
beta[0, :p] = np.random.default_rng(1).normal(scale=0.05, size=p)
eta = torch.from_numpy(beta[0, :p].astype(np.float32)).to(dev) @ X
y = (torch.rand(n, device=dev, generator=g) < torch.sigmoid(eta)).float()
C = X[:, :k].T.contiguous()
Cn = C.cpu().numpy()   # host centroids, as the K-Means model passes them
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
NA_FREE = len(sys.argv) > 2 and sys.argv[2] == "na_free"   # the K-Means model's imputed design
out = {}
WHICH = sys.argv[3] if len(sys.argv) > 3 else "both"
for name, fn, flops in (("glm_irls", lambda: D.glm_irls_pass(X, y, None, None, beta, "binomial", "logit"),
                         n * (p + 2) * (p + 2)),
                        ("kmeans", lambda: D.kmeans_step(X, Cn if NA_FREE else C, na_free=NA_FREE), 2.0 * n * k * p)):
    if WHICH not in ("both", name.split("_")[0]):
        continue
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    out[name] = {"ms_per_pass": dt * 1e3, "useful_tflops": flops / dt / 1e12, "rows": n, "cols": p}
if "kmeans" in out:
    out["kmeans"]["k"] = k
print(json.dumps(out))
