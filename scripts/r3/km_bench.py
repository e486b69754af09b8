"""K-Means Lloyd pass timing at 10M x 100, k = 10: wave kernel vs tile kernel."""
import json, sys, time
import torch
sys.path.insert(0, ".")
import h2omx.ops.dense as OD
dev = torch.device("cuda", 0)
n, d, k = 10_000_000, 100, 10
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn((d, n), device=dev, generator=g)
C = torch.randn((k, d), device=dev, generator=g)
out = {}
for wave in (True, False):
    OD.KM_WAVE = wave
    for _ in range(2):
        OD.kmeans_step(X, C)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        a, s, c, e = OD.kmeans_step(X, C)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 10 * 1e3
    out["wave" if wave else "tile"] = {"ms_per_pass_incl_host": ms, "counts": c.tolist()[:3], "sse": float(e.sum())}
print(json.dumps(out))
