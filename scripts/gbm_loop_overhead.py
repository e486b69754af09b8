"""Where the end-to-end fit's per-tree time goes: booster init, host launch time of step(), GPU time, finish."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from h2omx.frame.synthetic import higgs_like  # noqa: E402
from h2omx.models.tree import TreeParams, bin_matrix, compute_edges  # noqa: E402
from h2omx.models.tree.boost import GpuBooster, TreeEnsemble, init_margin  # noqa: E402

X, y = higgs_like(11_000_000, seed=1000, device="cuda")
tp = TreeParams(max_depth=5, min_rows=10.0, learn_rate=0.1, mode=0, leaf_mode=0, min_split_improvement=1e-5, seed=1)
edges, nvb, nbt = compute_edges(X, 255)
bm = bin_matrix(X, edges, nvb, nbt)
y_np = y.float().cpu().numpy()
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ens = TreeEnsemble(trees=np.zeros((0, 1)), K=1, dist="bernoulli", init_f=init_margin("bernoulli", y_np, None, 1),
                       nbt=nbt, feature_names=bm.names)
    gb = GpuBooster(bm, y_np, None, ens, tp, 1.0, 1, None, {})
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    host = []
    for t in range(50):
        a = time.perf_counter()
        gb.step()
        host.append(time.perf_counter() - a)
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    gb.finish()
    t4 = time.perf_counter()
    h = np.array(host) * 1e3
    print(f"rep {rep}: init {1e3 * (t1 - t0):.1f} ms | 50 steps host-issue {1e3 * (t2 - t1):.1f} ms "
          f"(per step median {np.median(h):.3f} max {h.max():.2f}) | drain {1e3 * (t3 - t2):.1f} ms | "
          f"finish {1e3 * (t4 - t3):.1f} ms", flush=True)
