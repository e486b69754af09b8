"""Stage timings of the end-to-end GBM fit of bench.py (HIGGS-shape 11M x 28, 50 trees)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from h2omx.frame.synthetic import higgs_like  # noqa: E402
from h2omx.metrics.core import auc_from_scores  # noqa: E402
from h2omx.models.tree import TreeParams, bin_matrix, compute_edges  # noqa: E402
from h2omx.models.tree.boost import train_ensemble  # noqa: E402

X, y = higgs_like(11_000_000, seed=1000, device="cuda")
tp = TreeParams(max_depth=5, min_rows=10.0, learn_rate=0.1, mode=0, leaf_mode=0, min_split_improvement=1e-5, seed=1)


def tick(msg, t0):
    torch.cuda.synchronize()
    t = time.perf_counter()
    print(f"{msg:>14s}: {1000 * (t - t0):8.1f} ms", flush=True)
    return t


for rep in range(3):
    torch.cuda.synchronize()
    t0 = t = time.perf_counter()
    edges, nvb, nbt = compute_edges(X, 255)
    t = tick("sketch", t)
    bm = bin_matrix(X, edges, nvb, nbt)
    t = tick("bin", t)
    ens = train_ensemble(bm, y, dist="bernoulli", ntrees=50, tparams=tp, seed=1)
    t = tick("50 trees", t)
    auc = auc_from_scores(ens._state.Fm[0, : bm.n], y)
    t = tick("auc", t)
    tick(f"total (AUC {auc:.4f})", t0)
