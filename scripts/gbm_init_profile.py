"""cProfile of train_ensemble's non-tree work (booster init, y transfer, finish) on the HIGGS shape."""
import cProfile
import os
import pstats
import sys

import numpy as np
import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from h2omx.frame.synthetic import higgs_like  # noqa: E402
from h2omx.models.tree import TreeParams, bin_matrix, compute_edges  # noqa: E402
from h2omx.models.tree.boost import train_ensemble  # noqa: E402

X, y = higgs_like(11_000_000, seed=1000, device="cuda")
tp = TreeParams(max_depth=5, min_rows=10.0, learn_rate=0.1, mode=0, leaf_mode=0, min_split_improvement=1e-5, seed=1)
edges, nvb, nbt = compute_edges(X, 255)
bm = bin_matrix(X, edges, nvb, nbt)
train_ensemble(bm, y, dist="bernoulli", ntrees=2, tparams=tp, seed=1)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(2):
    train_ensemble(bm, y, dist="bernoulli", ntrees=2, tparams=tp, seed=1)
    torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
