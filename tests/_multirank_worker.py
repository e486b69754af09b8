"""Worker for test_multirank_gpu.py: trains on this rank's row shard with the
multi-rank GPU path (collectives over gloo so several ranks can share the
box's one GPU) and rank 0 saves the trees."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2omx.models.tree import TreeParams, bin_matrix, compute_edges, train_ensemble  # noqa: E402
from h2omx.parallel.comm import Comm  # noqa: E402


def run(out_path, dist, depth, sample_rate, comm, n=30001, split=0.5):
    rng = np.random.default_rng(11)
    F = 8
    X = rng.normal(size=(F, n)).astype(np.float32)
    X[3, rng.random(n) < 0.05] = np.nan
    logit = X[0] - 0.8 * X[1] * X[2] + np.nan_to_num(X[3])
    y = ((rng.random(n) < 1 / (1 + np.exp(-logit))).astype(np.float32) if dist == "bernoulli"
         else (logit + 0.3 * rng.normal(size=n)).astype(np.float32))
    dev = torch.device("cuda", 0)
    edges, nvb, nbt = compute_edges(torch.from_numpy(X), 63)       # identical cut points everywhere
    world = comm.world_size if comm else 1
    rank = comm.rank if comm else 0
    # world 2: rank 0 takes the first `split` of the rows (unequal shards straddle
    # the fixed-point scale boundaries of tree_begin when n is large enough)
    cuts = [0, int(n * split), n] if world == 2 else [n * r // world for r in range(world + 1)]
    lo, hi = cuts[rank], cuts[rank + 1]
    bm = bin_matrix(torch.from_numpy(X[:, lo:hi]).to(dev), edges, nvb, nbt)
    tp = TreeParams(max_depth=depth, min_rows=2, learn_rate=0.3)
    ens = train_ensemble(bm, torch.from_numpy(y[lo:hi]).to(dev), dist=dist, ntrees=4, tparams=tp,
                         sample_rate=sample_rate, seed=5, comm=comm)
    if rank == 0:
        np.save(out_path, ens.trees)


if __name__ == "__main__":
    out, dist, depth, sr = sys.argv[1], sys.argv[2], int(sys.argv[3]), float(sys.argv[4])
    n = int(sys.argv[5]) if len(sys.argv) > 5 else 30001
    split = float(sys.argv[6]) if len(sys.argv) > 6 else 0.5
    comm = Comm.from_env("cuda") if int(os.environ.get("WORLD_SIZE", "1")) > 1 else None
    run(out, dist, depth, sr, comm, n, split)
    if comm is not None:
        comm.shutdown()
