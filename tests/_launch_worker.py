"""Worker for tests/test_launch.py: one rank started by h2omx.runtime.launch
(or alone).  Trains a GBM on this rank's row shard through the tree engine
(the CPU reference builder on gloo, or the HIP engine when H2OMX_WORKER_DEVICE
is "cuda") and rank 0 saves the trees.  ``fail:<rank>`` as the output path
makes that rank exit with code 3 right away (the others sleep)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from h2omx.models.tree import TreeParams, bin_matrix, compute_edges, train_ensemble  # noqa: E402
from h2omx.parallel.comm import Comm  # noqa: E402


def main():
    out = sys.argv[1]
    rank = int(os.environ.get("RANK", "0"))
    if out.startswith("fail:"):
        if rank == int(out.split(":")[1]):
            sys.exit(3)
        time.sleep(120)
        return
    device = os.environ.get("H2OMX_WORKER_DEVICE", "cpu")
    comm = Comm.from_env(device) if int(os.environ.get("WORLD_SIZE", "1")) > 1 else None
    world = comm.world_size if comm else 1
    rng = np.random.default_rng(7)
    n, F = 4001, 6
    X = rng.normal(size=(F, n)).astype(np.float32)
    X[2, rng.random(n) < 0.1] = np.nan
    logit = X[0] - X[1] * X[3] + np.nan_to_num(X[2])
    y = (rng.random(n) < 1 / (1 + np.exp(-logit))).astype(np.float32)
    edges, nvb, nbt = compute_edges(torch.from_numpy(X), 31)
    lo, hi = n * rank // world, n * (rank + 1) // world
    dev = torch.device("cuda", comm.device.index if comm else 0) if device == "cuda" else torch.device("cpu")
    bm = bin_matrix(torch.from_numpy(X[:, lo:hi]).to(dev), edges, nvb, nbt)
    ens = train_ensemble(bm, torch.from_numpy(y[lo:hi]).to(dev), dist="bernoulli", ntrees=3,
                         tparams=TreeParams(max_depth=4, min_rows=2, learn_rate=0.3), seed=3, comm=comm)
    if rank == 0:
        np.save(out, ens.trees)
    if comm is not None:
        comm.shutdown()


if __name__ == "__main__":
    main()
