"""Rank body of tests/test_tree_dp_gpu.py (torch.distributed.run, ranks sharing
the one GPU over gloo): a DRF-style deep forest (mtries, depth 14) grown over
the ranks' row shards of ONE data set with the direct deep-level engine forced
early, so its levels run build -> all-reduce -> scan (h2omx_direct_dp).  Rank 0
saves the trees; the test compares them with a 1-rank run."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from h2omx.models.tree import TreeParams, bin_matrix, compute_edges, train_ensemble  # noqa: E402
from h2omx.models.tree import boost as B  # noqa: E402
from h2omx.parallel.comm import Comm  # noqa: E402


def main() -> int:
    from h2omx.models.tree.engine import HipTreeBuilder

    HipTreeBuilder.DIRECT_MIN_NODES = 8   # the direct deep-level engine from 8 nodes on
    out = sys.argv[1]
    comm = Comm.from_env("cuda")
    dev, r, w = comm.device, comm.rank, comm.world_size
    n, F = 120_000, 24
    g = torch.Generator(device="cpu").manual_seed(7)
    X = torch.randn((F, n), generator=g)
    y = (X[0] * X[1] + 0.5 * X[2] - X[3].abs() + 0.3 * torch.randn((n,), generator=g) > 0).float()
    edges, nvb, nbt = compute_edges(X.to(dev), 20)
    lo, hi = n * r // w, n * (r + 1) // w
    bm = bin_matrix(X[:, lo:hi].contiguous().to(dev), edges, nvb, nbt)
    made = []
    init = B.GpuBooster.__init__

    def spy(self, *a, **k):
        init(self, *a, **k)
        made.append(self)

    B.GpuBooster.__init__ = spy
    tp = TreeParams(max_depth=14, min_rows=1.0, mtries=5, mode=0, leaf_mode=1, seed=3)
    ens = train_ensemble(bm, y[lo:hi].contiguous().to(dev), dist="drf", ntrees=3, tparams=tp, sample_rate=0.632,
                         seed=3, comm=comm if w > 1 else None)
    stats = made[0].builder.stats
    if r == 0:
        np.save(out, ens.trees)
        print(json.dumps({"rank": r, "world": w, "segmented": bool(made[0].builder.segmented),
                          "direct_dp_levels": int(stats.get("direct_dp_levels", 0))}), flush=True)
    comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
