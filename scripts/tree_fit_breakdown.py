"""Stage timings of one GBM fit on the AutoML shape (10M x 100 by default)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from h2omx.frame import Frame  # noqa: E402
from h2omx.frame.synthetic import wide_gaussian  # noqa: E402
from h2omx.models import H2OGradientBoostingEstimator  # noqa: E402
from h2omx.models.base import compute_metrics  # noqa: E402
from h2omx.models.tree import TreeParams, bin_matrix, compute_edges, train_ensemble  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
X, y = wide_gaussian(rows, 100, seed=5, device="cuda")
fr = Frame.from_tensor(X, y=y, y_categorical=True)
xs = [n for n in fr.names if n != "response"]


def tick(msg, t0):
    torch.cuda.synchronize()
    t = time.time()
    print(f"{msg:>18s}: {1000 * (t - t0):8.1f} ms", flush=True)
    return t


for rep in range(2):
    t = time.time()
    Xf = fr.feature_matrix(xs)
    t = tick("feature_matrix", t)
    e, nv, nbt = compute_edges(Xf, 255, seed=1)
    t = tick("compute_edges", t)
    bm = bin_matrix(Xf, e, nv, nbt, names=xs)
    t = tick("bin_matrix", t)
    ens = train_ensemble(bm, fr.vec("response").data.float(), None, dist="bernoulli", ntrees=50,
                         tparams=TreeParams(max_depth=6), seed=1)
    t = tick("train 50 trees", t)
    m = ens.raw_margin(Xf)
    t = tick("predict", t)
    P = torch.stack([1 - torch.sigmoid(m[0]), torch.sigmoid(m[0])])
    met = compute_metrics("Binomial", P, fr.vec("response"))
    t = tick("metrics", t)
    t0 = time.time()
    H2OGradientBoostingEstimator(ntrees=50, max_depth=6, seed=1).train(y="response", training_frame=fr)
    tick("estimator total", t0)
