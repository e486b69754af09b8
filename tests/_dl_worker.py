"""Worker for tests/test_dl_model_averaging.py: one rank of a gloo world with a
row shard trains H2ODeepLearningEstimator under each replica-sync mode and
writes the final weights' checksum, the scoring AUC and the iteration length."""
import json
import os
import sys

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from h2omx.frame import Frame  # noqa: E402
from h2omx.frame.distributed import unify_domains  # noqa: E402
from h2omx.models import H2ODeepLearningEstimator  # noqa: E402
from h2omx.parallel.comm import Comm  # noqa: E402


def main():
    out_path = sys.argv[1]
    comm = Comm.from_env(device="cpu")
    c = comm if comm.world_size > 1 else None
    rng = np.random.default_rng(5)
    n = 40000
    X = rng.normal(size=(n, 6))
    logit = 1.5 * X[:, 0] - X[:, 1] + 0.8 * X[:, 2] * X[:, 3]
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(6)])
    df["y"] = pd.Categorical(np.where(rng.random(n) < 1 / (1 + np.exp(-logit)), "b", "a"))
    lo, hi = n * comm.rank // comm.world_size, n * (comm.rank + 1) // comm.world_size
    fr = unify_domains(Frame.from_pandas(df.iloc[lo:hi].reset_index(drop=True)), c)
    res = {}
    for name, kw in (("auto", {}), ("fixed", {"train_samples_per_iteration": 5120}),
                     ("epoch", {"train_samples_per_iteration": 0}), ("grad", {"sync_gradients": True})):
        m = H2ODeepLearningEstimator(hidden=[32, 32], epochs=2, seed=3, **kw).train(y="y", training_frame=fr,
                                                                                    comm=c)
        res[name] = {"wsum": float(m.net.flat.double().abs().sum()), "w0": m.net.flat[:8].tolist(),
                     "auc": float(m.training_metrics["AUC"]), "tspi": int(m.train_samples_per_iteration)}
    json.dump(res, open(out_path, "w"))
    comm.shutdown()


if __name__ == "__main__":
    main()
