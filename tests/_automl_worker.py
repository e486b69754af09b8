"""Worker for tests/test_automl_parallel.py: one rank of a gloo world holding
a row shard; runs AutoML with the given scheduler and writes its leaderboard."""
import json
import os
import sys

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from h2omx.automl import H2OAutoML  # noqa: E402
from h2omx.frame import Frame  # noqa: E402
from h2omx.frame.distributed import unify_domains  # noqa: E402
from h2omx.parallel.comm import Comm  # noqa: E402


def main():
    out_path, parallelism = sys.argv[1], sys.argv[2]
    explo = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    comm = Comm.from_env(device="cpu")
    c = comm if comm.world_size > 1 else None
    rng = np.random.default_rng(21)
    n = 900
    X = rng.normal(size=(n, 4))
    df = pd.DataFrame(X, columns=["a", "b", "c", "d"])
    df["g"] = pd.Categorical(rng.choice(list("pqr"), n))
    eta = X[:, 0] - 0.7 * X[:, 1] + (df["g"] == "p") * 0.8
    df["y"] = pd.Categorical(np.where(rng.random(n) < 1 / (1 + np.exp(-eta)), "1", "0"))
    lo, hi = n * comm.rank // comm.world_size, n * (comm.rank + 1) // comm.world_size
    fr = unify_domains(Frame.from_pandas(df.iloc[lo:hi].reset_index(drop=True)), c)
    aml = H2OAutoML(max_models=5 if explo else 3, nfolds=2, seed=5, project_name=f"p_{parallelism}",
                    parallelism=parallelism, exploitation_ratio=explo)
    aml.train(y="y", training_frame=fr, comm=c)
    json.dump({"leaderboard": aml.leaderboard, "events": aml.events}, open(f"{out_path}.{comm.rank}", "w"))
    comm.shutdown()


if __name__ == "__main__":
    main()
