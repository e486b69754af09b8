"""Worker for tests/test_munging.py: one rank of a gloo world holding a row
shard of a fixed frame; runs the munging ops and writes results (JSON)."""
import json
import os
import sys

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from h2omx.frame import Frame  # noqa: E402
from h2omx.frame import munging as M  # noqa: E402
from h2omx.frame.distributed import unify_domains  # noqa: E402
from h2omx.parallel.comm import Comm  # noqa: E402


def data(n=1000):
    rng = np.random.default_rng(7)
    df = pd.DataFrame({"g": rng.choice(["a", "b", "c"], n), "h": rng.integers(0, 3, n).astype(float),
                       "x": rng.normal(size=n), "y": rng.integers(0, 100, n).astype(float)})
    df.loc[::37, "x"] = np.nan
    df["g"] = pd.Categorical(df["g"])
    return df


def main():
    out_path = sys.argv[1]
    comm = Comm.from_env(device="cpu")
    c = comm if comm.world_size > 1 else None
    df = data()
    n = len(df)
    lo = n * comm.rank // comm.world_size
    hi = n * (comm.rank + 1) // comm.world_size
    part = df.iloc[lo:hi].reset_index(drop=True)
    fr = unify_domains(Frame.from_pandas(part), c)
    res = {}
    gb = M.group_by(fr, [0], [("sum", 2, "rm"), ("mean", 3, "all"), ("nrow", 0, "all"), ("max", 2, "rm"),
                              ("median", 3, "all")], c)
    res["gb"] = gb.to_pandas().to_dict("list") if comm.rank == 0 else None
    q = M.quantile(Frame([fr.vec("x"), fr.vec("y")]), [0.0, 0.1, 0.5, 0.99, 1.0], c)
    res["q"] = q.to_pandas().to_dict("list")
    res["cumsum"] = M.cumulative(Frame([fr.vec("y")]), "cumsum", c).to_pandas()["y"].tolist()
    res["kfold"] = M.kfold_column(fr, 5, 42, c).to_pandas()["fold"].tolist()
    res["which"] = M.which(Frame([fr.vec("h")]), c).to_pandas()["which"].tolist()
    sc = M.scale(Frame([fr.vec("y")]), True, True, c).to_pandas()["y"].tolist()
    res["scale"] = sc
    tab = M.table(Frame([fr.vec("g"), fr.vec("h")]), c)
    res["table"] = tab.to_pandas().to_dict("list") if comm.rank == 0 else None
    srt = M.sort(fr, [3, 2], [False, True], c)
    res["sort"] = srt.to_pandas()[["y", "x"]].fillna(-999).values.tolist() if comm.rank == 0 else None
    imp, fill = M.impute(fr, 2, "median", c)
    res["impute"] = fill
    with open(out_path, "w") as f:
        json.dump(res, f)
    comm.barrier()


if __name__ == "__main__":
    main()
