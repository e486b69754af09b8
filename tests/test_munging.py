"""Frame munging (Rapids ops behind h2o-py H2OFrame methods) vs pandas /
NumPy, on one process and on a 2-rank gloo world where every rank holds a
row shard (results must equal the single-process ones)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pandas as pd
import pytest

from h2omx.api.rapids import evaluate
from h2omx.frame import Frame
from h2omx.frame.frame import DKV

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from _munging_worker import data  # noqa: E402


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, tmp_path):
    port = _port()
    procs, outs = [], []
    for r in range(world):
        out = tmp_path / f"res{world}_{r}.json"
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_munging_worker.py"), str(out)], env=env))
        outs.append(out)
    for p in procs:
        assert p.wait(timeout=240) == 0
    return [json.load(open(o)) for o in outs]


@pytest.fixture(scope="module")
def results(tmp_path_factory):
    t = tmp_path_factory.mktemp("munge")
    return _run(1, t)[0], _run(2, t)


def test_group_by_and_table(results):
    single, multi = results
    df = data()
    ref = df.groupby("g", observed=True).agg(sx=("x", "sum"), my=("y", "mean"), n=("y", "size"), mx=("x", "max"),
                                             md=("y", "median"))
    for res in (single["gb"], multi[0]["gb"]):
        np.testing.assert_allclose(res["sum_x"], ref["sx"], rtol=1e-4)
        np.testing.assert_allclose(res["mean_y"], ref["my"], rtol=1e-5)
        assert res["nrow"] == ref["n"].tolist() and res["g"] == ["a", "b", "c"]
        np.testing.assert_allclose(res["max_x"], ref["mx"], rtol=1e-5)
        np.testing.assert_allclose(res["median_y"], ref["md"])
    tref = df.groupby(["g", "h"], observed=True).size()
    for res in (single["table"], multi[0]["table"]):
        assert res["Count"] == tref.tolist()


def test_quantile_cumsum_kfold_scale_which(results):
    single, multi = results
    df = data()
    for col in ("x", "y"):
        ref = np.nanquantile(df[col].values, [0.0, 0.1, 0.5, 0.99, 1.0])
        np.testing.assert_allclose(single["q"][f"{col}Quantiles"], ref, rtol=1e-5)
        np.testing.assert_allclose(multi[0]["q"][f"{col}Quantiles"], ref, rtol=1e-5)
        assert multi[1]["q"] == multi[0]["q"]
    cs = multi[0]["cumsum"] + multi[1]["cumsum"]
    np.testing.assert_allclose(cs, np.cumsum(df["y"].values), rtol=1e-6)
    np.testing.assert_allclose(single["cumsum"], np.cumsum(df["y"].values), rtol=1e-6)
    assert single["kfold"] == multi[0]["kfold"] + multi[1]["kfold"]
    assert sorted(set(single["kfold"])) == [0, 1, 2, 3, 4]
    np.testing.assert_allclose(multi[0]["scale"] + multi[1]["scale"], single["scale"], atol=1e-5)
    np.testing.assert_allclose(single["scale"], (df.y - df.y.mean()) / df.y.std(), atol=1e-5)
    assert single["which"] == multi[0]["which"] + multi[1]["which"]
    assert single["which"] == np.nonzero(df["h"].values)[0].tolist()
    assert single["impute"] == multi[0]["impute"]
    np.testing.assert_allclose(single["impute"][0], df["x"].median(), rtol=1e-6)


def test_sort(results):
    single, multi = results
    df = data()
    ref = df.sort_values(["y", "x"], ascending=[False, True], na_position="first", kind="stable")
    for res in (single["sort"], multi[0]["sort"]):
        got = np.array(res)
        assert got[:, 0].tolist() == ref["y"].tolist()


def test_rapids_expressions():
    df = pd.DataFrame({"k": pd.Categorical(["u", "v", "u", "w"]), "a": [1.0, np.nan, 3.0, 4.0],
                       "b": [10.0, 20.0, 30.0, 40.0]})
    fr = Frame.from_pandas(df, key="mfr")
    DKV.put("mfr", fr)
    r = evaluate('(tmp= t1 (ifelse (> (cols_py mfr "b") 15) 1 0))')
    assert DKV.get("t1").to_pandas().iloc[:, 0].tolist() == [0.0, 1.0, 1.0, 1.0]
    evaluate("(tmp= t2 (na.omit mfr))")
    assert DKV.get("t2").nrows == 3
    evaluate('(tmp= t3 (cut (cols_py mfr "b") [0 15 35 50] ["lo" "mid" "hi"] FALSE TRUE 3))')
    assert DKV.get("t3").to_pandas().iloc[:, 0].tolist() == ["lo", "mid", "mid", "hi"]
    evaluate('(tmp= t4 (GB mfr [0] "sum" 2 "all" "nrow" 0 "all"))')
    g = DKV.get("t4").to_pandas()
    assert g["sum_b"].tolist() == [40.0, 20.0, 40.0] and g["nrow"].tolist() == [2, 1, 1]
    evaluate("(tmp= t5 (sort mfr [2] [0]))")
    assert DKV.get("t5").to_pandas()["b"].tolist() == [40.0, 30.0, 20.0, 10.0]
    other = Frame.from_pandas(pd.DataFrame({"k": pd.Categorical(["u", "w"]), "c": [7.0, 9.0]}), key="ofr")
    DKV.put("ofr", other)
    evaluate("(tmp= t6 (merge mfr ofr TRUE FALSE [0] [0] 'auto'))")
    m = DKV.get("t6").to_pandas()
    assert len(m) == 4 and m.loc[m.k == "w", "c"].tolist() == [9.0]
    assert evaluate("(naCnt mfr)")["scalar"] == [0.0, 1.0, 0.0]
    evaluate('(h2o.impute mfr 1 "mean" "interpolate" [] _ [])')
    assert abs(DKV.get("mfr").to_pandas()["a"][1] - 8.0 / 3) < 1e-5
    q = evaluate('(tmp= t7 (quantile (cols_py mfr "b") [0.5] "interpolate" _))')
    assert DKV.get("t7").to_pandas()["bQuantiles"].tolist() == [25.0]
    evaluate('(tmp= t8 (relevel (cols_py mfr "k") "w"))')
    assert DKV.get("t8").vecs[0].domain == ["w", "u", "v"]
    evaluate("(tmp= t9 (unique (cols_py mfr [0]) FALSE))")
    assert DKV.get("t9").to_pandas()["k"].tolist() == ["u", "v", "w"]
