"""REST frame tools and diagnostics: /3/CreateFrame, /3/Interaction,
/3/MissingInserter, /3/Frames/{id}/export, /3/Word2VecSynonyms|Transform,
/3/NetworkTest, /3/Typeahead/files, /3/GarbageCollect, /3/JStack,
/3/ModelMetrics, generic MOJO import.  (Interaction on 2 gloo ranks: test_algos_multirank.)"""
import socket

import numpy as np
import pandas as pd
import pytest
import torch

from h2omx.api.server import H2OApi, serve
from h2omx.client import H2OConnection
from h2omx.frame import Frame
from h2omx.frame.frame import DKV
from h2omx.frame.tools import create_frame, insert_missing_values, interaction
from h2omx.runtime.cluster import ClusterConfig, form_cluster


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def conn():
    cl = form_cluster(ClusterConfig(), device="cpu")
    api = H2OApi(cl)
    port = _free_port()
    srv = serve(api, "127.0.0.1", port)
    c = H2OConnection(f"http://127.0.0.1:{port}")
    c.connect()
    yield c
    srv.shutdown()
    DKV.clear()


def test_create_frame_mix():
    fr = create_frame(rows=2000, cols=10, categorical_fraction=0.3, integer_fraction=0.2, binary_fraction=0.1,
                      missing_fraction=0.05, has_response=True, response_factors=3, seed=7)
    assert fr.nrows == 2000 and fr.ncols == 11 and fr.names[0] == "response"
    kinds = [v.vtype for v in fr.vecs[1:]]
    assert kinds.count("enum") == 3
    na = np.mean([float(torch.isnan(v.as_float()).float().mean()) for v in fr.vecs[1:]])
    assert 0.03 < na < 0.07
    again = create_frame(rows=2000, cols=10, categorical_fraction=0.3, integer_fraction=0.2, binary_fraction=0.1,
                         missing_fraction=0.05, has_response=True, response_factors=3, seed=7)
    assert again.to_pandas().equals(fr.to_pandas())


def test_interaction_levels():
    df = pd.DataFrame({"a": pd.Categorical(["x", "y", "x", "y", "x", None]),
                       "b": pd.Categorical(["p", "p", "q", "q", "p", "q"])})
    fr = Frame.from_pandas(df)
    out = interaction(fr, ["a", "b"])
    assert out.names == ["a_b"]
    vals = out.to_pandas()["a_b"].tolist()
    assert vals[:5] == ["x_p", "y_p", "x_q", "y_q", "x_p"] and pd.isna(vals[5])
    top = interaction(fr, ["a", "b"], max_factors=1)
    assert top.vecs[0].domain == ["x_p", "other"]
    pw = interaction(Frame.from_pandas(df.assign(c=pd.Categorical(list("uuvvuv")))), ["a", "b", "c"], pairwise=True)
    assert pw.names == ["a_b", "a_c", "b_c"]


def test_insert_missing():
    fr = Frame.from_pandas(pd.DataFrame({"a": np.arange(10000.0), "g": pd.Categorical(["u", "v"] * 5000)}))
    insert_missing_values(fr, 0.2, seed=3)
    assert abs(float(torch.isnan(fr.vec("a").data).float().mean()) - 0.2) < 0.02
    assert abs(float((fr.vec("g").data < 0).float().mean()) - 0.2) < 0.02


def test_rest_frame_tools(conn, tmp_path):
    r = conn.request("POST /3/CreateFrame", {"dest": "cf.hex", "rows": 500, "cols": 6, "categorical_fraction": 0.5,
                                             "factors": 4, "missing_fraction": 0.0, "seed": 3})
    assert r["dest"]["name"] == "cf.hex"
    fr = conn.request("GET /3/Frames/cf.hex")["frames"][0]
    assert fr["rows"] == 500 and len(fr["columns"]) == 6
    cats = [c["label"] for c in fr["columns"] if c["type"] == "enum"]
    r = conn.request("POST /3/Interaction", {"source_frame": "cf.hex", "factor_columns": cats[:2], "dest": "ia.hex"})
    ia = conn.request("GET /3/Frames/ia.hex")["frames"][0]
    assert ia["columns"][0]["label"] == "_".join(cats[:2])
    conn.request("POST /3/MissingInserter", {"dataset": "cf.hex", "fraction": 0.3, "seed": 1})
    fr = conn.request("GET /3/Frames/cf.hex")["frames"][0]
    assert all(c["missing_count"] > 50 for c in fr["columns"])
    path = str(tmp_path / "out" / "cf.csv")
    conn.request("POST /3/Frames/cf.hex/export", {"path": path})
    assert len(pd.read_csv(path)) == 500
    ta = conn.request("GET /3/Typeahead/files", {"src": str(tmp_path / "out" / "c")})
    assert ta["matches"] == [path]


def test_rest_diagnostics(conn):
    nt = conn.request("GET /3/NetworkTest")
    assert nt["world_size"] == 1 and len(nt["results"]) == 4
    conn.request("POST /3/GarbageCollect")
    js = conn.request("GET /3/JStack")
    assert js["traces"][0]["thread_traces"]
    assert "model_metrics" in conn.request("GET /3/ModelMetrics")


def test_rest_word2vec(conn):
    from h2omx.models import H2OWord2vecEstimator

    rng = np.random.default_rng(0)
    toks = []
    for _ in range(400):
        toks += list(rng.choice([f"w{i}" for i in range(8)], size=5)) + [None]
    fr = Frame.from_pandas(pd.DataFrame({"w": toks}), key="words.hex")
    DKV.put("words.hex", fr)
    m = H2OWord2vecEstimator(vec_size=6, epochs=1, min_word_freq=1, seed=1, model_id="w2v").train(training_frame=fr)
    s = conn.request("GET /3/Word2VecSynonyms", {"model": "w2v", "word": "w1", "count": 3})
    assert len(s["synonyms"]) == 3 and len(s["scores"]) == 3
    t = conn.request("GET /3/Word2VecTransform", {"model": "w2v", "words_frame": "words.hex",
                                                  "aggregate_method": "AVERAGE"})
    vf = conn.request(f"GET /3/Frames/{t['vectors_frame']['name']}")["frames"][0]
    assert vf["rows"] == 400 and len(vf["columns"]) == 6
    assert m.model_id == "w2v"


def test_rest_generic_import(conn, tmp_path):
    from h2omx.models import H2OGenericEstimator, H2OGradientBoostingEstimator

    rng = np.random.default_rng(1)
    df = pd.DataFrame(rng.normal(size=(600, 3)), columns=list("abc"))
    df["y"] = pd.Categorical(np.where(df.a + df.b > 0, "t", "f"))
    fr = Frame.from_pandas(df, key="gen.hex")
    DKV.put("gen.hex", fr)
    m = H2OGradientBoostingEstimator(ntrees=5, max_depth=3, seed=1).train(y="y", training_frame=fr)
    path = m.download_mojo(str(tmp_path))
    g = H2OGenericEstimator.from_file(path)
    np.testing.assert_allclose(g.predict_raw(fr).numpy(), m.predict_raw(fr).numpy(), rtol=1e-5, atol=1e-6)
    r = conn.request("POST /3/ModelBuilders/generic", {"path": path, "model_id": "imported_gbm"})
    assert r["job"]["status"] == "DONE"
    mj = conn.request("GET /3/Models/imported_gbm")["models"][0]
    assert mj["algo"] == "generic"
    pr = conn.request("POST /3/Predictions/models/imported_gbm/frames/gen.hex")
    assert pr["model_metrics"][0]["AUC"] > 0.9


def test_rest_metrics_permutation_segments(conn):
    from h2omx.models import H2OGradientBoostingEstimator

    rng = np.random.default_rng(4)
    n = 900
    df = pd.DataFrame(rng.normal(size=(n, 3)), columns=list("abc"))
    df["seg"] = pd.Categorical(rng.choice(["u", "v"], n))
    df["y"] = pd.Categorical(np.where(df.a > 0, "t", "f"))
    fr = Frame.from_pandas(df, key="pm.hex")
    DKV.put("pm.hex", fr)
    m = H2OGradientBoostingEstimator(ntrees=5, seed=1, model_id="pm_gbm").train(x=list("abc"), y="y",
                                                                                 training_frame=fr)
    pv = conn.request("POST /3/PermutationVarImp", {"model_id": "pm_gbm", "frame_id": "pm.hex", "metric": "AUC"})
    assert pv["permutation_varimp"]["data"][0][0] == "a"
    pred = m.predict(fr)
    DKV.put("pm_pred.hex", Frame([pred.vecs[-1]], key="pm_pred.hex"))
    DKV.put("pm_act.hex", Frame([fr.vec("y")], key="pm_act.hex"))
    mm = conn.request("POST /3/ModelMetrics/predictions_frame/pm_pred.hex/actuals_frame/pm_act.hex")
    assert abs(mm["model_metrics"]["AUC"] - m.training_metrics["AUC"]) < 1e-9
    r = conn.request("POST /99/SegmentModelsBuilders/gbm", {"training_frame": "pm.hex", "response_column": "y",
                                                            "segment_columns": "[seg]", "ntrees": 3,
                                                            "segment_models_id": "pm_segs"})
    assert r["job"]["status"] == "DONE"
    segs = conn.request("GET /3/SegmentModels/pm_segs")["segments"]
    assert [s["seg"] for s in segs] == ["u", "v"] and all(s["status"] == "SUCCEEDED" for s in segs)
