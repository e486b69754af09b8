"""REST API tests: a one-node cluster serves the H2O routes over HTTP and
h2omx.client drives the h2o-py workflow against it (connect, import /
upload, parse, frames, model builders, jobs, predictions, metrics, MOJO,
Rapids, AutoML, DKV removal, error shapes)."""
import io
import socket
import zipfile

import numpy as np
import pandas as pd
import pytest

from h2omx.api.server import H2OApi, serve
from h2omx.client import H2OConnection, H2OResponseError
from h2omx.frame.frame import DKV
from h2omx.runtime.cluster import ClusterConfig, form_cluster


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def csv_path(tmp_path_factory):
    rng = np.random.default_rng(0)
    n = 3000
    df = pd.DataFrame({"a": rng.normal(size=n), "b": rng.normal(size=n), "c": rng.choice(["x", "y", "z"], n)})
    logit = df.a - df.b + (df.c == "x") * 1.0
    df["label"] = np.where(rng.random(n) < 1 / (1 + np.exp(-logit)), "yes", "no")
    p = tmp_path_factory.mktemp("data") / "train.csv"
    df.to_csv(p, index=False)
    return str(p)


@pytest.fixture(scope="module")
def conn(csv_path):
    cl = form_cluster(ClusterConfig(), device="cpu")
    api = H2OApi(cl)
    port = _free_port()
    srv = serve(api, "127.0.0.1", port)
    c = H2OConnection(f"http://127.0.0.1:{port}")
    # every test may run alone (-k, xdist): the shared training frame is
    # imported here rather than by test_import_parse_frame
    c.import_file(csv_path, destination_frame="train.hex")
    yield c
    srv.shutdown()
    DKV.clear()


def test_cloud_and_session(conn):
    cloud = conn.connect()
    assert cloud["cloud_size"] == 1 and cloud["cloud_healthy"] and cloud["consensus"]
    assert cloud["version"].count(".") == 3
    assert conn.session_key.startswith("_sid_")
    about = conn.request("GET /3/About")
    assert any(e["name"] == "Build project version" for e in about["entries"])


def test_import_parse_frame(conn, csv_path):
    key = conn.import_file(csv_path, destination_frame="train.hex")
    assert key == "train.hex"
    fr = conn.frame(key, rows=5)
    assert fr["rows"] == 3000
    labels = [c["label"] for c in fr["columns"]]
    assert labels == ["a", "b", "c", "label"]
    c = fr["columns"][2]
    assert c["type"] == "enum" and c["domain"] == ["x", "y", "z"]
    assert len(fr["columns"][0]["data"]) == 5
    assert abs(fr["columns"][0]["mean"]) < 0.1
    lst = conn.request("GET /3/Frames")
    assert any(f["frame_id"]["name"] == "train.hex" for f in lst["frames"])


def test_upload_file(conn, csv_path):
    key = conn.upload_file(csv_path, destination_frame="uploaded.hex")
    assert conn.frame(key)["rows"] == 3000


@pytest.mark.parametrize("algo,params", [("gbm", {"ntrees": 10, "max_depth": 3, "seed": 1}),
                                         ("glm", {"family": "binomial", "lambda": 0}),
                                         ("drf", {"ntrees": 5, "seed": 1}),
                                         ("deeplearning", {"hidden": [16], "epochs": 10, "seed": 1}),
                                         ("xgboost", {"ntrees": 5, "max_depth": 3})])
def test_build_predict_metrics(conn, algo, params):
    m = conn.train(algo, "train.hex", y="label", **params)
    tm = m["output"]["training_metrics"]
    assert m["algo"] == algo
    assert tm["__meta"]["schema_type"] == "ModelMetricsBinomial"
    assert tm["AUC"] > 0.7
    assert tm["cm"]["table"]["columns"][1]["name"] == "no"
    pred = conn.predict(m["model_id"]["name"], "train.hex")
    pf = conn.frame(pred, rows=3)
    assert [c["label"] for c in pf["columns"]] == ["predict", "no", "yes"]
    mm = conn.model_performance(m["model_id"]["name"], "train.hex")
    if algo == "drf":
        # DRF training metrics are out-of-bag (H2O): below the in-sample score
        assert "out-of-bag" in str(tm.get("description", "")).lower() and mm["AUC"] > tm["AUC"]
    else:
        assert abs(mm["AUC"] - tm["AUC"]) < 1e-9
    vi = m["output"]["variable_importances"]
    if vi is not None:
        assert vi["columns"][0]["name"] == "variable"


def test_unknown_param_is_warning_and_ignored_columns(conn):
    m = conn.train("gbm", "train.hex", y="label", x=["a", "b"], ntrees=3, histogram_type="UniformAdaptive",
                   build_tree_one_node="true")
    names = m["output"]["names"]
    assert names == ["a", "b", "label"]


def test_histogram_deviation_warnings_over_rest(conn):
    """GBM's AUTO histograms are H2O's per-node UniformAdaptive; what still
    deviates reaches the REST caller as model warnings (H2O's output.warnings)."""
    m = conn.train("gbm", "train.hex", y="label", ntrees=2, max_depth=3, seed=1)
    assert any("fine quantile bins" in w for w in (m["output"].get("warnings") or []))
    r = conn.train("gbm", "train.hex", y="label", ntrees=2, max_depth=3, seed=1, histogram_type="UniformRobust")
    assert any("one global grid" in w for w in r["output"]["warnings"])
    q = conn.train("gbm", "train.hex", y="label", ntrees=2, max_depth=3, seed=1, histogram_type="QuantilesGlobal")
    assert not q["output"].get("warnings")


def test_kmeans_rest_and_mojo_roundtrip(conn):
    from h2omx.frame.frame import DKV as dkv
    from h2omx.mojo import GenericModel

    m = conn.train("kmeans", "train.hex", x=["a", "b", "c"], k=3, seed=2)
    assert m["output"]["model_category"] == "Clustering"
    data = conn.download_mojo(m["model_id"]["name"])
    z = zipfile.ZipFile(io.BytesIO(data))
    assert "model.ini" in z.namelist()
    g = GenericModel(data)
    fr = dkv.get("train.hex")
    orig = dkv.get(m["model_id"]["name"])
    assert (g.predict_raw(fr) == orig.predict_raw(fr)).all()


def test_rapids_split_and_slice(conn):
    r = conn.rapids('(tmp= rnd_1 (h2o.runif train.hex 42))')
    assert r["num_rows"] == 3000
    r = conn.rapids('(tmp= part_a (rows train.hex (< rnd_1 0.75)))')
    r2 = conn.rapids('(tmp= part_b (rows train.hex (>= rnd_1 0.75)))')
    assert r["num_rows"] + r2["num_rows"] == 3000 and 2000 < r["num_rows"] < 2500
    r = conn.rapids('(cols_py train.hex ["a" "c"])')
    assert r["num_cols"] == 2
    s = conn.rapids("(mean (cols_py train.hex 0) true)")
    assert abs(s["scalar"]) < 0.1
    r = conn.rapids('(tmp= t2 (:= train.hex (as.factor (cols_py train.hex "a")) 0 []))')
    assert r["num_cols"] == 4
    conn.rapids("(rm rnd_1)")


def test_automl_rest(conn):
    res = conn.automl("train.hex", "label", max_models=3, nfolds=3, project_name="aml_test",
                      build_models={"include_algos": ["GLM", "GBM", "DRF", "StackedEnsemble"]})
    lb = res["leaderboard_table"]
    ids = lb["data"][0]
    assert len(ids) >= 3
    assert any(i.startswith("StackedEnsemble") for i in ids)
    aucs = lb["data"][[c["name"] for c in lb["columns"]].index("auc")]
    assert aucs == sorted(aucs, reverse=True)


def test_grid_rest(conn):
    g = conn.grid("gbm", "train.hex", {"max_depth": [2, 3], "learn_rate": [0.1, 0.3]}, y="label", ntrees=5,
                  grid_id="gbm_grid_rest", seed=1)
    assert len(g["model_ids"]) == 4 and g["hyper_names"] == ["max_depth", "learn_rate"]
    s = conn.get_grid("gbm_grid_rest", sort_by="auc", decreasing=True)
    names = [c["name"] for c in s["summary_table"]["columns"]]
    aucs = s["summary_table"]["data"][names.index("auc")]
    assert aucs == sorted(aucs, reverse=True)
    assert any(gr["grid_id"]["name"] == "gbm_grid_rest" for gr in conn.request("GET /99/Grids")["grids"])
    r = conn.grid("glm", "train.hex", {"alpha": [0.0, 0.5, 1.0]}, y="label", grid_id="glm_grid_rest",
                  search_criteria={"strategy": "RandomDiscrete", "max_models": 2, "seed": 3})
    assert len(r["model_ids"]) == 2


@pytest.mark.parametrize("algo,params", [("isolationforest", {"ntrees": 10, "seed": 1}),
                                         ("pca", {"k": 2, "transform": "STANDARDIZE"}),
                                         ("naivebayes", {"laplace": 1.0})])
def test_more_algorithms_rest(conn, algo, params):
    y = "label" if algo == "naivebayes" else None
    m = conn.train(algo, "train.hex", y=y, **params)
    assert m["algo"] == algo
    pred = conn.predict(m["model_id"]["name"], "train.hex")
    fr = conn.frame(pred, rows=3)
    cols = [c["label"] for c in fr["columns"]]
    expect = {"isolationforest": ["predict", "mean_length"], "pca": ["PC1", "PC2"],
              "naivebayes": ["predict", "no", "yes"]}[algo]
    assert cols == expect


def test_contributions_and_partial_dependence_rest(conn):
    m = conn.train("gbm", "train.hex", y="label", ntrees=5, max_depth=3, seed=1)
    mid = m["model_id"]["name"]
    key = conn.predict_contributions(mid, "train.hex")
    fr = conn.frame(key, rows=5)
    assert [c["label"] for c in fr["columns"]] == ["a", "b", "c", "BiasTerm"]
    tabs = conn.partial_dependence(mid, "train.hex", cols=["a", "c"], nbins=5)
    assert len(tabs) == 2
    assert [c["name"] for c in tabs[0]["columns"]] == ["a", "mean_response", "stddev_response",
                                                        "std_error_mean_response"]
    assert len(tabs[0]["data"][0]) == 5 and tabs[1]["data"][0] == ["x", "y", "z"]


def test_errors_and_delete(conn, csv_path):
    with pytest.raises(H2OResponseError) as e:
        conn.request("GET /3/Frames/nope.hex")
    assert e.value.status == 404 and e.value.payload["__meta"]["schema_type"] == "H2OError"
    with pytest.raises(H2OResponseError) as e:
        conn.request("POST /3/ModelBuilders/gbm", {"training_frame": "missing.hex", "response_column": "y"})
    assert e.value.status == 404
    txt = conn.request("GET /metrics", raw=True).decode()
    assert "h2omx_models_built_total" in txt
    conn.upload_file(csv_path, destination_frame="uploaded.hex")   # may run alone (-k, xdist)
    conn.request("DELETE /3/Frames/uploaded.hex")
    assert not any(f["frame_id"]["name"] == "uploaded.hex" for f in conn.request("GET /3/Frames")["frames"])
    conn.remove_all()
    assert conn.request("GET /3/Frames")["frames"] == []
