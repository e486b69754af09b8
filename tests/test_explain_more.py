"""Leaf node assignment, staged probabilities, feature frequencies, linear
SHAP for GLM, ICE, fairness metrics, explain() bundle; REST prediction flags."""
import numpy as np
import pandas as pd
import pytest
import torch

from h2omx.explain_more import model_correlation, varimp_heatmap
from h2omx.frame import Frame
from h2omx.models import (H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator,
                          H2ORandomForestEstimator)


def _df(n=1500, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 3))
    df = pd.DataFrame(X, columns=list("abc"))
    df.loc[::11, "c"] = np.nan
    df["grp"] = pd.Categorical(rng.choice(["A", "B"], n, p=[0.7, 0.3]))
    logit = X[:, 0] - X[:, 1] + 0.5 * (df.grp == "B")
    df["y"] = pd.Categorical(np.where(rng.random(n) < 1 / (1 + np.exp(-logit)), "1", "0"))
    return df


@pytest.fixture(scope="module")
def gbm():
    fr = Frame.from_pandas(_df())
    m = H2OGradientBoostingEstimator(ntrees=6, max_depth=3, seed=1).train(x=["a", "b", "c", "grp"], y="y",
                                                                          training_frame=fr)
    return m, fr


def test_leaf_assignment_consistent_with_scores(gbm):
    m, fr = gbm
    paths = m.predict_leaf_node_assignment(fr, "Path")
    ids = m.predict_leaf_node_assignment(fr, "Node_ID")
    assert paths.names == [f"T{t}.C1" for t in range(1, 7)]
    ens = m.ens
    X = fr.feature_matrix(m.x) if not hasattr(m, "_matrix") else m._matrix(fr)
    margin = np.full(fr.nrows, float(ens.init_f[0]))
    for t in range(6):
        nid = ids.vec(f"T{t + 1}.C1").data.long().numpy()
        margin += ens.trees[t]["value"][nid]
        lens = {len(p) for p in paths.vec(f"T{t + 1}.C1").domain}
        assert max(lens) <= 3 and set("".join(paths.vec(f"T{t + 1}.C1").domain)) <= {"L", "R"}
    np.testing.assert_allclose(margin, ens.raw_margin(X)[0].numpy(), rtol=1e-5, atol=1e-5)


def test_staged_proba_ends_at_prediction(gbm):
    m, fr = gbm
    st = m.staged_predict_proba(fr)
    assert st.names == [f"T{t}.C1" for t in range(1, 7)]
    np.testing.assert_allclose(st.vec("T6.C1").data.numpy(), m.predict_raw(fr)[1].numpy(), atol=1e-5)


def test_feature_frequencies(gbm):
    m, fr = gbm
    ff = m.feature_frequencies(fr)
    tot = sum(ff.vec(c).data for c in m.x)
    assert ff.names == m.x
    assert float(tot.max()) <= 6 * 3 and float(tot.min()) >= 6


def test_drf_staged_and_leaves():
    fr = Frame.from_pandas(_df())
    m = H2ORandomForestEstimator(ntrees=4, max_depth=4, seed=1).train(x=["a", "b", "c"], y="y", training_frame=fr)
    st = m.staged_predict_proba(fr)
    np.testing.assert_allclose(st.vec("T4.C1").data.numpy(), m.predict_raw(fr)[1].numpy(), atol=1e-5)


def test_glm_linear_shap_sums_to_link():
    fr = Frame.from_pandas(_df())
    m = H2OGeneralizedLinearEstimator(family="binomial", lambda_=0.0).train(x=["a", "b", "c", "grp"], y="y",
                                                                            training_frame=fr)
    sh = m.predict_contributions(fr)
    assert sh.names == ["a", "b", "c", "grp", "BiasTerm"]
    tot = sum(sh.vec(c).data.double() for c in sh.names)
    p1 = m.predict_raw(fr)[1].double()
    np.testing.assert_allclose(torch.sigmoid(tot).numpy(), p1.numpy(), atol=1e-5)


def test_ice_mean_is_partial_dependence(gbm):
    m, fr = gbm
    ic = m.ice(fr, "a", nbins=5)
    sub = fr.rows(torch.arange(1000))
    pd_ = m.partial_dependence(sub, ["a"], nbins=5)[0]["data"]
    np.testing.assert_allclose(ic["mean"], [r["mean_response"] for r in pd_], atol=1e-5)
    assert np.array(ic["curves"]).shape == (1000, 5)


def test_fairness_metrics(gbm):
    m, fr = gbm
    fm = m.fairness_metrics(fr, ["grp"], reference=["A"], favorable_class="1")
    rows = {r["grp"]: r for r in fm["overview"]}
    assert set(rows) == {"A", "B"}
    assert rows["A"]["AIR_selectedRatio"] == pytest.approx(1.0)
    assert rows["B"]["AIR_selectedRatio"] > 1.0       # group B is favoured by construction
    assert abs(rows["A"]["relativeSize"] + rows["B"]["relativeSize"] - 1) < 1e-9
    assert 0 <= rows["B"]["p.value"] <= 1


def test_explain_bundle(gbm):
    m, fr = gbm
    glm = H2OGeneralizedLinearEstimator(family="binomial").train(x=["a", "b", "c", "grp"], y="y", training_frame=fr)
    ex = m.explain(fr, top_n_features=2)
    assert len(ex["pdp"]) == 2 and "shap_summary" in ex
    mc = model_correlation([m, glm], fr)
    assert mc["correlation"][0][1] > 0.8
    vh = varimp_heatmap([m, glm])
    assert len(vh["model_ids"]) == 2


def test_rest_prediction_flags():
    import socket

    from h2omx.api.server import H2OApi, serve
    from h2omx.client import H2OConnection
    from h2omx.frame.frame import DKV
    from h2omx.runtime.cluster import ClusterConfig, form_cluster

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    srv = serve(H2OApi(form_cluster(ClusterConfig(), device="cpu")), "127.0.0.1", port)
    try:
        c = H2OConnection(f"http://127.0.0.1:{port}")
        c.connect()
        fr = Frame.from_pandas(_df(400), key="ex.hex")
        DKV.put("ex.hex", fr)
        H2OGradientBoostingEstimator(ntrees=3, max_depth=2, seed=1, model_id="exg").train(
            x=["a", "b"], y="y", training_frame=fr)
        for flag, ncol in (("leaf_node_assignment", 3), ("predict_staged_proba", 3), ("feature_frequencies", 2),
                           ("predict_contributions", 3)):
            r = c.request("POST /3/Predictions/models/exg/frames/ex.hex", {flag: "true", "predictions_frame": flag})
            f = c.request(f"GET /3/Frames/{r['predictions_frame']['name']}")["frames"][0]
            assert len(f["columns"]) == ncol, flag
    finally:
        srv.shutdown()


@pytest.mark.gpu
def test_explain_more_gpu(cuda_dev):
    fr = Frame.from_pandas(_df(), device=cuda_dev)
    m = H2OGradientBoostingEstimator(ntrees=5, max_depth=3, seed=1).train(x=["a", "b", "c", "grp"], y="y",
                                                                          training_frame=fr)
    st = m.staged_predict_proba(fr)
    np.testing.assert_allclose(st.vec("T5.C1").data.cpu().numpy(), m.predict_raw(fr)[1].cpu().numpy(), atol=1e-5)
    ids = m.predict_leaf_node_assignment(fr, "Node_ID")
    assert ids.vec("T1.C1").data.is_cuda
    glm = H2OGeneralizedLinearEstimator(family="binomial", lambda_=0.0).train(x=["a", "b", "c", "grp"], y="y",
                                                                              training_frame=fr)
    sh = glm.predict_contributions(fr)
    tot = sum(sh.vec(c).data.double() for c in sh.names)
    np.testing.assert_allclose(torch.sigmoid(tot).cpu().numpy(), glm.predict_raw(fr)[1].double().cpu().numpy(),
                               atol=1e-4)
