"""make_metrics, permutation importance and segment models."""
import numpy as np
import pandas as pd
import torch

from h2omx.frame import Frame
from h2omx.frame.frame import ENUM, Vec
from h2omx.models import H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator
from h2omx.tools import make_metrics, permutation_importance, train_segments


def _df(n=2000, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 3))
    df = pd.DataFrame(X, columns=list("abc"))
    df["seg"] = pd.Categorical(rng.choice(["s1", "s2", "s3"], n))
    df["y"] = pd.Categorical(np.where(X[:, 0] + 0.2 * rng.normal(size=n) > 0, "1", "0"))
    df["r"] = 2 * X[:, 0] + rng.normal(size=n)
    return df


def test_make_metrics_matches_model_metrics():
    fr = Frame.from_pandas(_df())
    m = H2OGradientBoostingEstimator(ntrees=5, seed=1).train(x=list("abc"), y="y", training_frame=fr)
    P = m.predict(fr)
    mm = make_metrics(Frame([P.vecs[-1]]), Frame([fr.vec("y")]))
    assert abs(mm["AUC"] - m.training_metrics["AUC"]) < 1e-9
    g = H2OGeneralizedLinearEstimator().train(x=list("abc"), y="r", training_frame=fr)
    rm = make_metrics(g.predict(fr), Frame([fr.vec("r")]))
    assert abs(rm["RMSE"] - g.training_metrics["RMSE"]) < 1e-6
    # multinomial from explicit probability columns
    probs = torch.tensor([[0.7, 0.2, 0.1], [0.1, 0.8, 0.1], [0.2, 0.2, 0.6]])
    pf = Frame([Vec(d, probs[:, k], "real") for k, d in enumerate(["x", "y", "z"])])
    af = Frame([Vec("t", torch.tensor([0, 1, 2], dtype=torch.int32), ENUM, ["x", "y", "z"])])
    mmn = make_metrics(pf, af)
    assert mmn["model_category"] == "Multinomial" and mmn["logloss"] > 0


def test_permutation_importance_ranks_signal_first():
    fr = Frame.from_pandas(_df())
    m = H2OGradientBoostingEstimator(ntrees=10, seed=1).train(x=list("abc"), y="y", training_frame=fr)
    pi = m.permutation_importance(fr, metric="AUC", seed=3)
    assert pi[0]["variable"] == "a" and pi[0]["relative_importance"] > 0.2
    assert abs(pi[0]["scaled_importance"] - 1.0) < 1e-12
    ll = permutation_importance(m, fr, n_repeats=2)
    assert ll[0]["variable"] == "a"


def test_train_segments():
    fr = Frame.from_pandas(_df())
    out = train_segments(H2OGradientBoostingEstimator, dict(ntrees=3, seed=1), "seg", x=list("abc"), y="y",
                         training_frame=fr, segment_models_id="segs")
    rows = out["segments"]
    assert [r["seg"] for r in rows] == ["s1", "s2", "s3"]
    assert all(r["status"] == "SUCCEEDED" for r in rows)
    assert sum(r["rows"] for r in rows) == fr.nrows
