"""balance_classes / class_sampling_factors / max_after_balance_size for GBM
and DRF (H2O semantics: the class mix is rebalanced for training and the
predicted probabilities are mapped back with correctProbabilities)."""
import numpy as np
import pandas as pd
import torch

from h2omx.frame import Frame
from h2omx.models import H2OGradientBoostingEstimator, H2ORandomForestEstimator
from h2omx.models.tree_models import _balance_weights, correct_probabilities
from h2omx.mojo import import_mojo


def _imbalanced(n=4000, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, 3))
    eta = -3.0 + 1.5 * x[:, 0]
    y = rng.random(n) < 1 / (1 + np.exp(-eta))
    df = pd.DataFrame(x, columns=["a", "b", "c"])
    df["y"] = pd.Categorical(np.where(y, "pos", "neg"), categories=["neg", "pos"])
    return df


def test_balance_weights_follow_h2o_sampling_rules():
    y = torch.tensor([0.0] * 90 + [1.0] * 10)
    w, (prior, modelled) = _balance_weights(y, None, 2, {"max_after_balance_size": 5.0})
    np.testing.assert_allclose(prior, [0.9, 0.1])
    np.testing.assert_allclose(modelled, [0.5, 0.5])
    assert float(w[:90].sum()) == float(w[90:].sum()) == 90.0
    # cap: at most max_after_balance_size x N rows after balancing
    w, _ = _balance_weights(y, None, 2, {"max_after_balance_size": 1.0})
    assert abs(float(w.sum()) - 100.0) < 1e-4
    # explicit per-class factors
    w, (_, modelled) = _balance_weights(y, None, 2, {"class_sampling_factors": [1.0, 3.0],
                                                     "max_after_balance_size": 5.0})
    np.testing.assert_allclose(modelled, [90 / 120, 30 / 120])
    P = torch.tensor([[0.5], [0.5]])
    np.testing.assert_allclose(correct_probabilities(P, [0.9, 0.1], [0.5, 0.5]).numpy().ravel(), [0.9, 0.1])


def test_gbm_and_drf_balance_classes(tmp_path):
    df = _imbalanced()
    fr = Frame.from_pandas(df)
    for est in (H2OGradientBoostingEstimator(ntrees=20, max_depth=3, seed=1),
                H2ORandomForestEstimator(ntrees=10, max_depth=6, seed=1)):
        plain = type(est)(**{k: est.params[k] for k in ("ntrees", "max_depth", "seed")}).train(
            x=["a", "b", "c"], y="y", training_frame=fr)
        est.params["balance_classes"] = True
        bal = est.train(x=["a", "b", "c"], y="y", training_frame=fr)
        assert bal.class_dist is not None
        p_bal = bal.predict(fr).to_pandas()["pos"].to_numpy()
        p_plain = plain.predict(fr).to_pandas()["pos"].to_numpy()
        # corrected probabilities stay calibrated to the original prior
        rate = (df.y == "pos").mean()
        assert abs(p_bal.mean() - rate) < 0.5 * rate
        assert bal.training_metrics["AUC"] > 0.75 and plain.training_metrics["AUC"] > 0.75
        assert not np.allclose(p_bal, p_plain)
        g = import_mojo(bal.download_mojo(str(tmp_path)))
        np.testing.assert_allclose(g.predict(fr).to_pandas()["pos"].to_numpy(), p_bal, rtol=1e-5, atol=1e-6)
