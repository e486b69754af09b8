"""DRF out-of-bag training metrics (H2O reports DRF training metrics on the
out-of-bag rows of every tree): the engine accumulates, per row, the leaf
values of the trees whose bag left the row out; the metrics equal a
recomputation from the trees and the bag hash."""
import numpy as np
import pandas as pd
import pytest
import torch

from h2omx.frame import Frame
from h2omx.models import H2ORandomForestEstimator


def _frame(n, device, seed=3):
    rng = np.random.default_rng(seed)
    df = pd.DataFrame({f"x{i}": rng.normal(size=n) for i in range(6)})
    logit = df.x0 - 0.8 * df.x1 + 0.5 * df.x2 * df.x3
    df["y"] = pd.Categorical(np.where(rng.random(n) < 1 / (1 + np.exp(-logit)), "b", "a"))
    df["r"] = logit + rng.normal(size=n)
    df["c"] = pd.Categorical(np.digitize(logit + 0.3 * rng.normal(size=n), [-0.7, 0.6]).astype(str))
    return df, Frame.from_pandas(df, device=device)


def _manual_oob(model, df, sample_rate, seed):
    from h2omx.models.tree.boost import TreeEnsemble
    from h2omx.reference.tree import bag_weights

    ens = model.ens
    X = torch.from_numpy(df[model.x].to_numpy(np.float32).T.copy())
    n = len(df)
    K = ens.K
    s = np.zeros((K, n))
    cnt = np.zeros(n)
    for t in range(ens.ntrees):
        one = TreeEnsemble(ens.trees[t * K:(t + 1) * K], K, ens.dist, np.zeros(K), average=False)
        m = one.raw_margin(X, 1).cpu().numpy().astype(np.float64)
        oob = bag_weights(n, sample_rate, seed, t) == 0
        s[:, oob] += m[:, oob]
        cnt[oob] += 1
    return s, cnt


@pytest.mark.parametrize("target", ["y", "r", "c"])
def test_drf_oob_metrics_cpu(target):
    from sklearn.metrics import roc_auc_score

    df, fr = _frame(3000, "cpu")
    x = [f"x{i}" for i in range(6)]
    m = H2ORandomForestEstimator(ntrees=12, max_depth=8, seed=5, sample_rate=0.632).train(x=x, y=target,
                                                                                           training_frame=fr)
    tm = m.training_metrics
    assert "Out-Of-Bag" in tm["description"]
    s, cnt = _manual_oob(m, df, 0.632, 5)
    ok = cnt > 0
    assert tm["oob_rows"] == int(ok.sum())
    if target == "y":
        p1 = np.clip(s[0, ok] / cnt[ok], 0, 1)
        yb = (df.y == "b").to_numpy()[ok]
        # (h2omx AUC: H2O's 400-bin histogram AUC -> agrees with the exact AUC to ~1e-5)
        np.testing.assert_allclose(tm["AUC"], roc_auc_score(yb, p1), rtol=1e-4)
        # out-of-bag is an honest estimate: below the in-sample AUC
        assert tm["AUC"] < m.model_performance(fr)["AUC"]
    elif target == "r":
        pred = s[0, ok] / cnt[ok]
        np.testing.assert_allclose(tm["MSE"], np.mean((df.r.to_numpy()[ok] - pred) ** 2), rtol=1e-5)
    else:
        assert 0 < tm["logloss"] and tm["oob_rows"] > 2500


@pytest.mark.gpu
def test_drf_oob_metrics_gpu(cuda_dev):
    """oob_accumulate_kernel (after every tree, bag hash of the iteration)."""
    from sklearn.metrics import roc_auc_score

    df, fr = _frame(50_000, cuda_dev, seed=4)
    x = [f"x{i}" for i in range(6)]
    for target in ("y", "c"):
        m = H2ORandomForestEstimator(ntrees=8, max_depth=10, seed=5).train(x=x, y=target, training_frame=fr)
        s, cnt = _manual_oob(m, df, 0.632, 5)
        ok = cnt > 0
        tm = m.training_metrics
        assert tm["oob_rows"] == int(ok.sum())
        if target == "y":
            p1 = np.clip(s[0, ok] / cnt[ok], 0, 1)
            np.testing.assert_allclose(tm["AUC"], roc_auc_score((df.y == "b").to_numpy()[ok], p1), rtol=1e-4)
