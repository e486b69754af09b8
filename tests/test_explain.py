"""TreeSHAP contributions vs a brute-force path-dependent Shapley oracle,
additivity (contributions + bias = raw margin), and partial dependence
(CPU; tests/test_explain_gpu.py runs the HIP kernel against the same oracle)."""
import itertools
import math

import numpy as np
import pandas as pd
import pytest

from h2omx.explain import partial_dependence, predict_contributions, tree_paths
from h2omx.frame import Frame
from h2omx.models import H2OGradientBoostingEstimator, H2ORandomForestEstimator


def cond_expect(tree, x, S, i=0):
    """E[f(x) | x_S] with the path-dependent (cover-weighted) rule."""
    nd = tree[i]
    if nd["feat"] < 0:
        return float(nd["value"])
    f, left = int(nd["feat"]), int(nd["left"])
    if f in S:
        v = x[f]
        go_left = bool(nd["na_left"]) if np.isnan(v) else v <= nd["thr"]
        return cond_expect(tree, x, S, left if go_left else left + 1)
    w = float(nd["weight"])
    wl, wr = float(tree[left]["weight"]), float(tree[left + 1]["weight"])
    return (wl * cond_expect(tree, x, S, left) + wr * cond_expect(tree, x, S, left + 1)) / w


def brute_shap(trees, x, F, scale=1.0):
    phi = np.zeros(F)
    for tr in trees:
        for i in range(F):
            others = [j for j in range(F) if j != i]
            for k in range(F):
                for S in itertools.combinations(others, k):
                    wgt = math.factorial(k) * math.factorial(F - k - 1) / math.factorial(F)
                    phi[i] += scale * wgt * (cond_expect(tr, x, set(S) | {i}) - cond_expect(tr, x, set(S)))
    return phi


def _data(n=3000, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 4)).astype(np.float32)
    X[::17, 1] = np.nan
    logit = X[:, 0] - np.nan_to_num(X[:, 1]) * X[:, 2] + 0.3 * X[:, 3]
    y = np.where(rng.random(n) < 1 / (1 + np.exp(-logit)), "a", "b")
    df = pd.DataFrame(X, columns=list("pqrs"))
    df["y"] = pd.Categorical(y)
    return df


@pytest.mark.parametrize("cls,kw", [(H2OGradientBoostingEstimator, dict(ntrees=6, max_depth=3)),
                                    (H2ORandomForestEstimator, dict(ntrees=4, max_depth=4))])
def test_tree_shap_matches_bruteforce(cls, kw):
    df = _data()
    fr = Frame.from_pandas(df)
    m = cls(seed=1, **kw).train(y="y", training_frame=fr)
    C = predict_contributions(m, fr).to_pandas()
    assert list(C.columns) == ["p", "q", "r", "s", "BiasTerm"]
    margin = m.ens.raw_margin(fr.feature_matrix(m.x))[0].numpy()
    np.testing.assert_allclose(C.values.sum(1), margin, atol=2e-4)
    scale = 1.0 / m.ens.ntrees if m.ens.average else 1.0
    X = df[list("pqrs")].values.astype(np.float64)
    for r in (0, 17, 123):
        ref = brute_shap(m.ens.trees, X[r], 4, scale)
        np.testing.assert_allclose(C.values[r, :4], ref, atol=1e-4)


def test_tree_paths_expected_value():
    df = _data(seed=2)
    m = H2OGradientBoostingEstimator(ntrees=3, max_depth=2, seed=1).train(y="y", training_frame=Frame.from_pandas(df))
    lv, el, expected, maxm, _ = tree_paths(m.ens.trees)
    ref = sum(cond_expect(t, np.zeros(4), set()) for t in m.ens.trees)
    assert abs(expected - ref) < 1e-6 and maxm <= 2
    assert lv.shape[0] <= 3 * 4 and el.shape[0] == lv[:, 1].sum()


def test_partial_dependence_monotone():
    df = _data()
    fr = Frame.from_pandas(df)
    m = H2OGradientBoostingEstimator(ntrees=20, max_depth=3, seed=1).train(y="y", training_frame=fr)
    pd_ = partial_dependence(m, fr, "p", nbins=10)
    means = [r["mean_response"] for r in pd_["data"]]
    assert len(means) == 10
    # y = "b" (second level) is less likely for larger p (logit of "a" rises with p... domain ["a","b"])
    assert means[0] > means[-1]
    assert all(r["std_error_mean_response"] >= 0 for r in pd_["data"])
