"""categorical_encoding="SortByResponse" for tree models: levels reordered by
mean response, so one ordinal split separates a scattered set of high-
response levels that the lexicographic order interleaves."""
import numpy as np
import pandas as pd

from h2omx.frame import Frame
from h2omx.models import H2OGradientBoostingEstimator
from h2omx.mojo import import_mojo


def test_sort_by_response_separates_interleaved_levels(tmp_path):
    rng = np.random.default_rng(0)
    n = 4000
    levels = [f"L{i:02d}" for i in range(20)]
    g = rng.choice(levels, n)
    hi = {lv for i, lv in enumerate(levels) if i % 2 == 0}      # every other level is "high"
    y = np.array([3.0 if v in hi else 0.0 for v in g]) + 0.1 * rng.normal(size=n)
    df = pd.DataFrame({"g": pd.Categorical(g, categories=levels), "x": rng.normal(size=n), "y": y})
    fr = Frame.from_pandas(df)
    kw = dict(ntrees=1, max_depth=1, learn_rate=1.0, min_rows=1, seed=1)
    # ordinal codes in lexicographic level order (no group splits)
    lab = H2OGradientBoostingEstimator(categorical_encoding="LabelEncoder", **kw).train(
        x=["g", "x"], y="y", training_frame=fr)
    # AUTO: H2O's group split sends the set of high levels one way in one split
    auto = H2OGradientBoostingEstimator(**kw).train(x=["g", "x"], y="y", training_frame=fr)
    sbr = H2OGradientBoostingEstimator(categorical_encoding="SortByResponse", **kw).train(
        x=["g", "x"], y="y", training_frame=fr)
    dom = sbr.feature_domains["g"]
    assert set(dom[:10]) == set(levels) - hi and set(dom[10:]) == hi
    mse = lambda m: float(np.mean((m.predict(fr).to_pandas()["predict"].to_numpy() - y) ** 2))
    assert mse(sbr) < 0.1 < mse(lab)            # a depth-1 ordinal stump: one split does it only after sorting
    assert mse(auto) < 0.1
    g2 = import_mojo(sbr.download_mojo(str(tmp_path)))
    np.testing.assert_allclose(g2.predict(fr).to_pandas()["predict"].to_numpy(),
                               sbr.predict(fr).to_pandas()["predict"].to_numpy(), rtol=1e-5, atol=1e-5)
