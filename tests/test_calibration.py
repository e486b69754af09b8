"""calibrate_model / calibration_frame / calibration_method for tree models
(H2O: Platt scaling or isotonic regression of y on p1 over the calibration
frame; predictions gain cal_p0 / cal_p1)."""
import numpy as np
import pandas as pd
import pytest

from h2omx.frame import Frame
from h2omx.models import H2OGradientBoostingEstimator, H2ORandomForestEstimator


def _df(n, seed):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, 3))
    p = 1 / (1 + np.exp(-(0.5 + 1.2 * x[:, 0] - x[:, 1])))
    df = pd.DataFrame(x, columns=["a", "b", "c"])
    df["y"] = pd.Categorical(np.where(rng.random(n) < p, "1", "0"), categories=["0", "1"])
    return df


@pytest.mark.parametrize("method", ["PlattScaling", "IsotonicRegression"])
def test_calibrated_probabilities(method):
    tr, cal = Frame.from_pandas(_df(3000, 0)), Frame.from_pandas(_df(2000, 1))
    # DRF leaves are class fractions of bagged deep trees: over-confident on the
    # training rows, calibration pulls them back
    m = H2ORandomForestEstimator(ntrees=10, max_depth=12, seed=1, calibrate_model=True, calibration_frame=cal,
                                 calibration_method=method).train(x=["a", "b", "c"], y="y", training_frame=tr)
    out = m.predict(cal).to_pandas()
    assert {"cal_p0", "cal_p1"} <= set(out.columns)
    np.testing.assert_allclose(out.cal_p0 + out.cal_p1, 1.0, atol=1e-6)
    y = (cal.to_pandas().y == "1").to_numpy(float)

    def logloss(p):
        p = np.clip(p, 1e-6, 1 - 1e-6)
        return -np.mean(y * np.log(p) + (1 - y) * np.log(1 - p))

    assert logloss(out.cal_p1.to_numpy()) <= logloss(out["1"].to_numpy()) + 1e-9
    if method == "IsotonicRegression":
        order = np.argsort(out["1"].to_numpy(), kind="stable")
        assert np.all(np.diff(out.cal_p1.to_numpy()[order]) >= -1e-7)


def test_calibration_requires_binomial_and_frame():
    tr = Frame.from_pandas(_df(500, 2))
    with pytest.raises(ValueError, match="calibration_frame"):
        H2OGradientBoostingEstimator(ntrees=2, calibrate_model=True).train(x=["a", "b"], y="y", training_frame=tr)


def test_platt_calibration_in_mojo(tmp_path):
    from h2omx.mojo import import_mojo

    tr, cal = Frame.from_pandas(_df(2000, 3)), Frame.from_pandas(_df(1000, 4))
    m = H2OGradientBoostingEstimator(ntrees=10, max_depth=3, seed=1, calibrate_model=True,
                                     calibration_frame=cal).train(x=["a", "b", "c"], y="y", training_frame=tr)
    g = import_mojo(m.download_mojo(str(tmp_path)))
    a, b = m.predict(cal).to_pandas(), g.predict(cal).to_pandas()
    np.testing.assert_allclose(b.cal_p1.to_numpy(), a.cal_p1.to_numpy(), rtol=1e-5, atol=1e-6)
