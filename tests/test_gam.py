"""GAM: cubic regression splines (basis interpolates, penalty = ∫f''²) and a
penalised GLM fit of a smooth nonlinear effect."""
import numpy as np
import pandas as pd
import pytest
import torch

from h2omx.frame import Frame
from h2omx.models.gam import H2OGeneralizedAdditiveEstimator, cr_basis, cr_basis_matrices
from h2omx.models.glm import H2OGeneralizedLinearEstimator


def test_cr_basis_interpolates_and_penalty_is_curvature():
    knots = np.array([0.0, 0.7, 1.5, 2.2, 3.0, 4.1])
    F, S = cr_basis_matrices(knots)
    X = cr_basis(torch.from_numpy(knots), knots, F).numpy()
    np.testing.assert_allclose(X, np.eye(knots.size), atol=1e-12)     # values at knots = beta
    lin = 2 * knots + 1                                                # a line has zero curvature
    assert abs(lin @ S @ lin) < 1e-9
    xs = np.linspace(-1, 5, 50)
    Xs = cr_basis(torch.from_numpy(xs), knots, F).numpy()
    np.testing.assert_allclose(Xs @ lin, 2 * xs + 1, atol=1e-9)       # reproduces (and extrapolates) lines
    q = knots ** 2                                                     # f'' = 2 -> ∫ f''² = 4 (b - a)
    assert abs(q @ S @ q - 4 * (knots[-1] - knots[0])) / (4 * (knots[-1] - knots[0])) < 0.15


def _df(n=4000, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-3, 3, n)
    z = rng.normal(size=n)
    y = np.sin(2 * x) + 0.5 * z + 0.1 * rng.normal(size=n)
    return pd.DataFrame({"x": x, "z": z, "y": y})


def test_gam_fits_smooth_effect_and_scale_controls_wiggliness():
    df = _df()
    fr = Frame.from_pandas(df)
    g = H2OGeneralizedAdditiveEstimator(family="gaussian", gam_columns=["x"], num_knots=[12], scale=[1e-4],
                                        lambda_=0.0).train(x=["x", "z"], y="y", training_frame=fr)
    lin = H2OGeneralizedLinearEstimator(family="gaussian", lambda_=0.0).train(x=["x", "z"], y="y", training_frame=fr)
    mse_g = g.training_metrics["MSE"]
    assert mse_g < 0.05 and mse_g < 0.3 * lin.training_metrics["MSE"]
    test = _df(n=500, seed=1)
    pr = g.predict(Frame.from_pandas(test)).to_pandas()["predict"].to_numpy()
    assert np.mean((pr - test.y) ** 2) < 0.06
    assert abs(g.coef()["z"] - 0.5) < 0.05
    stiff = H2OGeneralizedAdditiveEstimator(family="gaussian", gam_columns=["x"], num_knots=[12], scale=[1e4],
                                            lambda_=0.0).train(x=["x", "z"], y="y", training_frame=fr)
    assert stiff.training_metrics["MSE"] > 2 * mse_g
    with pytest.raises(ValueError):
        H2OGeneralizedAdditiveEstimator(family="gaussian").train(x=["x"], y="y", training_frame=fr)


def test_gam_binomial():
    rng = np.random.default_rng(3)
    x = rng.uniform(-3, 3, 5000)
    yb = (rng.random(5000) < 1 / (1 + np.exp(-3 * np.sin(2 * x)))).astype(int)
    fr = Frame.from_pandas(pd.DataFrame({"x": x, "y": pd.Categorical(np.where(yb == 1, "b", "a"))}))
    g = H2OGeneralizedAdditiveEstimator(family="binomial", gam_columns=["x"], num_knots=[10],
                                        lambda_=0.0).train(x=["x"], y="y", training_frame=fr)
    assert g.training_metrics["AUC"] > 0.8
