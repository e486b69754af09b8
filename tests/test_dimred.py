"""SVD and GLRM vs NumPy oracles (CPU path; the same code drives the GPU GEMMs)."""
import numpy as np
import pandas as pd
import pytest

from h2omx.frame import Frame
from h2omx.models.glrm import H2OGeneralizedLowRankEstimator
from h2omx.models.svd import H2OSingularValueDecompositionEstimator


def _lowrank(n=2000, p=8, k=3, seed=0, noise=0.01):
    rng = np.random.default_rng(seed)
    U = rng.normal(size=(n, k))
    V = rng.normal(size=(k, p))
    A = U @ V + noise * rng.normal(size=(n, p))
    return pd.DataFrame(A.astype(np.float32), columns=[f"c{i}" for i in range(p)])


def test_svd_matches_numpy():
    df = _lowrank()
    fr = Frame.from_pandas(df)
    m = H2OSingularValueDecompositionEstimator(nv=3).train(training_frame=fr)
    _, s, vt = np.linalg.svd(df.to_numpy().astype(np.float64), full_matrices=False)
    np.testing.assert_allclose(m.d, s[:3], rtol=1e-3)
    for j in range(3):
        assert abs(abs(float(np.dot(m.v[:, j], vt[j]))) - 1.0) < 1e-3
    U = m.u.to_pandas().to_numpy()
    np.testing.assert_allclose(np.abs(U.T @ U), np.eye(3), atol=2e-3)
    proj = m.predict(fr).to_pandas().to_numpy()
    np.testing.assert_allclose(proj, df.to_numpy() @ m.v, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("init", ["SVD", "PlusPlus", "Random"])
def test_glrm_recovers_low_rank(init):
    df = _lowrank(seed=1)
    fr = Frame.from_pandas(df)
    m = H2OGeneralizedLowRankEstimator(k=3, init=init, max_iterations=200, seed=5).train(training_frame=fr)
    R = m.predict(fr).to_pandas().to_numpy()
    A = df.to_numpy()
    assert np.abs(R - A).mean() < 0.05 * np.abs(A).mean()
    assert m.representation.ncols == 3 and m.Y.shape == (3, 8)


def test_glrm_imputes_missing_and_regularizes():
    df = _lowrank(seed=2, noise=0.0)
    A = df.to_numpy().copy()
    rng = np.random.default_rng(9)
    miss = rng.random(A.shape) < 0.15
    dfm = df.mask(miss)
    fr = Frame.from_pandas(dfm)
    m = H2OGeneralizedLowRankEstimator(k=3, init="SVD", max_iterations=400, seed=1).train(training_frame=fr)
    R = m.predict(fr).to_pandas().to_numpy()
    err_missing = np.abs(R[miss] - A[miss]).mean()
    assert err_missing < 0.1 * np.abs(A).mean(), err_missing
    nn = H2OGeneralizedLowRankEstimator(k=2, regularization_x="NonNegative", regularization_y="NonNegative",
                                        max_iterations=50, seed=1).train(training_frame=Frame.from_pandas(df.abs()))
    assert (nn.Y >= 0).all() and float(nn.representation.to_pandas().to_numpy().min()) >= 0
    q = H2OGeneralizedLowRankEstimator(k=3, regularization_x="Quadratic", regularization_y="Quadratic",
                                       gamma_x=5.0, gamma_y=5.0, max_iterations=50).train(training_frame=fr)
    assert np.isfinite(q.objective)
    with pytest.raises(ValueError):
        H2OGeneralizedLowRankEstimator(k=2, loss="Huber").train(training_frame=fr)
