"""GLM ``solver`` (H2O GLMParameters.Solver): L_BFGS (OWL-QN over Gram-free
gradient passes), COORDINATE_DESCENT, AUTO resolution and rejection of
unsupported values.  CPU tests run the NumPy oracle passes; GPU tests check
the HIP gradient kernels (glm_resid_kernel / glm_xtr_kernel) against it and
a GPU L_BFGS fit against the IRLSM optimum."""
from __future__ import annotations

import numpy as np
import pandas as pd
import pytest
import torch

from h2omx.frame.frame import Frame
from h2omx.models.glm import H2OGeneralizedLinearEstimator as GLM
from h2omx.models.glm_solvers import owlqn, resolve_solver


def _frame(n=3000, seed=0, kind="binomial", p=6):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, p))
    b = np.linspace(-1.5, 1.5, p)
    eta = X @ b * 0.5 - 0.3
    df = pd.DataFrame(X, columns=[f"x{i}" for i in range(p)])
    if kind == "binomial":
        df["y"] = pd.Categorical(np.where(rng.uniform(size=n) < 1 / (1 + np.exp(-eta)), "b", "a"))
    elif kind == "poisson":
        df["y"] = rng.poisson(np.exp(0.3 * eta)).astype(float)
    elif kind == "multinomial":
        logits = np.stack([eta, -eta, 0.5 * X[:, 0]])
        pr = np.exp(logits - logits.max(0))
        pr /= pr.sum(0)
        u = rng.uniform(size=n)
        df["y"] = pd.Categorical((u[None] > np.cumsum(pr, 0)).sum(0).astype(str))
    else:
        df["y"] = eta + 0.5 * rng.normal(size=n)
    return df


@pytest.mark.parametrize("family,alpha,lam", [
    ("binomial", 0.0, 0.0), ("binomial", 0.5, 0.01), ("gaussian", 1.0, 0.02), ("poisson", 0.0, 1e-3),
])
def test_lbfgs_matches_irlsm(family, alpha, lam):
    fr = Frame.from_pandas(_frame(kind=family))
    a = GLM(family=family, solver="IRLSM", alpha=alpha, lambda_=lam).train(y="y", training_frame=fr)
    b = GLM(family=family, solver="L_BFGS", alpha=alpha, lambda_=lam).train(y="y", training_frame=fr)
    assert b.stats["solver"] == "L_BFGS" and a.stats["solver"] == "IRLSM"
    ca, cb = np.array(list(a.coef().values())), np.array(list(b.coef().values()))
    np.testing.assert_allclose(cb, ca, atol=2e-4)
    assert abs(a.stats["residual_deviance"] - b.stats["residual_deviance"]) < 1e-5 * a.stats["residual_deviance"]
    if alpha > 0:
        # lasso zeros: the same coefficients are exactly zero
        assert ((np.abs(ca) < 1e-8) == (np.abs(cb) < 1e-8)).all()


def test_multinomial_lbfgs_and_deviance():
    fr = Frame.from_pandas(_frame(kind="multinomial"))
    a = GLM(family="multinomial", solver="IRLSM", alpha=0.0, lambda_=1e-3, beta_epsilon=1e-7,
            max_iterations=200).train(y="y", training_frame=fr)
    b = GLM(family="multinomial", solver="L_BFGS", alpha=0.0, lambda_=1e-3).train(y="y", training_frame=fr)
    # residual deviance covers every class's rows (not only class 0's)
    assert a.stats["residual_deviance"] > 0.5 * a.stats["null_deviance"]
    assert abs(a.stats["residual_deviance"] - b.stats["residual_deviance"]) < 1e-3 * a.stats["residual_deviance"]
    pa = a.predict(fr).to_pandas().iloc[:, 1:].to_numpy()
    pb = b.predict(fr).to_pandas().iloc[:, 1:].to_numpy()
    assert np.abs(pa - pb).max() < 5e-3


def test_coordinate_descent_solver_same_optimum():
    fr = Frame.from_pandas(_frame(kind="gaussian"))
    a = GLM(family="gaussian", solver="IRLSM", alpha=0.0, lambda_=0.01).train(y="y", training_frame=fr)
    b = GLM(family="gaussian", solver="COORDINATE_DESCENT", alpha=0.0, lambda_=0.01).train(y="y", training_frame=fr)
    np.testing.assert_allclose(list(b.coef().values()), list(a.coef().values()), atol=1e-6)
    assert b.stats["solver"] == "COORDINATE_DESCENT"


def test_solver_validation_and_auto():
    fr = Frame.from_pandas(_frame(n=300))
    with pytest.raises(ValueError, match="unknown solver"):
        GLM(family="binomial", solver="NEWTON").train(y="y", training_frame=fr)
    with pytest.raises(ValueError, match="only supported for family='ordinal'"):
        GLM(family="binomial", solver="GRADIENT_DESCENT_LH").train(y="y", training_frame=fr)
    assert resolve_solver("AUTO", "binomial", 100, 1) == "IRLSM"
    assert resolve_solver("AUTO", "binomial", 6000, 1) == "L_BFGS"
    assert resolve_solver("AUTO", "multinomial", 2000, 20) == "L_BFGS"
    assert resolve_solver(None, "ordinal", 10, 3) == "GRADIENT_DESCENT_LH"
    with pytest.raises(ValueError):
        resolve_solver("L_BFGS", "ordinal", 10, 3)
    m = GLM(family="binomial").train(y="y", training_frame=fr)
    assert m.stats["solver"] == "IRLSM"


def test_owlqn_quadratic_lasso():
    """OWL-QN on 1/2 |Ab - c|^2 + l1 |b|_1 against the coordinate-descent optimum."""
    rng = np.random.default_rng(3)
    A = rng.normal(size=(50, 8))
    c = A @ np.array([1.0, 0, 0, -2, 0, 0.5, 0, 0]) + 0.1 * rng.normal(size=50)

    def fg(b):
        r = A @ b - c
        return 0.5 * r @ r, A.T @ r, 0.0

    l1 = 3.0
    res = owlqn(fg, np.zeros(8), np.ones(8, bool), l1, max_iter=500, grad_eps=1e-10)
    b = np.zeros(8)
    for _ in range(2000):   # reference: cyclic coordinate descent
        for j in range(8):
            rj = c - A @ b + A[:, j] * b[j]
            z = A[:, j] @ rj
            b[j] = np.sign(z) * max(abs(z) - l1, 0) / (A[:, j] @ A[:, j])
    np.testing.assert_allclose(res.beta, b, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("family,link", [("binomial", "logit"), ("gaussian", "identity"), ("poisson", "log"),
                                         ("gamma", "inverse"), ("multinomial", "logit")])
def test_glm_grad_pass_gpu_matches_reference(cuda_dev, family, link):
    from h2omx.ops import dense as dev_ops
    from h2omx.reference import dense as ref_ops

    rng = np.random.default_rng(5)
    p, n = 37, 70001
    X = torch.tensor(rng.normal(size=(p, n)), dtype=torch.float32)
    K = 4 if family == "multinomial" else 1
    beta = rng.normal(size=(K, p + 1)) * 0.05
    if family == "gamma":
        beta[0, p] = 2.0
        y = torch.tensor(rng.gamma(2.0, 0.25, n), dtype=torch.float32)
    elif family == "multinomial":
        y = torch.tensor(rng.integers(0, K, n), dtype=torch.float32)
    elif family == "poisson":
        y = torch.tensor(rng.poisson(1.0, n), dtype=torch.float32)
    elif family == "binomial":
        y = torch.tensor(rng.integers(0, 2, n), dtype=torch.float32)
    else:
        y = torch.tensor(rng.normal(size=n), dtype=torch.float32)
    w = torch.tensor(rng.uniform(0.5, 2.0, n), dtype=torch.float32)
    gr, dr = ref_ops.glm_grad_pass(X, y, w, None, beta, family, link)
    gd, dd = dev_ops.glm_grad_pass(X.to(cuda_dev), y.to(cuda_dev), w.to(cuda_dev), None, beta, family, link)
    scale = np.abs(gr).max()
    np.testing.assert_allclose(gd, gr, atol=2e-5 * scale, rtol=1e-4)
    assert abs(dd - dr) < 1e-6 * abs(dr)


@pytest.mark.gpu
def test_lbfgs_gpu_matches_irlsm(cuda_dev):
    df = _frame(n=200_000, kind="binomial", p=20, seed=2)
    fr = Frame.from_pandas(df).to(cuda_dev)
    a = GLM(family="binomial", solver="IRLSM", alpha=0.5, lambda_=1e-3).train(y="y", training_frame=fr)
    b = GLM(family="binomial", solver="L_BFGS", alpha=0.5, lambda_=1e-3).train(y="y", training_frame=fr)
    np.testing.assert_allclose(list(b.coef().values()), list(a.coef().values()), atol=5e-4)


def test_owlqn_line_search_failure_is_not_convergence():
    """A direction that never satisfies Armijo (here: a gradient of the wrong
    sign, as a badly rounded gradient pass could give) stops the solver with
    converged=False and the stop reason recorded - not a claimed optimum."""
    import numpy as np

    from h2omx.models.glm_solvers import owlqn

    def fg(b):
        return float((b ** 2).sum()), -2.0 * b, float((b ** 2).sum())

    res = owlqn(fg, np.array([1.0, -2.0]), np.array([False, False]), 0.0, max_iter=20)
    assert not res.converged and res.stop_reason == "line_search_failed"

    def fg_ok(b):
        return float(((b - 3.0) ** 2).sum()), 2.0 * (b - 3.0), 0.0

    ok = owlqn(fg_ok, np.zeros(3), np.zeros(3, bool), 0.0)
    assert ok.converged and ok.stop_reason in ("gradient", "objective")
    assert np.allclose(ok.beta, 3.0, atol=1e-5)
