"""CPU reference implementations of the dense kernels (test oracle and the
CPU-only plumbing path, e.g. the kind/iris deployment).

The HIP kernel layer (``h2omx/ops/dense.py``, ``csrc/dense_kernels.hip``)
contains no CPU code: :mod:`h2omx.backend` routes device tensors there and
host tensors here, so production GPU runs never import this module.  Every
function has the same signature and contract as its HIP counterpart.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops.dense import ACTS, DEFAULT_LINK, FAMILIES, LINKS  # noqa: F401 - shared constants


def glm_irls_pass(X: torch.Tensor, y: torch.Tensor, wprior, offset, beta: np.ndarray, family: str, link: str,
                  cls: int = 0, var_power: float = 1.5, link_power: float = 0.0):
    """fp64 NumPy IRLS pass: the augmented weighted Gram [x | 1 | z] and the deviance."""
    return _irls_pass_ref(X, y, wprior, offset, beta, family, link, cls, var_power, link_power)


def glm_grad_pass(X: torch.Tensor, y: torch.Tensor, wprior, offset, beta: np.ndarray, family: str, link: str,
                  var_power: float = 1.5, link_power: float = 0.0):
    """fp64 NumPy mirror of the HIP gradient pass: (sum_i r_ki [x_i | 1], deviance)."""
    Xn = X.detach().cpu().double().numpy()
    yn = y.detach().cpu().double().numpy()
    w = np.ones_like(yn) if wprior is None else wprior.detach().cpu().double().numpy()
    off = 0.0 if offset is None else offset.detach().cpu().double().numpy()
    p, n = Xn.shape
    K = beta.shape[0]
    eta = beta[:, :p] @ Xn + beta[:, p:p + 1]
    if family == "multinomial":
        e = np.exp(eta - eta.max(0))
        pr = e / e.sum(0)
        Y = (yn[None, :].astype(np.int64) == np.arange(K)[:, None]).astype(np.float64)
        R = w * (pr - Y)
        dev = float((w * -2 * np.log(np.maximum(pr[yn.astype(np.int64), np.arange(n)], 1e-300))).sum())
    else:
        e0 = eta[0] + off
        mu, dmu = _linkinv(e0, link, link_power)
        if dmu is None:
            dmu = np.maximum(mu * (1 - mu), 1e-10)
        dmu = np.maximum(dmu, 1e-10) if link in ("log", "tweedie") and link_power == 0 else dmu
        R = (w * (mu - yn) * dmu / glm_variance(family, mu, var_power))[None, :]
        dev = float((w * glm_deviance(family, yn, mu, var_power)).sum())
    g = np.concatenate([R @ Xn.T, R.sum(1, keepdims=True)], axis=1)
    return g, dev


def _linkinv(eta, link, link_power=0.0):
    if link == "logit":
        return 1 / (1 + np.exp(-eta)), None
    if link == "log":
        mu = np.exp(np.minimum(eta, 700))
        return mu, mu
    if link == "inverse":
        e = np.where(np.abs(eta) < 1e-10, np.copysign(1e-10, eta), eta)
        mu = 1 / e
        return mu, -mu * mu
    if link == "tweedie":
        if link_power == 0:
            mu = np.exp(np.minimum(eta, 700))
            return mu, mu
        e = np.maximum(eta, 1e-10)
        mu = e ** (1 / link_power)
        return mu, mu / (link_power * e)
    return eta, np.ones_like(eta)


def glm_variance(family, mu, var_power=1.5):
    if family in ("binomial", "quasibinomial", "fractionalbinomial"):
        return np.maximum(mu * (1 - mu), 1e-10)
    if family == "negativebinomial":                       # var_power carries theta
        return np.maximum(mu + var_power * mu * mu, 1e-10)
    if family == "poisson":
        return np.maximum(mu, 1e-10)
    if family == "gamma":
        return np.maximum(mu * mu, 1e-20)
    if family == "tweedie":
        return np.maximum(np.maximum(mu, 1e-10) ** var_power, 1e-20)
    return np.ones_like(mu)


def glm_deviance(family, y, mu, var_power=1.5):
    if family == "negativebinomial":
        th, m = var_power, np.maximum(mu, 1e-15)
        with np.errstate(divide="ignore", invalid="ignore"):
            a = np.where(y > 0, y * np.log(np.where(y > 0, y, 1) / m), 0.0)
        return 2 * (a - (y + 1 / th) * np.log((1 + th * y) / (1 + th * m)))
    if family in ("binomial", "quasibinomial", "fractionalbinomial"):
        m = np.clip(mu, 1e-15, 1 - 1e-15)
        return -2 * (y * np.log(m) + (1 - y) * np.log(1 - m))
    if family == "poisson":
        m = np.maximum(mu, 1e-15)
        with np.errstate(divide="ignore", invalid="ignore"):
            t = np.where(y > 0, y * np.log(np.where(y > 0, y, 1) / m), 0.0)
        return 2 * (t - (y - m))
    if family == "gamma":
        m = np.maximum(mu, 1e-15)
        return 2 * (-np.log(np.maximum(y, 1e-15) / m) + (y - m) / m)
    if family == "tweedie":
        r = var_power
        m = np.maximum(mu, 1e-15)
        a = np.where(y > 0, np.maximum(y, 0) ** (2 - r) / ((1 - r) * (2 - r)), 0.0)
        return 2 * (a - y * m ** (1 - r) / (1 - r) + m ** (2 - r) / (2 - r))
    return (y - mu) ** 2


def _irls_pass_ref(X, y, wprior, offset, beta, family, link, cls, var_power, link_power):
    Xn = X.double().numpy()
    p, n = Xn.shape
    yv = y.double().numpy()
    wp = np.ones(n) if wprior is None else wprior.double().numpy()
    off = np.zeros(n) if offset is None else offset.double().numpy()
    if family == "multinomial":
        etas = beta[:, :p] @ Xn + beta[:, p:p + 1]
        etas -= etas.max(axis=0, keepdims=True)
        pr = np.exp(etas)
        pr /= pr.sum(axis=0, keepdims=True)
        pk = np.clip(pr[cls], 1e-10, 1 - 1e-10)
        yk = (yv.astype(np.int64) == cls).astype(np.float64)
        eta_k = beta[cls, :p] @ Xn + beta[cls, p]
        w = pk * (1 - pk)
        z = eta_k + (yk - pk) / w
        w = w * wp
        dev = float((wp * np.where(yk > 0, -2 * np.log(pk), 0.0)).sum())
    else:
        eta = beta[0, :p] @ Xn + beta[0, p] + off
        mu, dmu = _linkinv(eta, link, link_power)
        if link == "logit":
            dmu = np.maximum(mu * (1 - mu), 1e-10)
        elif link == "log" or (link == "tweedie" and link_power == 0):
            dmu = np.maximum(mu, 1e-10)
        w = wp * dmu * dmu / glm_variance(family, mu, var_power)
        z = eta - off + (yv - mu) / dmu
        dev = float((wp * glm_deviance(family, yv, mu, var_power)).sum())
    A = np.vstack([Xn, np.ones((1, n)), z[None, :]])
    sw = np.sqrt(np.maximum(w, 0))
    As = A * sw[None, :]
    return As @ As.T, dev



def kmeans_step(X: torch.Tensor, C, na_free: bool = False):
    """One Lloyd pass in fp64 (same outputs as the HIP kernel; ``na_free`` is
    the device kernels' no-NA hint, unused here; C a tensor or host array)."""
    if isinstance(C, np.ndarray):
        C = torch.from_numpy(np.ascontiguousarray(C, np.float32))
    d, n = X.shape
    k = C.shape[0]
    Xn = X.double().numpy()
    Cn = C.double().numpy()
    d2 = (Cn ** 2).sum(1)[:, None] - 2 * Cn @ Xn
    a = np.argmin(d2, axis=0)
    x2 = (Xn ** 2).sum(0)
    sums = np.zeros((k, d))
    np.add.at(sums, a, Xn.T)
    counts = np.bincount(a, minlength=k).astype(np.float64)
    sse = np.bincount(a, weights=np.maximum(d2[a, np.arange(n)] + x2, 0), minlength=k)
    return torch.from_numpy(a.astype(np.int32)), sums, counts, sse


def gemm(A: torch.Tensor, B: torch.Tensor, bias=None, act: int = 0, ta: bool = False, tb: bool = False,
         out: torch.Tensor | None = None, beta_c: float = 0.0) -> torch.Tensor:
    a = A.T if ta else A
    b = B.T if tb else B
    c = a.float() @ b.float()
    if beta_c and out is not None:
        c = c + beta_c * out
    if bias is not None:
        c = c + bias
    if act == 1:
        c = torch.relu(c)
    elif act == 2:
        c = torch.tanh(c)
    if out is not None:
        out.copy_(c)
        return out
    return c


def act_backward(Y: torch.Tensor, dY: torch.Tensor, act: int) -> torch.Tensor:
    if act == 1:
        dY.mul_((Y > 0).float())
    elif act == 2:
        dY.mul_(1 - Y * Y)
    return dY


def act_backward_bias(Y: torch.Tensor, dY: torch.Tensor, act: int):
    """Reference of ops.dense.act_backward_bias: the 'slices' are the full column sums."""
    act_backward(Y, dY, act)
    return dY, (dY.sum(0)[None, :], 1)


def out_layer_ok(dZ: torch.Tensor, H: torch.Tensor) -> bool:
    return False


def out_wgrad(dZ: torch.Tensor, H: torch.Tensor, dW: torch.Tensor, db: torch.Tensor) -> None:
    dW.copy_(dZ.T @ H)
    db.copy_(dZ.sum(0))


def thin_dact(dZ: torch.Tensor, W: torch.Tensor, Y: torch.Tensor, act: int):
    C = dZ @ W
    act_backward(Y, C, act)
    return C, (C.sum(0)[None, :], 1)


def dact_ok(dZ: torch.Tensor, W: torch.Tensor) -> bool:
    """the CPU path keeps the unfused GEMM + act_backward_bias pair"""
    return False


def gemm_dact(dZ: torch.Tensor, W: torch.Tensor, Y: torch.Tensor, act: int, out: torch.Tensor | None = None,
              tile: int = 2):
    """Reference of ops.dense.gemm_dact: (dZ W) * act'(Y) and its column sums."""
    C = dZ @ W
    act_backward(Y, C, act)
    if out is not None:
        out.copy_(C)
        C = out
    return C, (C.sum(0)[None, :], 1)


def wgrad_bias(dZ: torch.Tensor, H: torch.Tensor, dW: torch.Tensor, db: torch.Tensor, bpart) -> None:
    dW.copy_(dZ.T @ H)
    db.copy_(bpart[0].sum(0))


def bias_grad(dY: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    r = dY.sum(0)
    if out is not None:
        out.copy_(r)
        return out
    return r


def softmax_xent(Z: torch.Tensor, y: torch.Tensor, with_loss: bool = True):
    M, K = Z.shape
    pr = torch.softmax(Z, 1)
    oh = torch.nn.functional.one_hot(y.long(), K).float()
    loss = -(torch.log(pr.clamp_min(1e-30)) * oh).sum(1).mean()
    return (pr - oh) / M, loss.reshape(1)


def adadelta_(W, G, Eg2, Edx2, rho=0.99, eps=1e-8, l2=0.0):
    g = G + l2 * W
    Eg2.mul_(rho).add_((1 - rho) * g * g)
    dx = -torch.sqrt(Edx2 + eps) / torch.sqrt(Eg2 + eps) * g
    Edx2.mul_(rho).add_((1 - rho) * dx * dx)
    W.add_(dx)


def sgd_momentum_(W, G, V, lr, mom, l2=0.0):
    V.mul_(mom).sub_(lr * (G + l2 * W))
    W.add_(V)


def gemm_bf16_nt(A: torch.Tensor, B: torch.Tensor, M: int, N: int, K: int, *, bias=None, act: int = 0,
                 ymask: torch.Tensor | None = None, mask_act: int = 0, out_f32: torch.Tensor | None = None,
                 out_bf16: torch.Tensor | None = None, out_bf16_t: torch.Tensor | None = None,
                 beta_c: float = 0.0, splitk: int = 1, c_last: torch.Tensor | None = None) -> None:
    """The bf16 GEMM contract computed in fp32 from the bf16 operand values."""
    c = A[:M, :K].float() @ B[:N, :K].float().T
    if out_f32 is not None and beta_c:
        c = c + beta_c * out_f32[:M, :N]
    if bias is not None:
        c = c + bias[:N]
    if act == 1:
        c = torch.relu(c)
    elif act == 2:
        c = torch.tanh(c)
    if mask_act:
        y = ymask[:M, :N].float()
        c = torch.where(y > 0, c, torch.zeros_like(c)) if mask_act == 1 else c * (1 - y * y)
    if c_last is not None:
        c_last[:M] = c[:, N - 1]
        c = c[:, : N - 1]
    if out_f32 is not None:
        out_f32[:M, : c.shape[1]] = c
    if out_bf16 is not None:
        out_bf16[:M, :N] = c.to(torch.bfloat16)
    if out_bf16_t is not None:
        out_bf16_t[:N, :M] = c.T.to(torch.bfloat16)


def cvt_bf16(X: torch.Tensor, out: torch.Tensor | None = None, out_t: torch.Tensor | None = None) -> None:
    R, C = X.shape
    if out is not None:
        out[:R, :C] = X.to(torch.bfloat16)
        if out.shape[1] > C:
            out[:R, C:] = 0
    if out_t is not None:
        out_t[:C, :R] = X.T.to(torch.bfloat16)


def rowsum_bf16(X: torch.Tensor, R: int, C: int, out: torch.Tensor) -> None:
    out[:R] = X[:R, :C].float().sum(1)


def cvt_bf16_multi(jobs) -> None:
    for X, out, out_t in jobs:
        cvt_bf16(X, out, out_t)


def softmax_xent_bf16(Z: torch.Tensor, y: torch.Tensor, dZ: torch.Tensor, dZt: torch.Tensor,
                      loss: torch.Tensor) -> None:
    M, K = Z.shape
    g, l = softmax_xent(Z, y)
    dZ[:M, :K] = g.to(torch.bfloat16)
    dZt[:K, :M] = g.T.to(torch.bfloat16)
    loss += l
