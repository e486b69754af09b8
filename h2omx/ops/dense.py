"""Python entry points of csrc/dense_kernels.hip (GLM IRLS Gram, K-Means,
MLP GEMM + elementwise) with their CPU reference implementations.

Every function takes tensors on one device.  On a GPU tensor the HIP kernel
is the only implementation (``ops.dense_lib()`` raises if the library is
missing); on CPU tensors the NumPy/PyTorch reference runs (test oracle and
the CPU plumbing path).
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import P, check, dense_lib, stream

KBADARG = 1  # common.h kBadArg

FAMILIES = {"gaussian": 0, "binomial": 1, "poisson": 2, "gamma": 3, "tweedie": 4, "multinomial": 5,
            "quasibinomial": 6, "fractionalbinomial": 6, "negativebinomial": 7}
LINKS = {"identity": 0, "logit": 1, "log": 2, "inverse": 3, "tweedie": 4}
DEFAULT_LINK = {"gaussian": "identity", "binomial": "logit", "quasibinomial": "logit", "poisson": "log",
                "gamma": "inverse", "tweedie": "tweedie", "multinomial": "logit", "fractionalbinomial": "logit",
                "negativebinomial": "log", "ordinal": "ologit"}


class GlmParams(ctypes.Structure):
    _fields_ = [("family", ctypes.c_int), ("link", ctypes.c_int), ("p", ctypes.c_int), ("K", ctypes.c_int),
                ("cls", ctypes.c_int), ("pad", ctypes.c_int), ("var_power", ctypes.c_double),
                ("link_power", ctypes.c_double)]


def _tp_for(p: int) -> int:
    for tp in (1, 2, 4, 8):
        if p + 2 <= 32 * tp:
            return tp
    raise ValueError(f"GLM with {p} predictors exceeds the 254-column Gram kernel; reduce predictors")


def glm_irls_pass(X: torch.Tensor, y: torch.Tensor, wprior, offset, beta: np.ndarray, family: str, link: str,
                  cls: int = 0, var_power: float = 1.5, link_power: float = 0.0):
    """One IRLS pass.  X: feature-major standardized float32 [p][n] (no NA).
    beta: float64 [K][p+1] (coefficients then intercept).
    Returns (G float64 [p+2][p+2] of the augmented [x | 1 | z] weighted Gram, deviance)."""
    p, n = X.shape
    K = beta.shape[0]
    if X.is_cuda:
        lib = dense_lib()
        dev = X.device
        tp = _tp_for(p)
        PP = 32 * tp
        n_wg = max(1, min(512, math.ceil(n / 4096)))
        slab = torch.empty((n_wg * PP * PP,), dtype=torch.float32, device=dev)
        devs = torch.empty((n_wg,), dtype=torch.float64, device=dev)
        out = torch.empty((PP * PP,), dtype=torch.float64, device=dev)
        b32 = torch.from_numpy(np.ascontiguousarray(beta, np.float32)).to(dev)
        means = torch.zeros((max(p, 1),), dtype=torch.float32, device=dev)
        gp = GlmParams(FAMILIES[family], LINKS[link], p, K, cls, 0, var_power, link_power)
        Xc = X.contiguous()
        st = stream(dev)
        check(lib.h2omx_glm_irls(P(Xc), Xc.stride(0), n, P(y), P(wprior), P(offset), P(means), P(b32),
                                 ctypes.addressof(gp), n_wg, tp, P(slab), P(devs), st), "glm_irls")
        check(lib.h2omx_slab_reduce_upper(P(slab), n_wg, PP * PP, P(out), st), "slab_reduce_upper")
        G = out.view(PP, PP)[: p + 2, : p + 2].cpu().numpy()
        G = np.triu(G) + np.triu(G, 1).T
        return G, float(devs.sum().item())
    return _irls_pass_ref(X, y, wprior, offset, beta, family, link, cls, var_power, link_power)


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


# ---------------------------------------------------------------------------
# K-Means
# ---------------------------------------------------------------------------
def kmeans_step(X: torch.Tensor, C: torch.Tensor):
    """One Lloyd pass.  X feature-major float32 [d][n] (standardized, NA -> 0),
    C [k][d].  Returns (assign int32 [n], sums float64 [k][d], counts [k], sse [k])."""
    d, n = X.shape
    k = C.shape[0]
    if X.is_cuda:
        lib = dense_lib()
        dev = X.device
        Xc = X.contiguous()
        Cc = C.float().contiguous()
        cn = (Cc.double() ** 2).sum(1).float()
        n_wg = max(1, min(1024, math.ceil(n / 4096)))
        width = k * d + 2 * k
        slab = torch.empty((n_wg * width,), dtype=torch.float32, device=dev)
        out = torch.empty((width,), dtype=torch.float64, device=dev)
        assign = torch.empty((n,), dtype=torch.int32, device=dev)
        st = stream(dev)
        rc = lib.h2omx_kmeans(P(Xc), Xc.stride(0), n, d, P(Cc), P(cn), k, n_wg, P(assign), P(slab), st)
        if rc == KBADARG:
            return _kmeans_large(Xc, Cc)
        check(rc, "kmeans")
        check(lib.h2omx_slab_sum(P(slab), n_wg, width, P(out), st), "slab_sum")
        o = out.cpu().numpy()
        return assign, o[: k * d].reshape(k, d), o[k * d: k * d + k], o[k * d + k:]
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


def _kmeans_large(X: torch.Tensor, C: torch.Tensor):
    """Shapes beyond the fused kernel's LDS tiles (d > 256 or large k): the
    distance GEMM goes to hipBLASLt through torch, in row chunks."""
    d, n = X.shape
    k = C.shape[0]
    cn = (C.double() ** 2).sum(1)
    assign = torch.empty((n,), dtype=torch.int32, device=X.device)
    sums = torch.zeros((k, d), dtype=torch.float64, device=X.device)
    counts = torch.zeros((k,), dtype=torch.float64, device=X.device)
    sse = torch.zeros((k,), dtype=torch.float64, device=X.device)
    step = max(1, (1 << 26) // max(k, 1))
    for s in range(0, n, step):
        xb = X[:, s:s + step]
        d2 = cn[:, None] - 2 * (C @ xb).double()
        m, a = d2.min(0)
        assign[s:s + step] = a.to(torch.int32)
        x2 = (xb.double() ** 2).sum(0)
        counts += torch.bincount(a, minlength=k).double()
        sse += torch.bincount(a, weights=(m + x2).clamp_min(0), minlength=k)
        sums.index_add_(0, a, xb.T.double())
    return assign, sums.cpu().numpy(), counts.cpu().numpy(), sse.cpu().numpy()


# ---------------------------------------------------------------------------
# MLP building blocks
# ---------------------------------------------------------------------------
ACTS = {"linear": 0, "none": 0, "rectifier": 1, "relu": 1, "tanh": 2}  # maxout: models/deeplearning.py


_WS: dict = {}


def _workspace(dev, numel: int, slot: int = 0) -> torch.Tensor:
    """Per-device scratch for split-K partials (stream-ordered reuse)."""
    key = (str(dev), slot)
    w = _WS.get(key)
    if w is None or w.numel() < numel:
        w = torch.empty((numel,), dtype=torch.float32, device=dev)
        _WS[key] = w
    return w


def gemm(A: torch.Tensor, B: torch.Tensor, bias=None, act: int = 0, ta: bool = False, tb: bool = False,
         out: torch.Tensor | None = None, beta_c: float = 0.0) -> torch.Tensor:
    """C = act(op(A) op(B) + bias) with row-major fp32 operands."""
    M = A.shape[1] if ta else A.shape[0]
    K = A.shape[0] if ta else A.shape[1]
    N = B.shape[0] if tb else B.shape[1]
    if A.is_cuda:
        # the kernel indexes dense row-major operands: copy strided views (no-op otherwise)
        A = A.float().contiguous()
        B = B.float().contiguous()
        if bias is not None:
            bias = bias.float().contiguous()
        C = out if out is not None else torch.empty((M, N), dtype=torch.float32, device=A.device)
        if not C.is_contiguous():
            raise ValueError("gemm: out must be contiguous")
        # split-K when the output has too few 128x128 tiles to fill 256 CUs
        # (weight gradients: [out][in] outputs with K = batch rows)
        tiles = -(-M // 128) * -(-N // 128)
        S = 1
        if tiles < 128 and K >= 1024:
            S = max(1, min(64, 256 // tiles, K // 256))
        ws = _workspace(A.device, S * M * N) if S > 1 else None
        check(dense_lib().h2omx_gemm(P(A), P(B), P(C), P(bias), M, N, K, int(ta), int(tb), act, beta_c, S, P(ws),
                                 stream(A.device)), "gemm")
        return C
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
    if act == 0:
        return dY
    if Y.is_cuda:
        check(dense_lib().h2omx_act_backward(P(Y), P(dY), Y.numel(), act, stream(Y.device)), "act_backward")
        return dY
    if act == 1:
        dY.mul_((Y > 0).float())
    elif act == 2:
        dY.mul_(1 - Y * Y)
    return dY


def bias_grad(dY: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    M, N = dY.shape
    if dY.is_cuda:
        db = out if out is not None else torch.empty((N,), dtype=torch.float32, device=dY.device)
        # enough (64-column x row-slice) blocks to fill the GPU, few enough that
        # the second stage sums a short column
        splits = max(1, min(32, M // 256, 1024 // max(1, -(-N // 64))))
        ws = _workspace(dY.device, splits * N, slot=1)
        check(dense_lib().h2omx_bias_grad(P(dY), P(db), M, N, P(ws), splits, stream(dY.device)), "bias_grad")
        return db
    r = dY.sum(0)
    if out is not None:
        out.copy_(r)
        return out
    return r


def softmax_xent(Z: torch.Tensor, y: torch.Tensor):
    """Z [M][K] logits, y int32 class ids -> (dZ = (softmax - onehot) / M, mean loss)."""
    M, K = Z.shape
    if Z.is_cuda:
        y = y.to(torch.int32).contiguous()
        dZ = torch.empty_like(Z)
        loss = torch.zeros((1,), dtype=torch.float32, device=Z.device)
        check(dense_lib().h2omx_softmax_xent(P(Z), P(y), P(dZ), P(loss), M, K, stream(Z.device)), "softmax_xent")
        return dZ, loss
    pr = torch.softmax(Z, 1)
    oh = torch.nn.functional.one_hot(y.long(), K).float()
    loss = -(torch.log(pr.clamp_min(1e-30)) * oh).sum(1).mean()
    return (pr - oh) / M, loss.reshape(1)


def adadelta_(W, G, Eg2, Edx2, rho=0.99, eps=1e-8, l2=0.0):
    if W.is_cuda:
        check(dense_lib().h2omx_adadelta(P(W), P(G), P(Eg2), P(Edx2), W.numel(), rho, eps, l2, stream(W.device)),
              "adadelta")
        return
    g = G + l2 * W
    Eg2.mul_(rho).add_((1 - rho) * g * g)
    dx = -torch.sqrt(Edx2 + eps) / torch.sqrt(Eg2 + eps) * g
    Edx2.mul_(rho).add_((1 - rho) * dx * dx)
    W.add_(dx)


def sgd_momentum_(W, G, V, lr, mom, l2=0.0):
    if W.is_cuda:
        check(dense_lib().h2omx_sgd_momentum(P(W), P(G), P(V), W.numel(), lr, mom, l2, stream(W.device)), "sgd")
        return
    V.mul_(mom).sub_(lr * (G + l2 * W))
    W.add_(V)


# ---------------------------------------------------------------------------
# bf16 MLP path (csrc/dense_kernels.hip gemm_bf16_nt_kernel): operands are
# torch.bfloat16 row-major matrices whose row strides are multiples of 8
# elements (16-byte rows, zero-padded K).  GPU only: on CPU tensors the same
# contract is computed in fp32 from the bf16 values (test oracle).
# ---------------------------------------------------------------------------
def gemm_bf16_nt(A: torch.Tensor, B: torch.Tensor, M: int, N: int, K: int, *, bias=None, act: int = 0,
                 ymask: torch.Tensor | None = None, mask_act: int = 0, out_f32: torch.Tensor | None = None,
                 out_bf16: torch.Tensor | None = None, out_bf16_t: torch.Tensor | None = None,
                 beta_c: float = 0.0, splitk: int = 1, c_last: torch.Tensor | None = None) -> None:
    """C[m][n] = sum_{k<K} A[m][k] B[n][k] (fp32 accumulate), epilogue
    act(C + bias), optionally times act'(ymask) (1 relu, 2 tanh), written to
    out_f32 [M][>=N] and/or out_bf16 [M][>=N] and/or out_bf16_t [N][>=M].
    With ``c_last`` (plain products only) column N-1 goes to c_last [M] and
    out_f32 receives columns < N-1: a weight gradient and, through a ones row
    appended to B, its bias gradient in one GEMM.
    Views with unit inner stride; A/B/out row strides multiples of 8."""
    for t in (A, B):
        assert t.dtype == torch.bfloat16 and t.stride(-1) == 1
    if A.is_cuda:
        ldc = (out_f32 if out_f32 is not None else out_bf16).stride(0) if (out_f32 is not None or out_bf16 is not None) else N
        if out_f32 is not None and out_bf16 is not None:
            assert out_f32.stride(0) == out_bf16.stride(0)
        ws = _workspace(A.device, splitk * M * N, slot=1) if splitk > 1 else None
        check(dense_lib().h2omx_gemm_bf16(
            P(A), A.stride(0), P(B), B.stride(0), M, N, K, P(bias), act, P(ymask),
            ymask.stride(0) if ymask is not None else 0, mask_act, P(out_f32), P(out_bf16), ldc, P(out_bf16_t),
            out_bf16_t.stride(0) if out_bf16_t is not None else 0, float(beta_c), splitk, P(ws), P(c_last),
            stream(A.device)), "gemm_bf16")
        return
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
    """fp32 [R][C] -> bf16 out [R][>=C] (pad columns zeroed up to out's row
    stride) and/or bf16 out_t [C][>=R]."""
    R, C = X.shape
    assert X.stride(-1) == 1
    if X.is_cuda:
        check(dense_lib().h2omx_cvt_bf16(P(X), X.stride(0), R, C, P(out), out.stride(0) if out is not None else 0,
                                         P(out_t), out_t.stride(0) if out_t is not None else 0, stream(X.device)),
              "cvt_bf16")
        return
    if out is not None:
        out[:R, :C] = X.to(torch.bfloat16)
        if out.shape[1] > C:
            out[:R, C:] = 0
    if out_t is not None:
        out_t[:C, :R] = X.T.to(torch.bfloat16)


def rowsum_bf16(X: torch.Tensor, R: int, C: int, out: torch.Tensor) -> None:
    """out[r] = sum_{c<C} X[r][c] (fp32) for a bf16 matrix (bias gradients from dZ^T)."""
    if X.is_cuda:
        check(dense_lib().h2omx_rowsum_bf16(P(X), X.stride(0), R, C, P(out), stream(X.device)), "rowsum_bf16")
        return
    out[:R] = X[:R, :C].float().sum(1)


class _CvtJob(ctypes.Structure):
    _fields_ = [("X", ctypes.c_void_p), ("out", ctypes.c_void_p), ("outT", ctypes.c_void_p), ("ldx", ctypes.c_int),
                ("R", ctypes.c_int), ("C", ctypes.c_int), ("ldo", ctypes.c_int), ("ldot", ctypes.c_int),
                ("pad", ctypes.c_int * 3)]


def cvt_bf16_multi(jobs) -> None:
    """Several ``cvt_bf16(X, out, out_t)`` conversions (<= 8) in one launch."""
    jobs = list(jobs)
    if not jobs:
        return
    if not jobs[0][0].is_cuda:
        for X, out, out_t in jobs:
            cvt_bf16(X, out, out_t)
        return
    arr = (_CvtJob * len(jobs))()
    mr = mc = 1
    for k, (X, out, out_t) in enumerate(jobs):
        R, C = X.shape
        arr[k] = _CvtJob(X.data_ptr(), P(out) or 0, P(out_t) or 0, X.stride(0), R, C,
                         out.stride(0) if out is not None else 0, out_t.stride(0) if out_t is not None else 0)
        mr = max(mr, R)
        mc = max(mc, C, out.stride(0) if out is not None else 0)
    check(dense_lib().h2omx_cvt_bf16_multi(ctypes.addressof(arr), len(jobs), mr, mc, stream(jobs[0][0].device)),
          "cvt_bf16_multi")


def softmax_xent_bf16(Z: torch.Tensor, y: torch.Tensor, dZ: torch.Tensor, dZt: torch.Tensor,
                      loss: torch.Tensor) -> None:
    """Softmax cross-entropy of fp32 logits Z [M][K]: bf16 dZ [M][>=K] and dZ^T
    [K][>=M] ((softmax - onehot) / M); mean loss added into loss[0]."""
    M, K = Z.shape
    if Z.is_cuda:
        check(dense_lib().h2omx_softmax_xent_bf16(P(Z), P(y), P(dZ), dZ.stride(0), P(dZt), dZt.stride(0), P(loss), M,
                                                  K, stream(Z.device)), "softmax_xent_bf16")
        return
    g, l = softmax_xent(Z, y)
    dZ[:M, :K] = g.to(torch.bfloat16)
    dZt[:K, :M] = g.T.to(torch.bfloat16)
    loss += l
