"""Python entry points of csrc/dense_kernels.hip (GLM IRLS Gram, K-Means,
MLP GEMM + elementwise).

Device tensors only: every function launches its HIP kernel on the current
stream (``ops.dense_lib()`` raises if the library is missing) and rejects
host tensors.  The CPU reference implementations (test oracle, CPU-only
deployments) live in :mod:`h2omx.reference.dense`; :mod:`h2omx.backend`
routes a call to one or the other by the device of its data.
"""
from __future__ import annotations

import contextlib
import ctypes
import math

import numpy as np
import torch

from .. import _native
from . import P, check, dense_lib, stream

KBADARG = 1  # common.h kBadArg
# workgroups of the fused GLM Gram / K-Means kernels (swept: profiles/r3/dense_pmc/, profiles/r4/dense/)
GLM_WGS = 512
# wave-unit IRLS kernel for p + 2 <= 128 (not multinomial; False: the workgroup
# kernel, which serves wider / multinomial designs); units = independent waves,
# each over a contiguous row range (fp32 within a unit, fp64 across).  Module
# flags, not environment knobs: tests pin each kernel family with them
GLM_WAVE = True
# Gram of the wave path: "split" = exact 3-way bf16 split on the bf16 matrix
# cores (glm_irls_split_kernel); "f32" = fp32 MFMA (glm_irls_wave_kernel, the
# intercept-only pass and the split kernel's test oracle)
GLM_GRAM = "split"
GLM_UNITS = 2048
GLM_UNIT_MIN_ROWS = 512
SLAB_SPLIT = 32          # dense_kernels.hip slab_reduce16_kernel
KM_WGS = 1024
# K-Means Lloyd pass: cluster sums on the fp32 matrix cores (kmeans_mfma_kernel,
# d + 2 <= 128 / 64, k <= 32), else the wave-unit kernel (k <= 32, d <= 128 / 64),
# else the workgroup-tile kernel; the wave kernel's grid is sized for 256 CUs
KM_MFMA = True
KM_WAVE = True
KM_WAVE_CUS = 256
KM_MFMA_WGS = 512

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


def _dev(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise ValueError(f"ops.dense.{what}: device tensors only (CPU runs go through h2omx.backend -> "
                         "h2omx.reference.dense)")


def _tp_for(p: int) -> int:
    for tp in (1, 2, 4, 8):
        if p + 2 <= 32 * tp:
            return tp
    raise ValueError(f"GLM with {p} predictors exceeds the 254-column fused Gram kernel")


def _glm_irls_wide(X, y, wprior, offset, beta, family, link, cls, var_power, link_power):
    """IRLS pass for p > 254 (e.g. one-hot categoricals with hundreds of levels):
    chunked eta GEMM -> glm_wz_kernel -> glm_aug_kernel -> Gram GEMM A A^T on the
    fp32 MFMA gemm_kernel, fp32 per chunk, fp64 across chunks (slab_sum)."""
    lib = dense_lib()
    p, n = X.shape
    K = beta.shape[0]
    dev = X.device
    st = stream(dev)
    PA = p + 2
    m_chunk = int(max(4096, min(n, (1 << 27) // PA)))
    nchunks = -(-n // m_chunk)
    B = torch.from_numpy(np.ascontiguousarray(beta[:, :p], np.float32)).to(dev)
    b_full = torch.from_numpy(np.ascontiguousarray(beta, np.float32)).to(dev)
    means = torch.zeros((p,), dtype=torch.float32, device=dev)
    gp = GlmParams(FAMILIES[family], LINKS[link], p, K, cls, 0, var_power, link_power)
    Xc = torch.empty((p * m_chunk,), dtype=torch.float32, device=dev)
    E = torch.empty((K * m_chunk,), dtype=torch.float32, device=dev)
    sw = torch.empty((m_chunk,), dtype=torch.float32, device=dev)
    z = torch.empty((m_chunk,), dtype=torch.float32, device=dev)
    A = torch.empty((PA * m_chunk,), dtype=torch.float32, device=dev)
    grams = torch.empty((nchunks, PA * PA), dtype=torch.float32, device=dev)
    n_blk = 256
    devs = torch.empty((nchunks * n_blk,), dtype=torch.float64, device=dev)
    Xs = X.contiguous()
    for ci in range(nchunks):
        s0 = ci * m_chunk
        m = min(m_chunk, n - s0)
        xc = Xc[: p * m].view(p, m)
        check(lib.h2omx_kmeans_stage(P(Xs), Xs.stride(0), p, s0, m, P(xc), st), "stage")
        e = E[: K * m].view(K, m)
        gemm(B, xc, out=e)
        yy = y[s0: s0 + m]
        wp = None if wprior is None else wprior[s0: s0 + m]
        of = None if offset is None else offset[s0: s0 + m]
        check(lib.h2omx_glm_wz(P(e), m, P(yy), P(wp), P(of), P(b_full), ctypes.addressof(gp), P(sw), P(z),
                               P(devs[ci * n_blk:]), n_blk, st), "glm_wz")
        a = A[: PA * m].view(PA, m)
        check(lib.h2omx_glm_aug(P(xc), p, m, P(means), P(sw), P(z), P(a), st), "glm_aug")
        gemm(a, a, tb=True, out=grams[ci].view(PA, PA))
    out = torch.empty((PA * PA,), dtype=torch.float64, device=dev)
    check(lib.h2omx_slab_sum(P(grams), nchunks, PA * PA, P(out), st), "slab_sum")
    G = out.view(PA, PA).cpu().numpy()
    G = 0.5 * (G + G.T)
    return G, float(devs.sum().item())


def glm_irls_pass(X: torch.Tensor, y: torch.Tensor, wprior, offset, beta: np.ndarray, family: str, link: str,
                  cls: int = 0, var_power: float = 1.5, link_power: float = 0.0):
    """One IRLS pass.  X: feature-major standardized float32 [p][n] (no NA).
    beta: float64 [K][p+1] (coefficients then intercept).
    Returns (G float64 [p+2][p+2] of the augmented [x | 1 | z] weighted Gram, deviance)."""
    _dev(X, "glm_irls_pass")
    p, n = X.shape
    K = beta.shape[0]
    if p + 2 > 256:
        return _glm_irls_wide(X, y, wprior, offset, beta, family, link, cls, var_power, link_power)
    lib = dense_lib()
    dev = X.device
    if GLM_WAVE and family != "multinomial" and p + 2 <= 128:
        return _glm_irls_wave(X, y, wprior, offset, beta, family, link, cls, var_power, link_power)
    tp = _tp_for(p)
    PP = 32 * tp
    n_wg = max(1, min(GLM_WGS, math.ceil(n / 4096)))
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


def glm_grad_pass(X: torch.Tensor, y: torch.Tensor, wprior, offset, beta: np.ndarray, family: str, link: str,
                  var_power: float = 1.5, link_power: float = 0.0):
    """Gradient pass of the GLM objective (solver L_BFGS): no Gram, two streaming
    HIP kernels over the feature-major design (glm_resid_kernel, glm_xtr_kernel).
    beta: float64 [K][p+1].  Returns (g float64 [K][p+1] = sum_i r_ki [x_i | 1],
    deviance); r = w (mu - y) mu' / V(mu) (multinomial: w (p_k - [y = k])), so
    d(deviance / 2) / d beta = g."""
    _dev(X, "glm_grad_pass")
    lib = dense_lib()
    p, n = X.shape
    K = beta.shape[0]
    if K > lib.h2omx_glm_grad_max_k():
        raise ValueError(f"glm_grad_pass: {K} classes > {lib.h2omx_glm_grad_max_k()} per pass")
    dev = X.device
    Xc = X if X.stride(1) == 1 else X.contiguous()
    R = _workspace(dev, K * n, slot=3)
    n_blk = int(max(1, min(2048, -(-n // 1024))))
    splits = int(max(1, min(64, -(-n // (1 << 16)), 4096 // max(p + 1, 1))))
    devs = torch.empty((n_blk,), dtype=torch.float64, device=dev)
    out = torch.empty((splits * K * (p + 1),), dtype=torch.float64, device=dev)
    b64 = torch.from_numpy(np.ascontiguousarray(beta, np.float64)).to(dev)
    gp = GlmParams(FAMILIES[family], LINKS[link], p, K, 0, 0, var_power, link_power)
    check(lib.h2omx_glm_grad(P(Xc), Xc.stride(0), n, P(b64), P(y), P(wprior), P(offset), ctypes.addressof(gp), P(R),
                             P(devs), n_blk, P(out), splits, stream(dev)), "glm_grad")
    g = out.view(splits, K, p + 1).cpu().numpy().sum(0)
    return g, float(devs.sum().item())


def _glm_irls_wave(X, y, wprior, offset, beta, family, link, cls, var_power, link_power):
    """glm_irls_split_kernel (GLM_GRAM "split": exact three-way bf16 split, 6
    bf16 MFMAs per 16x16 tile, designs staged through LDS by LDS-DMA) or
    glm_irls_wave_kernel ("f32", and the intercept-only p = 0 pass: 16x16x4 fp32
    MFMA): independent wave units over contiguous row ranges, register-resident
    32-row chunks, then the fp64 sum of the per-unit upper tiles.  X has no NA
    (the GLM imputes column means before the pass)."""
    lib = dense_lib()
    p, n = X.shape
    K = beta.shape[0]
    dev = X.device
    pw = 16 * math.ceil((p + 2) / 16)
    units = max(1, min(GLM_UNITS, math.ceil(n / GLM_UNIT_MIN_ROWS)))
    rows = max(32, -(-math.ceil(n / units) // 32) * 32)
    units = max(1, math.ceil(n / rows))
    slab = torch.empty((units * pw * pw,), dtype=torch.float32, device=dev)
    devs = torch.empty((units,), dtype=torch.float64, device=dev)
    # sum [pw * pw] | the deviance | SLAB_SPLIT partials (h2omx_slab_reduce16_dev)
    out = torch.empty(((SLAB_SPLIT + 1) * pw * pw + 1,), dtype=torch.float64, device=dev)
    b32 = _pinned_to(np.ascontiguousarray(beta, np.float32).ravel(), dev)
    split = GLM_GRAM == "split" and p >= 1
    means = None if split else torch.zeros((max(p, 1),), dtype=torch.float32, device=dev)
    gp = GlmParams(FAMILIES[family], LINKS[link], p, K, cls, 0, var_power, link_power)
    Xc = X if X.stride(1) == 1 else X.contiguous()
    st = stream(dev)
    fn = lib.h2omx_glm_irls_split if split else lib.h2omx_glm_irls_wave
    check(fn(P(Xc), Xc.stride(0), n, P(y), P(wprior), P(offset), P(means), P(b32),
             ctypes.addressof(gp), units, rows, P(slab), P(devs), st), "glm_irls_wave")
    # the Gram and the deviance come back in ONE device -> host copy (one sync)
    check(lib.h2omx_slab_reduce16_dev(P(slab), units, pw, P(devs), P(out), st), "slab_reduce16_dev")
    host = out[: pw * pw + 1].cpu().numpy()
    G = host[: pw * pw].reshape(pw, pw)[: p + 2, : p + 2]
    G = np.triu(G) + np.triu(G, 1).T
    return G, float(host[pw * pw])


# ---------------------------------------------------------------------------
# K-Means
# ---------------------------------------------------------------------------
def kmeans_step(X: torch.Tensor, C, na_free: bool = False):
    """One Lloyd pass.  X feature-major float32 [d][n] (standardized; NA cells
    count as 0 unless ``na_free`` asserts there are none), C [k][d] (tensor, or
    a host array: the MFMA path then builds its padded centroid tables on the
    host and uploads them in one copy).
    Returns (assign int32 [n], sums float64 [k][d], counts [k], sse [k])."""
    _dev(X, "kmeans_step")
    d, n = X.shape
    k = C.shape[0]
    lib = dense_lib()
    dev = X.device
    Xc = X.contiguous()
    width = k * d + 2 * k
    kp = -(-k // 4) * 4 if k <= 16 else -(-k // 8) * 8
    nt = -(-(d + 2) // 16)
    if isinstance(C, np.ndarray):
        if KM_MFMA and k <= 32 and nt <= (8 if kp <= 16 else 4):
            Cf = np.ascontiguousarray(C, np.float32)
            Cp = np.zeros((kp, 16 * nt), np.float32)
            Cp[:k, :d] = Cf
            cnp = np.full((kp,), np.inf, np.float32)
            cnp[:k] = (Cf.astype(np.float64) ** 2).sum(1).astype(np.float32)
            tab = _pinned_to(np.concatenate([Cp.reshape(kp, 8 * nt, 2).transpose(1, 0, 2).ravel(), cnp]), dev)
            return _kmeans_mfma(Xc, d, n, k, kp, nt, tab[: kp * 16 * nt], tab[kp * 16 * nt:], na_free, width)
        C = torch.from_numpy(np.ascontiguousarray(C, np.float32)).to(dev)
    Cc = C.float().contiguous()
    cn = (Cc.double() ** 2).sum(1).float()
    out = torch.empty((width,), dtype=torch.float64, device=dev)
    assign = torch.empty((n,), dtype=torch.int32, device=dev)
    st = stream(dev)
    dp = -(-d // 16) * 16
    if KM_MFMA and k <= 32 and nt <= (8 if kp <= 16 else 4):
        # csrc/kmeans_wave.hip kmeans_mfma_kernel: centroids by feature pair
        # CT2 [8 nt][kp][2] (zero padding), +inf norms for the padding clusters
        Cp = torch.zeros((kp, 16 * nt), dtype=torch.float32, device=dev)
        Cp[:k, :d] = Cc
        CT2 = Cp.view(kp, 8 * nt, 2).permute(1, 0, 2).contiguous()
        cnp = torch.full((kp,), float("inf"), dtype=torch.float32, device=dev)
        cnp[:k] = cn
        return _kmeans_mfma(Xc, d, n, k, kp, nt, CT2, cnp, na_free, width)
    elif KM_WAVE and k <= 32 and (dp <= 128 if kp <= 16 else dp <= 64):
        # wave-unit kernel (csrc/dense_kernels.hip kmeans_wave_kernel): zero-padded
        # centroids [kp][dp], +inf norms for the padding clusters
        Cp = torch.zeros((kp, dp), dtype=torch.float32, device=dev)
        Cp[:k, :d] = Cc
        cnp = torch.full((kp,), float("inf"), dtype=torch.float32, device=dev)
        cnp[:k] = cn
        CT = Cp.t().contiguous()   # [dp][kp]: one feature's centroid values per scalar load
        # one workgroup (4 waves) per CU at dp = 128 (LDS tiles 4 x dp x 65 floats);
        # smaller tiles fit more per CU.  >= ~4 chunks of 64 rows per wave
        per_cu = max(1, (160 * 1024) // ((4 * dp * 65 + dp * kp) * 4))
        n_wg = max(1, min(KM_WAVE_CUS * per_cu, math.ceil(n / (64 * 4 * 4))))
        slab = torch.empty((4 * n_wg * width,), dtype=torch.float32, device=dev)
        check(lib.h2omx_kmeans_wave(P(Xc), Xc.stride(0), n, d, P(Cp), P(CT), P(cnp), k, kp, dp, n_wg, P(assign), P(slab),
                                    st), "kmeans_wave")
        check(lib.h2omx_slab_sum(P(slab), 4 * n_wg, width, P(out), st), "slab_sum")
    else:
        n_wg = max(1, min(KM_WGS, math.ceil(n / 4096)))
        slab = torch.empty((n_wg * width,), dtype=torch.float32, device=dev)
        rc = lib.h2omx_kmeans(P(Xc), Xc.stride(0), n, d, P(Cc), P(cn), k, n_wg, P(assign), P(slab), st)
        if rc == KBADARG:
            return _kmeans_large(Xc, Cc)
        check(rc, "kmeans")
        check(lib.h2omx_slab_sum(P(slab), n_wg, width, P(out), st), "slab_sum")
    o = out.cpu().numpy()
    return assign, o[: k * d].reshape(k, d), o[k * d: k * d + k], o[k * d + k:]


def _kmeans_mfma(Xc, d, n, k, kp, nt, CT2, cnp, na_free, width):
    """kmeans_mfma_kernel + the fp64 slab sum; one device -> host copy"""
    lib = dense_lib()
    dev = Xc.device
    st = stream(dev)
    out = torch.empty((width,), dtype=torch.float64, device=dev)
    assign = torch.empty((n,), dtype=torch.int32, device=dev)
    n_wg = max(1, min(KM_MFMA_WGS, math.ceil(n / (64 * 4 * 4))))
    slab = torch.empty((4 * n_wg * width,), dtype=torch.float32, device=dev)
    check(lib.h2omx_kmeans_mfma(P(Xc), Xc.stride(0), n, d, P(CT2), P(cnp), k, kp, nt, 0 if na_free else 1, n_wg,
                                P(assign), P(slab), st), "kmeans_mfma")
    check(lib.h2omx_slab_sum(P(slab), 4 * n_wg, width, P(out), st), "slab_sum")
    o = out.cpu().numpy()
    return assign, o[: k * d].reshape(k, d), o[k * d: k * d + k], o[k * d + k:]


def _kmeans_large(X: torch.Tensor, C: torch.Tensor):
    """Shapes beyond the fused kernel's LDS tiles (d > 256 or k > 128), all on
    our HIP kernels: per row chunk the distance GEMM C x Xc and the sums GEMM
    OH x Xc^T on the fp32 MFMA gemm_kernel, argmin / one-hot / staging kernels
    in between (csrc/dense_kernels.hip, "K-Means beyond the fused kernel")."""
    lib = dense_lib()
    d, n = X.shape
    k = C.shape[0]
    dev = X.device
    st = stream(dev)
    Cc = C.float().contiguous()
    cn = (Cc.double() ** 2).sum(1).float().contiguous()
    # chunk so G / OH ([k][m]) and Xc ([d][m]) stay within ~1.5 GB of the 288 GB HBM
    m_chunk = int(max(4096, min(n, (1 << 27) // max(k, d))))
    nchunks = -(-n // m_chunk)
    assign = torch.empty((n,), dtype=torch.int32, device=dev)
    n_blk = 256
    stat = torch.empty((nchunks * n_blk * 2 * k,), dtype=torch.float32, device=dev)
    sums = torch.empty((nchunks, k * d), dtype=torch.float32, device=dev)
    Xc = torch.empty((d * m_chunk,), dtype=torch.float32, device=dev)
    G = torch.empty((k * m_chunk,), dtype=torch.float32, device=dev)
    for ci in range(nchunks):
        s0 = ci * m_chunk
        m = min(m_chunk, n - s0)
        xc = Xc[: d * m].view(d, m)
        g = G[: k * m].view(k, m)
        check(lib.h2omx_kmeans_stage(P(X), X.stride(0), d, s0, m, P(xc), st), "kmeans_stage")
        gemm(Cc, xc, out=g)
        a = assign[s0: s0 + m]
        check(lib.h2omx_kmeans_argmin(P(g), k, m, P(cn), P(xc), d, P(a), P(stat[ci * n_blk * 2 * k:]), n_blk, st),
              "kmeans_argmin")
        check(lib.h2omx_kmeans_onehot(P(a), k, m, P(g), st), "kmeans_onehot")    # G reused as OH
        gemm(g, xc, tb=True, out=sums[ci].view(k, d))
    o_stat = torch.empty((2 * k,), dtype=torch.float64, device=dev)
    check(lib.h2omx_slab_sum(P(stat), nchunks * n_blk, 2 * k, P(o_stat), st), "slab_sum")
    o_sums = torch.empty((k * d,), dtype=torch.float64, device=dev)
    check(lib.h2omx_slab_sum(P(sums), nchunks, k * d, P(o_sums), st), "slab_sum")
    o_stat = o_stat.cpu().numpy()
    return assign, o_sums.cpu().numpy().reshape(k, d), o_stat[:k], o_stat[k:]


# ---------------------------------------------------------------------------
# MLP building blocks
# ---------------------------------------------------------------------------
ACTS = {"linear": 0, "none": 0, "rectifier": 1, "relu": 1, "tanh": 2}  # maxout: models/deeplearning.py


_WS: dict = {}
_WS_RETIRED: list = []


_WS_NS = [0]


@contextlib.contextmanager
def workspace_ns(ns: int):
    """Scratch namespace for the ops issued inside: work that may run
    concurrently on another stream (the DL backward's weight-gradient side
    stream) takes a namespace of its own, so no two in-flight kernels share a
    workspace."""
    old = _WS_NS[0]
    _WS_NS[0] = ns
    try:
        yield
    finally:
        _WS_NS[0] = old


# deferred gradient folds (see defer_grad_folds): [(grad view, ws, splits, stride)]
_GRAD_FOLDS: list = [None]


@contextlib.contextmanager
def defer_grad_folds():
    """Inside: wgrad_bias (small path) and out_wgrad leave their last reduction
    (bias-gradient slices, the output layer's split partial rows) as pending
    folds instead of launching it; :func:`adadelta_` with ``folds`` performs
    them inside the optimizer kernel.  Yields the list of pending folds.  The
    workspaces must stay untouched until then (per-layer workspace_ns)."""
    old = _GRAD_FOLDS[0]
    _GRAD_FOLDS[0] = []
    try:
        yield _GRAD_FOLDS[0]
    finally:
        _GRAD_FOLDS[0] = old


_PINNED: dict = {}


def _pinned_to(a: np.ndarray, dev) -> torch.Tensor:
    """Small host array -> device through a reused pinned staging buffer (an
    asynchronous copy on the current stream; callers sync before the next
    reuse, e.g. the GLM pass reads its result back)."""
    key = (str(dev), a.dtype.str, a.size)
    hb = _PINNED.get(key)
    if hb is None:
        hb = torch.empty((a.size,), dtype=torch.from_numpy(a[:0]).dtype).pin_memory()
        _PINNED[key] = hb
    hb.numpy()[:] = a
    return hb.to(dev, non_blocking=True)


def _workspace(dev, numel: int, slot: int = 0) -> torch.Tensor:
    """Per-device scratch for split-K partials (stream-ordered reuse within a
    namespace, see workspace_ns).  A grown workspace keeps its predecessor
    alive: a captured HIP graph (DL training step) may still hold the old pointer."""
    key = (str(dev), slot, _WS_NS[0])
    w = _WS.get(key)
    if w is None or w.numel() < numel:
        if w is not None:
            _WS_RETIRED.append(w)
        w = torch.empty((numel,), dtype=torch.float32, device=dev)
        _WS[key] = w
    return w


def gemm(A: torch.Tensor, B: torch.Tensor, bias=None, act: int = 0, ta: bool = False, tb: bool = False,
         out: torch.Tensor | None = None, beta_c: float = 0.0) -> torch.Tensor:
    """C = act(op(A) op(B) + bias) with row-major fp32 operands."""
    M = A.shape[1] if ta else A.shape[0]
    K = A.shape[0] if ta else A.shape[1]
    N = B.shape[0] if tb else B.shape[1]
    _dev(A, "gemm")
    # the kernel indexes dense row-major operands: copy strided views (no-op otherwise)
    A = A.float().contiguous()
    B = B.float().contiguous()
    if bias is not None:
        bias = bias.float().contiguous()
    C = out if out is not None else torch.empty((M, N), dtype=torch.float32, device=A.device)
    if not C.is_contiguous():
        raise ValueError("gemm: out must be contiguous")
    if beta_c == 0.0 and not ta:
        if tb and N <= 8 and K >= 16:
            # skinny output (classifier layer): one wave per row, no 128 x 128 tile of zeros
            check(dense_lib().h2omx_gemm_skinny_nt(P(A), P(B), P(C), P(bias), M, N, K, act, stream(A.device)),
                  "gemm_skinny_nt")
            return C
        if not tb and K <= 8 and bias is None and act == 0:
            check(dense_lib().h2omx_gemm_thin_k(P(A), P(B), P(C), M, N, K, None, 0, stream(A.device)),
                  "gemm_thin_k")
            return C
    if X3_GEMM and not ta and tb and beta_c == 0.0 and M * N * K >= X3_MIN_MNK and _x3_ok(A, B, C):
        # large forward layers: the x3 bf16-split kernel on the bf16 matrix cores
        # (fp32-equivalent accuracy; 8192 x 512 x 512 + ReLU 40.1 us vs 56.6 us for
        # gemm_w64 and 41.0 us for hipBLASLt, profiles/r5/dl/gemm_x3_r5o.jsonl)
        from .mlp import gemm_x3

        return gemm_x3(A, B, bias, act, out=C)
    return gemm_fp32(A, B, bias, act, ta, tb, C, beta_c)


def gemm_fp32(A: torch.Tensor, B: torch.Tensor, bias=None, act: int = 0, ta: bool = False, tb: bool = False,
              out: torch.Tensor | None = None, beta_c: float = 0.0) -> torch.Tensor:
    """:func:`gemm` on the fp32 MFMA kernels (gemm_w64 / split-K) - every layout."""
    M = A.shape[1] if ta else A.shape[0]
    K = A.shape[0] if ta else A.shape[1]
    N = B.shape[0] if tb else B.shape[1]
    A = A.float().contiguous()
    B = B.float().contiguous()
    if bias is not None:
        bias = bias.float().contiguous()
    C = out if out is not None else torch.empty((M, N), dtype=torch.float32, device=A.device)
    S = _splitk(M, N, K)
    ws = _workspace(A.device, S * M * N) if S > 1 else None
    check(dense_lib().h2omx_gemm(P(A), P(B), P(C), P(bias), M, N, K, int(ta), int(tb), act, beta_c, S, P(ws),
                             stream(A.device)), "gemm")
    return C


# NT GEMMs of at least this many multiply-adds go to the x3 kernel (below it a
# 256-row mini-batch layer runs 13.8 us on gemm_w64 vs 34.4 us on x3: too few tiles)
X3_GEMM = True
X3_MIN_MNK = 1 << 27
# hidden-layer data gradients (gemm_dact) on the x3 kernel as well
X3_DACT = True


def _x3_ok(A, B, C) -> bool:
    K = A.shape[1]
    return (K % 4 == 0 and A.data_ptr() % 16 == 0 and B.data_ptr() % 16 == 0 and C.is_contiguous()
            and _native.available("mlp"))


def set_gemm_tile(tile: int) -> None:
    """fp32 GEMM tile edge: 0 = by shape (64 x 64 when 128 x 128 tiles would
    leave CUs short of work), 64 or 128 (tests / tuning); 1 / 2 = 64 x 64 wave
    tiles on 128 x 128 / 128 x 64 blocks (gemm_w64_kernel)."""
    check(dense_lib().h2omx_gemm_set_tile(int(tile)), "gemm_set_tile")


def set_gemm_full(on: int) -> None:
    """gemm_w64_kernel's whole-tile fast path (unchecked loads, XCD-aware tile
    order, mid-step LDS writes) when the shape allows it; 0 = always the checked
    kernel (A/B measurements)."""
    check(dense_lib().h2omx_gemm_set_full(int(on)), "gemm_set_full")


def _row_splits(M: int, N: int) -> int:
    # 256-column blocks x row slices of >= 64 rows: ~512 workgroups
    return max(1, min(256, M // 64, 512 // max(1, -(-N // 256))))


def out_layer_ok(dZ: torch.Tensor, H: torch.Tensor) -> bool:
    """few-class output layer (C <= 8) over a float4-aligned hidden width:
    streaming weight-gradient / activation-backward kernels instead of GEMMs"""
    return dZ.shape[1] <= 8 and H.shape[1] % 4 == 0 and H.is_contiguous()


def _grad_span(dW: torch.Tensor, db: torch.Tensor) -> bool:
    """db directly follows dW inside ONE storage (a layer's [W | b] span of the
    flat gradient), not merely at the next address of another allocation."""
    return (db.data_ptr() == dW.data_ptr() + dW.numel() * dW.element_size()
            and db.untyped_storage().data_ptr() == dW.untyped_storage().data_ptr())


def out_wgrad(dZ: torch.Tensor, H: torch.Tensor, dW: torch.Tensor, db: torch.Tensor) -> None:
    """dW [C][N] = dZ^T H and db = column sums of dZ for C <= 8 classes (one
    streaming pass over H, fixed-order split reduce)."""
    M, C = dZ.shape
    N = H.shape[1]
    _dev(dZ, "out_wgrad")
    S = _row_splits(M, N)
    T = C * N + C
    ws = _workspace(dZ.device, S * T)
    contiguous = (dW.is_contiguous() and db.is_contiguous()
                  and _grad_span(dW, db))
    out = dW.view(-1) if contiguous else torch.empty((T,), dtype=torch.float32, device=dZ.device)
    if contiguous:
        # the layer's [W | b] gradient span (models/deeplearning.py _Net): write it in place
        out = torch.as_strided(dW, (T,), (1,))
        if _GRAD_FOLDS[0] is not None and len(_GRAD_FOLDS[0]) < 8:
            check(dense_lib().h2omx_out_wgrad_partial(P(dZ.contiguous()), P(H), P(ws), M, N, C, S, stream(dZ.device)),
                  "out_wgrad_partial")
            _GRAD_FOLDS[0].append((out, ws, S, T))
            return
    check(dense_lib().h2omx_out_wgrad(P(dZ.contiguous()), P(H), P(out), P(ws), M, N, C, S, stream(dZ.device)),
          "out_wgrad")
    if not contiguous:
        dW.copy_(out[: C * N].view(C, N))
        db.copy_(out[C * N:])


def out_backward(dZ: torch.Tensor, H: torch.Tensor, W: torch.Tensor, dW: torch.Tensor, db: torch.Tensor, act: int):
    """The few-class output layer's backward in one pass (inside
    defer_grad_folds only): its weight / bias gradient partial rows become a
    pending fold into the contiguous [dW | db] span, and dZ_prev = (dZ W) *
    act'(H) comes back with its bias-gradient slices (like thin_dact)."""
    M, C = dZ.shape
    N = H.shape[1]
    _dev(dZ, "out_backward")
    S = _row_splits(M, N)
    T = C * N + C
    wsw = _workspace(dZ.device, S * T)
    wsb = _workspace(dZ.device, S * N, slot=1)
    out = torch.empty((M, N), dtype=torch.float32, device=dZ.device)
    check(dense_lib().h2omx_out_backward(P(dZ.contiguous()), P(H), P(W.contiguous()), P(out), P(wsw), P(wsb), M, N,
                                         C, S, int(act), stream(dZ.device)), "out_backward")
    _GRAD_FOLDS[0].append((torch.as_strided(dW, (T,), (1,)), wsw, S, T))
    return out, (wsb, S)


def out_backward_ok(dZ: torch.Tensor, H: torch.Tensor, dW: torch.Tensor, db: torch.Tensor) -> bool:
    return (_GRAD_FOLDS[0] is not None and len(_GRAD_FOLDS[0]) < 8 and out_layer_ok(dZ, H)
            and dW.is_contiguous() and db.is_contiguous()
            and _grad_span(dW, db))


def thin_dact(dZ: torch.Tensor, W: torch.Tensor, Y: torch.Tensor, act: int):
    """dZ_prev = (dZ [M][C] W [C][N]) * act'(Y) and its per-slice column sums
    (bias-gradient partials), one pass; returns (dZ_prev, (ws, splits))."""
    M, C = dZ.shape
    N = W.shape[1]
    _dev(dZ, "thin_dact")
    S = _row_splits(M, N)
    ws = _workspace(dZ.device, S * N, slot=1)
    out = torch.empty((M, N), dtype=torch.float32, device=dZ.device)
    check(dense_lib().h2omx_thin_dact(P(dZ.contiguous()), P(W.contiguous()), P(Y), P(out), P(ws), M, N, C, S,
                                      int(act), stream(dZ.device)), "thin_dact")
    return out, (ws, S)


# gemm_dact's 128 x 64 output blocks needed to prefer it over GEMM + act_backward_bias
# (256-row mini-batches: 16 blocks ran 38 us vs 8 + 5 us, profiles/r4/dl/gemm_dact_small_ab_r4ag.txt)
DACT_MIN_BLOCKS = 128


def dact_ok(dZ: torch.Tensor, W: torch.Tensor) -> bool:
    """gemm_dact (dZ [M][K] x W [K][N]) pays off when its 128 x 64 blocks fill the
    GPU without split-K (small mini-batches keep the split-K GEMM +
    act_backward_bias pair)"""
    M, K = dZ.shape
    N = W.shape[1]
    if M % 128 or N % 64 or K % 4:
        return False
    return (M // 128) * (N // 64) >= DACT_MIN_BLOCKS


def x3_dact_ok(M: int, K: int, N: int, act: int) -> bool:
    """gemm_dact of a [M][K] x [K][N] product takes the x3 route"""
    return X3_DACT and X3_GEMM and M * N * K >= X3_MIN_MNK and act in (1, 2) and K % 4 == 0 and \
        _native.available("mlp")


def x3_dact_layer(M: int, W: torch.Tensor, act: int) -> bool:
    """the data gradient through W ([K][N]) for a batch of M rows runs gemm_dact
    on the x3 route (dact_ok and x3_dact_ok)"""
    K, N = W.shape
    return (M % 128 == 0 and N % 64 == 0 and (M // 128) * (N // 64) >= DACT_MIN_BLOCKS
            and x3_dact_ok(M, K, N, act))


def transpose_weights(Ws) -> list:
    """W^T copies ([in][out]) of the given hidden weights for the x3 data
    gradients, in one launch; scratch per layer (workspace namespace
    2000 + position)."""
    from .mlp import x3_transpose

    outs = []
    for q, W in enumerate(Ws):
        with workspace_ns(2000 + q):
            outs.append(_workspace(W.device, W.numel(), slot=2)[: W.numel()].view(W.shape[1], W.shape[0]))
    x3_transpose([(W.contiguous(), Wt) for W, Wt in zip(Ws, outs)])
    return outs


def gemm_dact(dZ: torch.Tensor, W: torch.Tensor, Y: torch.Tensor, act: int, out: torch.Tensor | None = None,
              tile: int = 2, Wt: torch.Tensor | None = None):
    """Back-propagation through a Rectifier / Tanh layer in one GEMM:
    dZ_prev = (dZ[M][K] W[K][N]) * act'(Y[M][N]) (Y = that layer's output), plus
    the column sums of dZ_prev per 128-row block (its bias gradient before the
    fixed-order fold).  Returns (dZ_prev, (workspace, splits)) like
    :func:`act_backward_bias`."""
    M, K = dZ.shape
    N = W.shape[1]
    _dev(dZ, "gemm_dact")
    if W.shape[0] != K or tuple(Y.shape) != (M, N) or not (dZ.is_contiguous() and W.is_contiguous()
                                                            and Y.is_contiguous()):
        raise ValueError("gemm_dact: needs contiguous dZ [M][K], W [K][N], Y [M][N]")
    C = out if out is not None else torch.empty((M, N), dtype=torch.float32, device=dZ.device)
    if x3_dact_ok(M, K, N, act) and dZ.data_ptr() % 16 == 0 and C.is_contiguous():
        # x3 GEMM on W^T (``Wt`` from transpose_weights, else transposed here)
        # instead of the fp32 MFMA kernel (profiles/r5/dl/x3_dact_ab.txt)
        from .mlp import gemm_x3_dact
        if Wt is None:
            Wt = transpose_weights([W])[0]
        splits = -(-M // 64)
        ws = _workspace(dZ.device, splits * N, slot=1)
        gemm_x3_dact(dZ, Wt, Y, act, ws, out=C)
        return C, (ws, splits)
    splits = -(-M // 128)
    ws = _workspace(dZ.device, splits * N, slot=1)
    sp = ctypes.c_int(0)
    check(dense_lib().h2omx_gemm_dact(P(dZ), P(W), P(C), P(Y), P(ws), M, N, K, int(act), int(tile),
                                      ctypes.addressof(sp), stream(dZ.device)), "gemm_dact")
    return C, (ws, splits)


def _splitk(M: int, N: int, K: int) -> int:
    """split-K when the output has too few tiles to fill 256 CUs: weight
    gradients ([out][in] outputs, K = batch rows) and every GEMM of a small
    mini-batch (256 x 512 x 512: 32 64x64 tiles of 16 serial K-steps each ->
    8 K-splits of 2 steps, ~4x faster)"""
    tiles = -(-M // 128) * -(-N // 128)
    if tiles < 128 and K >= 1024:
        # (about one 128 x 128 tile per CU: 8 or 1024 / tiles splits measured slower,
        # profiles/r5/dl/wgrad_splitk_ab.txt)
        return max(1, min(64, 256 // tiles, K // 256))
    tiles64 = -(-M // 64) * -(-N // 64)
    if tiles64 < 128 and K >= 256:
        return max(1, min(16, 256 // tiles64, K // 64))
    return 1


def _bias_splits(M: int, N: int) -> int:
    # enough (64-column x row-slice) blocks to fill the GPU, few enough that
    # the second stage sums a short column
    return max(1, min(32, M // 256, 1024 // max(1, -(-N // 64))))


def act_backward_bias(Y: torch.Tensor, dY: torch.Tensor, act: int):
    """dZ = dY * act'(Y) in place, plus the per-slice column sums of dZ (the
    layer's bias gradient before its final fixed-order reduce) in one pass.
    Returns (dZ, (workspace, splits)) for :func:`wgrad_bias` / :func:`bias_reduce`."""
    M, N = dY.shape
    _dev(dY, "act_backward_bias")
    if N % 4 or not (Y.is_contiguous() and dY.is_contiguous()):
        act_backward(Y, dY, act)
        return dY, (bias_grad(dY)[None, :], 1)
    # 256-column blocks: enough row slices to put ~512 workgroups on the GPU
    splits = max(1, min(128, M // 32, 512 // max(1, -(-N // 256))))
    ws = _workspace(dY.device, splits * N, slot=1)
    check(dense_lib().h2omx_act_backward_bias(P(Y), P(dY), P(ws), M, N, splits, act, stream(dY.device)),
          "act_backward_bias")
    return dY, (ws, splits)


def wgrad_bias(dZ: torch.Tensor, H: torch.Tensor, dW: torch.Tensor, db: torch.Tensor, bpart) -> None:
    """dW = dZ^T H and db = the reduce of the slices in ``bpart`` (from
    :func:`act_backward_bias`), the bias reduce riding on the split-K reduce launch."""
    K, M = dZ.shape
    N = H.shape[1]
    S = _splitk(M, N, K)
    bws, bsplits = bpart
    if S < 2:
        gemm(dZ, H, ta=True, out=dW)
        if (_GRAD_FOLDS[0] is not None and len(_GRAD_FOLDS[0]) < 8 and db.dtype == torch.float32
                and db.is_contiguous()):
            _GRAD_FOLDS[0].append((db, bws, bsplits, M))
            return
        if db.dtype == torch.float32 and db.is_contiguous():
            check(dense_lib().h2omx_slab_sum_f32(P(bws), bsplits, M, P(db), stream(dZ.device)), "slab_sum_f32")
        else:
            tmp = torch.empty((M,), dtype=torch.float64, device=dZ.device)
            check(dense_lib().h2omx_slab_sum(P(bws), bsplits, M, P(tmp), stream(dZ.device)), "slab_sum")
            db.copy_(tmp)
        return
    ws = _workspace(dZ.device, S * M * N)
    check(dense_lib().h2omx_gemm_wgrad_bias(P(dZ.contiguous()), P(H.contiguous()), P(dW), M, N, K, S, P(ws), P(bws),
                                            bsplits, M, P(db), stream(dZ.device)), "gemm_wgrad_bias")


def act_backward(Y: torch.Tensor, dY: torch.Tensor, act: int) -> torch.Tensor:
    if act == 0:
        return dY
    _dev(Y, "act_backward")
    check(dense_lib().h2omx_act_backward(P(Y), P(dY), Y.numel(), act, stream(Y.device)), "act_backward")
    return dY


def bias_grad(dY: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    M, N = dY.shape
    _dev(dY, "bias_grad")
    db = out if out is not None else torch.empty((N,), dtype=torch.float32, device=dY.device)
    splits = _bias_splits(M, N)
    ws = _workspace(dY.device, splits * N, slot=1)
    check(dense_lib().h2omx_bias_grad(P(dY), P(db), M, N, P(ws), splits, stream(dY.device)), "bias_grad")
    return db


def out_softmax_ok(H: torch.Tensor, W: torch.Tensor) -> bool:
    """the output layer Z = H W^T + b of <= 8 classes runs as gemm_skinny_nt"""
    return W.shape[0] <= 8 and W.shape[1] >= 16 and H.is_cuda


def gemm_softmax_xent(H: torch.Tensor, W: torch.Tensor, b: torch.Tensor, y: torch.Tensor):
    """Output layer and softmax cross-entropy gradient in one launch: returns
    (Z = H W^T + b, dZ = (softmax(Z) - onehot(y)) / M), the same values as
    gemm(...) followed by softmax_xent(..., with_loss=False)."""
    _dev(H, "gemm_softmax_xent")
    M, K = H.shape
    N = W.shape[0]
    H = H.float().contiguous()
    W = W.float().contiguous()
    b = b.float().contiguous()
    y = y.to(torch.int32).contiguous()
    Z = torch.empty((M, N), dtype=torch.float32, device=H.device)
    dZ = torch.empty_like(Z)
    check(dense_lib().h2omx_gemm_skinny_softmax(P(H), P(W), P(Z), P(b), M, N, K, P(y), P(dZ), stream(H.device)),
          "gemm_skinny_softmax")
    return Z, dZ


def softmax_xent(Z: torch.Tensor, y: torch.Tensor, with_loss: bool = True):
    """Z [M][K] logits, y int32 class ids -> (dZ = (softmax - onehot) / M, mean
    loss); ``with_loss=False`` skips the loss (None) and its zero-fill launch."""
    M, K = Z.shape
    _dev(Z, "softmax_xent")
    y = y.to(torch.int32).contiguous()
    dZ = torch.empty_like(Z)
    loss = torch.zeros((1,), dtype=torch.float32, device=Z.device) if with_loss else None
    check(dense_lib().h2omx_softmax_xent(P(Z), P(y), P(dZ), P(loss), M, K, stream(Z.device)), "softmax_xent")
    return dZ, loss


class _GradFix(ctypes.Structure):
    _fields_ = [("off", ctypes.c_int64), ("ws", ctypes.c_void_p), ("len", ctypes.c_int), ("splits", ctypes.c_int),
                ("stride", ctypes.c_int), ("pad", ctypes.c_int)]


class _GradFixes(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("pad", ctypes.c_int), ("f", _GradFix * 8)]


def adadelta_(W, G, Eg2, Edx2, rho=0.99, eps=1e-8, l2=0.0, folds=None):
    """ADADELTA step; ``folds`` (from defer_grad_folds): pending gradient
    reductions, each a view of G summed from its partial rows first."""
    _dev(W, "adadelta_")
    if folds:
        fx = _GradFixes()
        fx.n = len(folds)
        base = G.data_ptr()
        for e, (view, ws, splits, stride) in enumerate(folds):
            fx.f[e].off = (view.data_ptr() - base) // 4
            fx.f[e].ws = ws.data_ptr()
            fx.f[e].len = view.numel()
            fx.f[e].splits = int(splits)
            fx.f[e].stride = int(stride)
        check(dense_lib().h2omx_adadelta_fix(P(W), P(G), P(Eg2), P(Edx2), W.numel(), rho, eps, l2,
                                             ctypes.addressof(fx), stream(W.device)), "adadelta_fix")
        return
    check(dense_lib().h2omx_adadelta(P(W), P(G), P(Eg2), P(Edx2), W.numel(), rho, eps, l2, stream(W.device)),
          "adadelta")


def sgd_momentum_(W, G, V, lr, mom, l2=0.0):
    _dev(W, "sgd_momentum_")
    check(dense_lib().h2omx_sgd_momentum(P(W), P(G), P(V), W.numel(), lr, mom, l2, stream(W.device)), "sgd")


# ---------------------------------------------------------------------------
# bf16 MLP path (csrc/dense_kernels.hip gemm_bf16_nt_kernel): operands are
# torch.bfloat16 row-major matrices whose row strides are multiples of 8
# elements (16-byte rows, zero-padded K).
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
    _dev(A, "gemm_bf16_nt")
    ldc = (out_f32 if out_f32 is not None else out_bf16).stride(0) if (out_f32 is not None or out_bf16 is not None) else N
    if out_f32 is not None and out_bf16 is not None:
        assert out_f32.stride(0) == out_bf16.stride(0)
    ws = _workspace(A.device, splitk * M * N, slot=1) if splitk > 1 else None
    check(dense_lib().h2omx_gemm_bf16(
        P(A), A.stride(0), P(B), B.stride(0), M, N, K, P(bias), act, P(ymask),
        ymask.stride(0) if ymask is not None else 0, mask_act, P(out_f32), P(out_bf16), ldc, P(out_bf16_t),
        out_bf16_t.stride(0) if out_bf16_t is not None else 0, float(beta_c), splitk, P(ws), P(c_last),
        stream(A.device)), "gemm_bf16")


def cvt_bf16(X: torch.Tensor, out: torch.Tensor | None = None, out_t: torch.Tensor | None = None) -> None:
    """fp32 [R][C] -> bf16 out [R][>=C] (pad columns zeroed up to out's row
    stride) and/or bf16 out_t [C][>=R]."""
    R, C = X.shape
    assert X.stride(-1) == 1
    _dev(X, "cvt_bf16")
    check(dense_lib().h2omx_cvt_bf16(P(X), X.stride(0), R, C, P(out), out.stride(0) if out is not None else 0,
                                     P(out_t), out_t.stride(0) if out_t is not None else 0, stream(X.device)),
          "cvt_bf16")


def rowsum_bf16(X: torch.Tensor, R: int, C: int, out: torch.Tensor) -> None:
    """out[r] = sum_{c<C} X[r][c] (fp32) for a bf16 matrix (bias gradients from dZ^T)."""
    _dev(X, "rowsum_bf16")
    check(dense_lib().h2omx_rowsum_bf16(P(X), X.stride(0), R, C, P(out), stream(X.device)), "rowsum_bf16")


class _CvtJob(ctypes.Structure):
    _fields_ = [("X", ctypes.c_void_p), ("out", ctypes.c_void_p), ("outT", ctypes.c_void_p), ("ldx", ctypes.c_int),
                ("R", ctypes.c_int), ("C", ctypes.c_int), ("ldo", ctypes.c_int), ("ldot", ctypes.c_int),
                ("pad", ctypes.c_int * 3)]


def cvt_bf16_multi(jobs) -> None:
    """Several ``cvt_bf16(X, out, out_t)`` conversions (<= 8) in one launch."""
    jobs = list(jobs)
    if not jobs:
        return
    _dev(jobs[0][0], "cvt_bf16_multi")
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
    _dev(Z, "softmax_xent_bf16")
    check(dense_lib().h2omx_softmax_xent_bf16(P(Z), P(y), P(dZ), dZ.stride(0), P(dZt), dZt.stride(0), P(loss), M,
                                              K, stream(Z.device)), "softmax_xent_bf16")
