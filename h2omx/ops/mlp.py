"""Small-batch MLP training step on the chain of ``csrc/mlp_kernels.hip``.

H2O DeepLearning's estimator defaults train on tiny mini-batches (256 rows
per GPU here), where every GEMM of the step is latency-bound: the library
GEMMs take ~8 us each whatever their size (``profiles/r4/dl``).  This module
runs one whole update - forward, loss gradient, backward, ADADELTA - as
``2 L - 1`` latency-optimised launches (L = number of layers; one more, an
ADADELTA-only tail, when L = 2):

    F_0 .. F_{L-2}, OUT, Q_{L-2} .. Q_0        (see the kernel file header)

Each launch is graph-capturable (fixed buffers; descriptors built once per
(network, batch) and re-pointed at the caller's batch).  The weight / bias
gradients land in ``net.grad`` as well (tests compare them with autograd).

Scope (``FusedMlpStep.supported``): Rectifier / Tanh hidden layers without
dropout or maxout, softmax cross-entropy with <= 8 classes or squared-error
regression, ADADELTA (H2O's default ``adaptive_rate``), L2 allowed; anything
else keeps the general path of ``models/deeplearning.py``.
"""
from __future__ import annotations

import ctypes

import torch

from .. import _native

_lib = None


def lib():
    global _lib
    if _lib is None:
        L = _native.require("mlp")
        for fn, args in (("h2omx_mlp_sizes", [ctypes.c_void_p]),
                         ("h2omx_mlp_phase", [ctypes.c_void_p, ctypes.c_void_p]),
                         ("h2omx_mlp_out", [ctypes.c_void_p, ctypes.c_void_p]),
                         ("h2omx_gemm_x3", [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
                         ("h2omx_gemm_x3_dact", [ctypes.c_void_p] * 5 + [ctypes.c_int] * 4 + [ctypes.c_void_p]),
                         ("h2omx_x3_transpose", [ctypes.c_int] + [ctypes.c_void_p] * 5)):
            f = getattr(L, fn)
            f.argtypes = args
            f.restype = ctypes.c_int
        _lib = L
        _check_layout(L)
    return _lib


class Opnd(ctypes.Structure):
    _fields_ = [("p", ctypes.c_void_p), ("ld", ctypes.c_int), ("kc", ctypes.c_int), ("vec", ctypes.c_int)]


class GemmJob(ctypes.Structure):
    _fields_ = [("A", Opnd), ("B", Opnd), ("I", ctypes.c_int), ("J", ctypes.c_int), ("K", ctypes.c_int),
                ("RI", ctypes.c_int), ("RJ", ctypes.c_int), ("tiles_j", ctypes.c_int), ("tiles", ctypes.c_int),
                ("epi", ctypes.c_int), ("act", ctypes.c_int), ("out", ctypes.c_void_p), ("ldo", ctypes.c_int),
                ("ldy", ctypes.c_int), ("bias", ctypes.c_void_p), ("Y", ctypes.c_void_p), ("db", ctypes.c_void_p),
                ("W", ctypes.c_void_p), ("Eg2", ctypes.c_void_p), ("Edx2", ctypes.c_void_p),
                ("bW", ctypes.c_void_p), ("bEg2", ctypes.c_void_p), ("bEdx2", ctypes.c_void_p),
                ("ada", ctypes.c_int), ("pad", ctypes.c_int)]


class AdaJob(ctypes.Structure):
    _fields_ = [("W", ctypes.c_void_p), ("G", ctypes.c_void_p), ("Eg2", ctypes.c_void_p), ("Edx2", ctypes.c_void_p),
                ("n", ctypes.c_longlong)]


MAX_JOBS, MAX_ADA = 3, 4


class Phase(ctypes.Structure):
    _fields_ = [("g", GemmJob * MAX_JOBS), ("a", AdaJob * MAX_ADA), ("ng", ctypes.c_int), ("na", ctypes.c_int),
                ("rho", ctypes.c_float), ("eps", ctypes.c_float), ("l2", ctypes.c_float), ("pad", ctypes.c_int)]


class OutDesc(ctypes.Structure):
    _fields_ = [("A", ctypes.c_void_p), ("W", ctypes.c_void_p), ("b", ctypes.c_void_p), ("y", ctypes.c_void_p),
                ("yr", ctypes.c_void_p), ("gout", ctypes.c_void_p), ("gprev", ctypes.c_void_p), ("M", ctypes.c_int),
                ("Hd", ctypes.c_int), ("C", ctypes.c_int), ("act", ctypes.c_int), ("mode", ctypes.c_int),
                ("vec", ctypes.c_int), ("lda", ctypes.c_int), ("ldp", ctypes.c_int), ("inv_m", ctypes.c_float),
                ("pad", ctypes.c_int)]


def _check_layout(L) -> None:
    s = (ctypes.c_int * 8)()
    _native.check(L.h2omx_mlp_sizes(ctypes.addressof(s)), "mlp_sizes")
    want = [ctypes.sizeof(Opnd), ctypes.sizeof(GemmJob), ctypes.sizeof(AdaJob), ctypes.sizeof(Phase),
            ctypes.sizeof(OutDesc), MAX_JOBS, MAX_ADA]
    if list(s[:7]) != want:
        raise RuntimeError(f"mlp descriptor layout mismatch: device {list(s[:7])} host {want}")


def _ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def _op(t: torch.Tensor | None, ld: int, kc: bool, ptr: int | None = None) -> Opnd:
    # vec: K-contiguous rows that are 16-byte aligned (float4 loads along k)
    p = ptr if ptr is not None else t.data_ptr()
    return Opnd(p, ld, 1 if kc else 0, 1 if (kc and ld % 4 == 0 and p % 16 == 0 and ld >= 4) else 0)


N_CUS = 256


# Tile override (tuning runs set it as a module attribute: "RI,RJ" forces one
# tile shape; "" = the per-shape choice below) and the 16-k load groups in
# flight per wave (1, 2, 4, 8 measured: 4 kept, profiles/r5/dl/)
_TILE = ""
DEPTH = 4
# activation rows padded off the 2 KB L2-channel period (A/B knob: no measured
# difference either way on MI355X, profiles/r5/dl/fused_step_ab_r5f.jsonl)


def padded_ld(n: int) -> int:
    """Row stride (floats) of an activation buffer: a multiple of 4 (float4
    loads) that is not a multiple of 256 floats (rows 1 KB apart or any
    multiple of it share L2 channels)."""
    ld = -(-n // 4) * 4
    if ld % 256 == 0:
        ld += 32
    return ld


def pick_tile(I: int, J: int) -> tuple[int, int]:
    """Largest 16 RI x 16 RJ tile that still puts >= ~N_CUS tiles on the chip
    (a tile's 4 waves split K, so tiles - not K - carry the parallelism)."""
    if _TILE:
        ri, rj = (int(v) for v in _TILE.split(","))
        return ri, rj
    best = None
    for ri, rj in ((2, 2), (1, 2), (2, 1), (1, 1)):
        tiles = -(-I // (16 * ri)) * -(-J // (16 * rj))
        if tiles >= N_CUS * 3 // 4:
            return ri, rj
        if best is None or tiles > best[2]:
            best = (ri, rj, tiles)
    return best[0], best[1]


def gemm_job(A: Opnd, B: Opnd, I: int, J: int, K: int, epi: int, act: int, out: torch.Tensor, ldo: int,
             bias=None, Y=None, ldy: int = 0, db=None, ada=None) -> GemmJob:
    ri, rj = pick_tile(I, J)
    tj = -(-J // (16 * rj))
    if K % 4:   # float4 (kLdV) operands need whole float4 groups of k
        A.vec = B.vec = 0
    j = GemmJob()
    j.A, j.B, j.I, j.J, j.K = A, B, I, J, K
    j.RI, j.RJ, j.tiles_j, j.tiles = ri, rj, tj, tj * -(-I // (16 * ri))
    j.epi, j.act, j.out, j.ldo, j.ldy = epi, act, _ptr(out), ldo, ldy
    j.bias, j.Y, j.db = _ptr(bias), _ptr(Y), _ptr(db)
    if ada is not None:
        W, Eg2, Edx2, bW, bEg2, bEdx2 = ada
        j.W, j.Eg2, j.Edx2, j.bW, j.bEg2, j.bEdx2 = (_ptr(W), _ptr(Eg2), _ptr(Edx2), _ptr(bW), _ptr(bEg2),
                                                     _ptr(bEdx2))
        j.ada = 1
    return j


class FusedMlpStep:
    """One rank's fused small-batch update of ``net`` (models/deeplearning.py
    ``_Net``: flat [W_l | b_l] spans) with ADADELTA state (Eg2, Edx2)."""

    @staticmethod
    def supported(net, act: int, classes: int, regression: bool, dropout: bool, adaptive: bool, M: int) -> bool:
        L = len(net.layers)
        return (net.flat.is_cuda and act in (1, 2) and not dropout and adaptive and L >= 2 and M >= 1
                and ((not regression and 2 <= classes <= 8) or (regression and classes == 1))
                and net.layers[-1][1] == classes and _native.available("mlp"))

    def __init__(self, net, act: int, M: int, Eg2: torch.Tensor, Edx2: torch.Tensor, rho: float, eps: float,
                 l2: float, regression: bool = False):
        self.net, self.act, self.M = net, act, M
        self.Eg2, self.Edx2 = Eg2, Edx2
        self.regression = regression
        self.rho, self.eps, self.l2 = float(rho), float(eps), float(l2)
        dev = net.flat.device
        L = len(net.layers)
        self.L = L
        dims = [net.layers[0][2]] + [w for (_, w, _) in net.layers]
        self.dims = dims
        # activations a_1 .. a_{L-1} and pre-activation gradients g_0 .. g_{L-1}
        # (row strides padded off the L2 channel period: padded_ld; the output
        # layer's few-class gradient keeps ld = classes)
        self.lda = [dims[0]] + [padded_ld(dims[l]) for l in range(1, L)]
        self.ldg = [padded_ld(dims[l + 1]) for l in range(L - 1)] + [dims[L]]
        self.a = [None] + [torch.empty((M * self.lda[l],), dtype=torch.float32, device=dev) for l in range(1, L)]
        self.gr = [torch.empty((M * self.ldg[l],), dtype=torch.float32, device=dev) for l in range(L)]
        self.lib = lib()
        self._x_ptr = None
        self._y_ptr = None
        self._build()

    # -- descriptors -------------------------------------------------------------
    def _span(self, l, buf):
        off, w, f = self.net.layers[l]
        return buf[off: off + w * f], buf[off + w * f: off + w * f + w]

    def _build(self) -> None:
        net, M, L, d, act = self.net, self.M, self.L, self.dims, self.act
        W = [self._span(l, net.flat) for l in range(L)]
        G = [self._span(l, net.grad) for l in range(L)]
        E1 = [self._span(l, self.Eg2) for l in range(L)]
        E2 = [self._span(l, self.Edx2) for l in range(L)]
        self._W, self._G, self._E1, self._E2 = W, G, E1, E2
        # forward phases F_1 .. F_{L-2} (F_0's A operand is the caller's batch, set per call)
        self.fwd = []
        for l in range(L - 1):
            A = None if l == 0 else _op(self.a[l], self.lda[l], True)
            ph = Phase()
            ph.ng, ph.na = 1, 0
            ph.g[0] = gemm_job(A or Opnd(), _op(W[l][0], d[l], True), M, d[l + 1], d[l], 0, act, self.a[l + 1],
                               self.lda[l + 1], bias=W[l][1])
            self.fwd.append(ph)
        self.out = OutDesc()
        o = self.out
        o.A, o.W, o.b = self.a[L - 1].data_ptr(), W[L - 1][0].data_ptr(), W[L - 1][1].data_ptr()
        o.gout, o.gprev = self.gr[L - 1].data_ptr(), self.gr[L - 2].data_ptr()
        o.M, o.Hd, o.C, o.act, o.mode = M, d[L - 1], d[L], act, 1 if self.regression else 0
        o.lda, o.ldp = self.lda[L - 1], self.ldg[L - 2]
        o.vec = 1 if (d[L - 1] % 4 == 0 and o.lda % 4 == 0 and o.ldp % 4 == 0 and o.A % 16 == 0 and o.W % 16 == 0
                      and o.gprev % 16 == 0) else 0
        o.inv_m = 1.0 / M
        # ADADELTA placement: layer l >= 1 as early as allowed - after the phase
        # that completes dW_l (Q_l; the output layer's in Q_{L-2}) and after the
        # last read of W_l (Q_l for g_{l-1}; OUT for the output layer):
        # Q_{l-1}, the output layer Q_{L-3}; -1 = an ADADELTA-only tail launch.
        # Layer 0 is updated inside its own dW tiles in Q_0 (nothing reads W_0 there).
        ada_at: dict[int, list[int]] = {}
        for l in range(1, L):
            at = l - 1 if l <= L - 2 else L - 3
            ada_at.setdefault(at if at >= 0 else -1, []).append(l)
        # backward phases Q_{L-2} .. Q_0
        self.bwd = []
        for j in range(L - 2, -1, -1):
            ph = Phase()
            ph.rho, ph.eps, ph.l2 = self.rho, self.eps, self.l2
            jobs = []
            aj = self.a[j] if j > 0 else None
            A_dw = _op(self.gr[j], self.ldg[j], False)
            B_dw = _op(aj, self.lda[j], False) if j > 0 else None
            # dW_j = g_j^T a_j (+ db_j); layer 0 updates its tiles in place (nothing reads W_0 here)
            ada0 = (W[0][0], E1[0][0], E2[0][0], W[0][1], E1[0][1], E2[0][1]) if j == 0 else None
            jobs.append(("dw", j, A_dw, B_dw, ada0))
            if j == L - 2:
                # the output layer's (few-class) weight gradient rides along in the first phase
                jobs.append(("dw", L - 1, _op(self.gr[L - 1], d[L], False), _op(self.a[L - 1], self.lda[L - 1], False),
                             None))
            if j >= 1:
                jobs.append(("dh", j, None, None, None))
            ph.ng = len(jobs)
            for q, (kind, l, A, B, ada) in enumerate(jobs):
                if kind == "dw":
                    if B is None:
                        B = Opnd()    # layer 0: the caller's batch (set per call)
                    ph.g[q] = gemm_job(A, B, d[l + 1], d[l], M, 2, act, G[l][0], d[l], db=G[l][1], ada=ada)
                else:
                    # g_{l-1} = (g_l W_l) * act'(a_l)
                    ph.g[q] = gemm_job(_op(self.gr[l], self.ldg[l], True), _op(W[l][0], d[l], False), M, d[l],
                                       d[l + 1], 1, act, self.gr[l - 1], self.ldg[l - 1], Y=self.a[l],
                                       ldy=self.lda[l])
            ph.na = 0
            for l in ada_at.get(j, []):
                for part in (0, 1):   # weights, bias
                    ph.a[ph.na] = AdaJob(W[l][part].data_ptr(), G[l][part].data_ptr(), E1[l][part].data_ptr(),
                                         E2[l][part].data_ptr(), W[l][part].numel())
                    ph.na += 1
            self.bwd.append(ph)
        self.tail = None
        if ada_at.get(-1):
            ph = Phase()
            ph.rho, ph.eps, ph.l2 = self.rho, self.eps, self.l2
            ph.ng, ph.na = 0, 0
            for l in ada_at[-1]:
                for part in (0, 1):
                    ph.a[ph.na] = AdaJob(W[l][part].data_ptr(), G[l][part].data_ptr(), E1[l][part].data_ptr(),
                                         E2[l][part].data_ptr(), W[l][part].numel())
                    ph.na += 1
            self.tail = ph

    def _set_batch(self, xb: torch.Tensor, yb: torch.Tensor) -> None:
        if xb.shape != (self.M, self.dims[0]) or not xb.is_contiguous() or xb.dtype != torch.float32:
            raise ValueError("fused MLP step: batch must be a contiguous float32 [M][features] tensor")
        xp = xb.data_ptr()
        if xp != self._x_ptr:
            self.fwd[0].g[0].A = _op(None, self.dims[0], True, ptr=xp)
            # Q_0's dW_0 job: B = the batch (element (j, m) at x[m][j])
            self.bwd[-1].g[0].B = _op(None, self.dims[0], False, ptr=xp)
            self._x_ptr = xp
        yp = yb.data_ptr()
        if yp != self._y_ptr:
            if self.regression:
                self.out.yr, self.out.y = yp, None
            else:
                self.out.y, self.out.yr = yp, None
            self._y_ptr = yp

    def step(self, xb: torch.Tensor, yb: torch.Tensor) -> None:
        """One update on the batch (xb [M][F] float32, yb int32 classes / float32 targets)."""
        self._set_batch(xb, yb)
        s = _native.stream_of(xb.device)
        L = self.lib
        for ph in self.fwd + self.bwd + ([self.tail] if self.tail is not None else []):
            ph.pad = DEPTH
        for ph in self.fwd:
            _native.check(L.h2omx_mlp_phase(ctypes.addressof(ph), s), "mlp_phase(fwd)")
        _native.check(L.h2omx_mlp_out(ctypes.addressof(self.out), s), "mlp_out")
        for ph in self.bwd:
            _native.check(L.h2omx_mlp_phase(ctypes.addressof(ph), s), "mlp_phase(bwd)")
        if self.tail is not None:
            _native.check(L.h2omx_mlp_phase(ctypes.addressof(self.tail), s), "mlp_phase(ada)")

    @property
    def launches(self) -> int:
        return len(self.fwd) + 1 + len(self.bwd) + (1 if self.tail is not None else 0)


def gemm_x3_ok(A: torch.Tensor, B: torch.Tensor) -> bool:
    """Operands the x3 GEMM takes: K-contiguous fp32 rows, 16-byte aligned, K % 4 == 0."""
    return (A.is_cuda and A.dtype == torch.float32 and B.dtype == torch.float32 and A.stride(1) == 1
            and B.stride(1) == 1 and A.stride(0) % 4 == 0 and B.stride(0) % 4 == 0 and A.shape[1] % 4 == 0
            and A.data_ptr() % 16 == 0 and B.data_ptr() % 16 == 0 and _native.available("mlp"))


def gemm_x3(A: torch.Tensor, B: torch.Tensor, bias: torch.Tensor | None = None, act: int = 0,
            out: torch.Tensor | None = None) -> torch.Tensor:
    """C = act(A B^T + bias) for fp32 A [M][K], B [N][K] on the bf16 matrix cores
    with an exact 3-piece operand split (csrc/mlp_kernels.hip gemm_x3_nt_kernel):
    fp32-equivalent accuracy at ~2.7x the fp32-MFMA rate."""
    M, K = A.shape
    N = B.shape[0]
    C = out if out is not None else torch.empty((M, N), dtype=torch.float32, device=A.device)
    if bias is not None:
        bias = bias.float().contiguous()
    _native.check(lib().h2omx_gemm_x3(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), C.data_ptr(), C.stride(0),
                                      0 if bias is None else bias.data_ptr(), M, N, K, act,
                                      _native.stream_of(A.device)), "gemm_x3")
    return C


def x3_transpose(pairs) -> None:
    """dst = src^T for up to 8 (src [R][C], dst [C][R]) fp32 pairs, one launch."""
    n = len(pairs)
    if n == 0:
        return
    src = (ctypes.c_void_p * n)(*[a.data_ptr() for a, _ in pairs])
    dst = (ctypes.c_void_p * n)(*[b.data_ptr() for _, b in pairs])
    R = (ctypes.c_int * n)(*[a.shape[0] for a, _ in pairs])
    C = (ctypes.c_int * n)(*[a.shape[1] for a, _ in pairs])
    for a, b in pairs:
        if not (a.is_contiguous() and b.numel() >= a.numel()):
            raise ValueError("x3_transpose: needs a contiguous source and a large enough destination")
    _native.check(lib().h2omx_x3_transpose(n, src, dst, R, C, _native.stream_of(pairs[0][0].device)), "x3_transpose")


def gemm_x3_dact(dZ: torch.Tensor, Wt: torch.Tensor, Y: torch.Tensor, act: int, ws: torch.Tensor,
                 out: torch.Tensor | None = None) -> torch.Tensor:
    """dZ_prev = (dZ [M][K] Wt [N][K]^T) * act'(Y [M][N]) on the x3 GEMM (Wt =
    the layer's W^T from :func:`x3_transpose`, so both operands are
    K-contiguous), with the column sums of dZ_prev per 64-row block in ``ws``
    [(M + 63) // 64][N]."""
    M, K = dZ.shape
    N = Y.shape[1]
    C = out if out is not None else torch.empty((M, N), dtype=torch.float32, device=dZ.device)
    _native.check(lib().h2omx_gemm_x3_dact(dZ.data_ptr(), Wt.data_ptr(), Y.data_ptr(), C.data_ptr(), ws.data_ptr(),
                                           M, N, K, int(act), _native.stream_of(dZ.device)), "gemm_x3_dact")
    return C
