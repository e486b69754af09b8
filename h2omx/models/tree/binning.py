"""K1: quantile sketch + feature binning into uint8 codes (feature-major).

Cut points are per-feature weighted-free quantiles of a row sample.  With
several ranks, every rank contributes a sample and the samples are
all-gathered so all ranks derive bit-identical cut points (SURVEY.md §2.5 K1,
collective C1).  Codes are stored ``[F][npad]`` with ``npad`` a multiple of 64
so that histogram lanes can issue 16-byte loads of 16 consecutive rows.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import numpy as np
import torch

from ... import ops

ROW_ALIGN = 64


@dataclass
class BinnedMatrix:
    codes: torch.Tensor      # uint8 [F][npad]
    edges: torch.Tensor      # float32 [F][nbt]  (edges[f][:nvb[f]-1] used)
    nvb: torch.Tensor        # int32 [F] number of value bins per feature
    n: int
    npad: int
    nbt: int                 # histogram width; bin nbt-1 is the NA bin
    names: list
    # categorical group splits: per feature True for an identity-binned enum
    # column (bin = level code, <= 255 levels); None = all numeric
    cat: np.ndarray | None = None
    # per-node histogram rules: float32 [F][4] (min, max, exact, integer) from
    # adaptive_ranges; None when every node scans all fine bins
    frange: torch.Tensor | None = None

    @property
    def catf(self) -> torch.Tensor | None:
        """Device uint8 [F] copy of ``cat`` (SplitParams::catf), None without
        categorical features."""
        if self.cat is None or not np.any(self.cat):
            return None
        t = getattr(self, "_catf", None)
        if t is None or t.device != self.codes.device:
            t = torch.from_numpy(np.asarray(self.cat, np.uint8)).to(self.codes.device)
            self._catf = t
        return t

    @property
    def F(self) -> int:
        return self.codes.shape[0]

    @property
    def device(self):
        return self.codes.device

    _codes_rm: torch.Tensor | None = None
    # row-major code rows padded to line-aligned strides (False: 4-byte strides)
    ROW_ALIGN = True
    # codes_rm built by codes_rowmajor_kernel (False: a strided torch copy)
    ROWMAJOR_KERNEL = True

    @property
    def fp(self) -> int:
        """Row stride of the row-major codes: a power of two up to 128 bytes
        (F = 100 -> 128), a multiple of 128 above, so no row straddles a
        128-byte line - a random row gather then fetches one line, not 1.8
        on average (100-byte rows).  The pad bytes are zero and never read as
        codes."""
        if not self.ROW_ALIGN:
            return (self.F + 3) // 4 * 4
        if self.F <= 128:
            fp = 4
            while fp < self.F:
                fp *= 2
            return fp
        return (self.F + 127) // 128 * 128

    @property
    def codes_rm(self) -> torch.Tensor:
        """Row-major copy uint8 [n][fp] (lazily built once): the segmented
        histogram kernel gathers whole rows (28 B for HIGGS) by row index."""
        if self._codes_rm is None:
            c = self.codes
            if self.ROWMAJOR_KERNEL and c.is_cuda and c.is_contiguous() and c.shape == (self.F, self.npad) and self.npad % 64 == 0:
                # (codes_rowmajor_kernel: LDS-tiled, writes the pad bytes too)
                rm = torch.empty((self.n, self.fp), dtype=torch.uint8, device=c.device)
                ops.check(ops.tree_lib().h2omx_codes_rowmajor(ops.P(c), self.npad, self.F, self.n, ops.P(rm),
                                                              self.fp, ops.stream(c.device)), "codes_rowmajor")
            else:
                rm = torch.zeros((self.n, self.fp), dtype=torch.uint8, device=c.device)
                rm[:, : self.F] = c[:, : self.n].t()
            self._codes_rm = rm
        return self._codes_rm

    def edges_numpy(self):
        e = self.edges.cpu().numpy()
        nv = self.nvb.cpu().numpy()
        return [e[f, : max(int(nv[f]) - 1, 0)].copy() for f in range(len(nv))]


def hist_width(nbins: int) -> int:
    """Smallest supported histogram width holding nbins value bins + NA."""
    for w in (32, 64, 128, 256):
        if nbins + 1 <= w:
            return w
    return 256


def _edges_from_sorted(col: np.ndarray, max_value_bins: int) -> np.ndarray:
    col = col[~np.isnan(col)]
    if col.size == 0:
        return np.zeros(0, np.float32)
    uniq = np.unique(col)
    if uniq.size <= max_value_bins:
        return uniq[:-1].astype(np.float32)
    qs = np.quantile(col, np.linspace(0.0, 1.0, max_value_bins + 1)[1:-1], method="lower")
    e = np.unique(qs.astype(np.float32))
    # the top edge must be below the max so the last bin is non-empty
    e = e[e < uniq[-1]]
    return e[: max_value_bins - 1]


HISTOGRAM_TYPES = {"quantilesglobal": "quantilesglobal", "uniformadaptive": "uniformadaptive",
                   "uniformrobust": "uniformrobust", "random": "random", "roundrobin": "roundrobin"}

# SplitParams::hist_mode of the per-node rules (csrc/tree_kernels.hip
# adaptive_candidates); QuantilesGlobal / UniformRobust scan every fine bin
PER_NODE_MODES = {"uniformadaptive": 1, "random": 2, "roundrobin": 3}


def resolve_histogram_type(h, auto: str = "quantilesglobal") -> str:
    """H2O ``histogram_type`` -> the binning rule (``auto``: what AUTO means
    for the caller - UniformAdaptive for GBM / DRF as in the H2O-3 image the
    reference deploys, /root/reference/src/k8s/mod.rs:115).

    * QuantilesGlobal: global quantile cut points.
    * UniformAdaptive / Random / RoundRobin are per-node rules on GBM / DRF
      (see :func:`adaptive_ranges`); callers without the per-node scan (the
      :func:`compute_edges` grids) get one global equal-width / random grid.
    * UniformRobust: equal-width bins over the central 99 % of the column
      (values beyond fall into the outer bins), one global grid."""
    key = str(h or "AUTO").replace("_", "").lower()
    if key == "auto":
        return auto
    if key not in HISTOGRAM_TYPES:
        raise ValueError(f"unknown histogram_type {h!r}")
    return HISTOGRAM_TYPES[key]


def node_bins(nbins_top_level: int, nbins: int, depth: int) -> int:
    """Equal-width bins of one node at ``depth`` (H2O: nbins_top_level at the
    root, halved per level, never below nbins; mirrors adaptive_candidates)."""
    top = int(nbins_top_level) >> depth if depth < 31 else 0
    return max(top, int(nbins), 2)


def adaptive_ranges(X: torch.Tensor, bm: "BinnedMatrix", comm=None, sample_rows: int = 1 << 20,
                    seed: int = 1234) -> torch.Tensor:
    """Per-feature facts the per-node histogram rules need, float32 [F][4]
    on the codes' device: (min, max, exact, integer), taken from the same row
    sample the cut points come from (:func:`compute_edges`: all-gathered, so
    every rank derives identical values; a full pass over a 10M x 100 frame
    per fit cost AutoML ~0.2 s a model).  ``min`` / ``max`` bound the first /
    last fine bin; ``exact`` = every sampled value equals its bin's value
    (low-cardinality columns binned one bin per distinct value: a node's
    range is then its own min / max); ``integer`` = all sampled values are
    whole numbers (H2O gives an integer column spanning at most nb values one
    bin per value)."""
    F, n = X.shape
    S = X if n <= sample_rows else X.index_select(
        1, torch.randint(0, n, (sample_rows,), generator=torch.Generator(device="cpu").manual_seed(seed)).to(X.device))
    if comm is not None and comm.world_size > 1:
        S = comm.all_gather_cat(S.contiguous(), dim=1)
    S = S.float()
    dev = S.device
    nan = torch.isnan(S)
    lo = torch.where(nan, float("inf"), S).amin(1)
    hi = torch.where(nan, float("-inf"), S).amax(1)
    isint = (nan | (S == torch.floor(S))).all(1)
    edges = bm.edges.to(dev)
    nvb = bm.nvb.to(dev).long()
    code = torch.searchsorted(edges.contiguous(), torch.nan_to_num(S, nan=0.0).contiguous(), side="left")
    last = (nvb - 1)[:, None]
    bval = torch.where(code < last, torch.gather(edges, 1, torch.minimum(code, (last - 1).clamp_min(0))), hi[:, None])
    exact = (nan | (S == bval)).all(1)
    out = torch.stack([lo, hi, exact.float(), isint.float()], 1).double().cpu().numpy()
    empty = ~(out[:, 0] <= out[:, 1])
    out[empty, 0] = out[empty, 1] = 0.0
    return torch.from_numpy(out.astype(np.float32)).to(bm.codes.device)


def _range_edges(lo: float, hi: float, nb: int, kind: str, rng: np.random.Generator) -> np.ndarray:
    if not (np.isfinite(lo) and np.isfinite(hi)) or hi <= lo or nb < 2:
        return np.zeros(0, np.float32)
    if kind == "random":
        e = np.sort(rng.uniform(lo, hi, nb - 1))
    else:
        e = lo + (hi - lo) * np.arange(1, nb) / nb
    e = np.unique(e.astype(np.float32))
    return e[(e >= lo) & (e < hi)]


def compute_edges(X: torch.Tensor, nbins: int, sample_rows: int = 1 << 20, seed: int = 1234,
                  comm=None, histogram_type: str = "QuantilesGlobal") -> tuple[np.ndarray, np.ndarray, int]:
    """Per-feature cut points from a row sample of feature-major ``X`` [F][n]
    (``histogram_type``: see :func:`resolve_histogram_type`; columns with at
    most ``nbins`` distinct values always get one bin per value).

    Returns (edges [F][nbt] float32, nvb [F] int32, nbt).
    """
    kind = resolve_histogram_type(histogram_type)
    edges, nvb, nbt = _quantile_edges(X, nbins, sample_rows, seed, comm)
    if kind in ("quantilesglobal", "roundrobin"):
        return edges, nvb, nbt
    max_value_bins = min(nbins, nbt - 1)
    # the column ranges over the same (all-gathered) sample on every rank
    F, n = X.shape
    Xs = X if n <= sample_rows else X.index_select(
        1, torch.randint(0, n, (sample_rows,), generator=torch.Generator(device="cpu").manual_seed(seed)).to(X.device))
    if comm is not None and comm.world_size > 1:
        Xs = comm.all_gather_cat(Xs.contiguous(), dim=1)
    Xs = Xs.float()
    if kind == "uniformrobust":
        q = torch.tensor([0.005, 0.995], dtype=torch.float32, device=Xs.device)
        los, his = [], []
        for f in range(F):
            col = Xs[f][~torch.isnan(Xs[f])]
            if col.numel() == 0:
                los.append(np.nan)
                his.append(np.nan)
                continue
            col = col[:: max(1, col.numel() // (1 << 22))]      # torch.quantile input limit
            a, b = torch.quantile(col, q).tolist()
            los.append(a)
            his.append(b)
        lo, hi = np.array(los), np.array(his)
    else:
        big = torch.finfo(torch.float32).max
        nanm = torch.isnan(Xs)
        lo = torch.where(nanm, big, Xs).amin(1).cpu().double().numpy()
        hi = torch.where(nanm, -big, Xs).amax(1).cpu().double().numpy()
    for f in range(F):
        if int(nvb[f]) - 1 < max_value_bins - 1:
            continue                     # few distinct values: exact value bins
        rng = np.random.default_rng([seed & 0xFFFFFFFF, f])
        e = _range_edges(float(lo[f]), float(hi[f]), max_value_bins, kind, rng)
        edges[f, :] = np.inf
        edges[f, : e.size] = e
        nvb[f] = e.size + 1
    return edges, nvb, nbt


def _quantile_edges(X: torch.Tensor, nbins: int, sample_rows: int, seed: int, comm):
    F, n = X.shape
    nbt = hist_width(nbins)
    max_value_bins = min(nbins, nbt - 1)
    if n > sample_rows:
        g = torch.Generator(device="cpu").manual_seed(seed)
        idx = torch.randint(0, n, (sample_rows,), generator=g).to(X.device)
        S = X.index_select(1, idx)
    else:
        S = X
    if comm is not None and comm.world_size > 1:
        S = comm.all_gather_cat(S.contiguous(), dim=1)
    edges = np.full((F, nbt), np.inf, np.float32)
    nvb = np.zeros(F, np.int32)
    if S.is_cuda:
        for f, e in enumerate(_edges_sketch(S.float(), max_value_bins)):
            edges[f, : e.size] = e
            nvb[f] = e.size + 1
        return edges, nvb, nbt
    Sn = S.float().cpu().numpy()
    for f in range(F):
        e = _edges_from_sorted(Sn[f], max_value_bins)
        edges[f, : e.size] = e
        nvb[f] = e.size + 1
    return edges, nvb, nbt


def sort_rows(S: torch.Tensor) -> torch.Tensor:
    """Ascending sort of every row of float32 ``S`` [F][m], NaNs last - as
    ``torch.sort(S, dim=1).values`` but through ONE radix sort of F*m int64
    keys (row index << 32 | order-preserving float bits) instead of F
    segmented merge sorts (HIGGS sketch, 28 x 1M: the segmented sort
    launched ~560 merge kernels)."""
    F, m = S.shape
    if F <= 1:
        return torch.sort(S, dim=1).values
    x = torch.where(torch.isnan(S), torch.full_like(S, float("nan")).abs(), S)   # canonical +NaN
    b = x.contiguous().view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    neg = (b >> 31) == 1
    ok = torch.where(neg, b ^ 0xFFFFFFFF, b | 0x80000000)      # order-preserving unsigned image
    rows = torch.arange(F, device=S.device, dtype=torch.int64)[:, None]
    keys = torch.sort(((rows << 32) | ok).view(-1)).values.view(F, m) & 0xFFFFFFFF
    back = torch.where(keys >= 0x80000000, keys & 0x7FFFFFFF, keys ^ 0xFFFFFFFF)
    return back.to(torch.int32).view(torch.float32)




# device quantile sketch (csrc/sketch_kernels.hip); False: sort the sample
# (the sketch's test oracle, tests/test_sketch_gpu.py)
SKETCH = True


def _key_to_float(k: np.ndarray) -> np.ndarray:
    k = k.astype(np.uint32)
    b = np.where(k >= 0x80000000, k & 0x7FFFFFFF, ~k)
    return b.astype(np.uint32).view(np.float32)


def _edges_sketch(S: torch.Tensor, max_value_bins: int) -> list:
    """``_edges_from_sorted`` for every row of the sample S [F][m] without
    sorting it: the two-level radix select of csrc/sketch_kernels.hip finds
    the numpy 'lower' quantile order statistics and the maximum exactly;
    low-cardinality features read their distinct values off the key
    histogram.  Features the sketch hands back (a refinement bin above 8192
    keys, or a low-cardinality candidate with two values in one bin) take the
    sort path."""
    F, m = S.shape
    if not SKETCH or m < 2:
        return _edges_device(sort_rows(S), max_value_bins)
    dev = S.device
    S = S.contiguous()
    lib = ops.tree_lib()
    NB = int(lib.h2omx_sketch_bins())
    qv = np.linspace(0.0, 1.0, max_value_bins + 1)[1:-1]
    T = qv.size
    u32 = torch.int32
    H, P, mark, off, fill = (torch.empty((F, NB), dtype=u32, device=dev) for _ in range(5))
    tbin, trank, okey = (torch.zeros((F, T + 1), dtype=u32, device=dev) for _ in range(3))
    lcbin, lckey = (torch.zeros((F, 256), dtype=u32, device=dev) for _ in range(2))
    info = torch.empty((F, 4), dtype=u32, device=dev)
    buf = torch.empty((F, m), dtype=u32, device=dev)
    qv_t = torch.from_numpy(qv).to(dev)
    P_ = ops.P
    ops.check(lib.h2omx_sketch(P_(S), S.stride(0), m, F, T, P_(qv_t), max_value_bins, P_(H), P_(P), P_(mark),
                               P_(off), P_(fill), P_(tbin), P_(trank), P_(okey), P_(lcbin), P_(lckey), P_(info),
                               P_(buf), ops.stream(dev)), "sketch")
    info_h = info.cpu().numpy()
    keys = okey.cpu().numpy().view(np.uint32)
    lck = lckey.cpu().numpy().view(np.uint32)
    cnt, nonempty, lowc, fb = info_h[:, 0], info_h[:, 1], info_h[:, 2], info_h[:, 3]
    dist = {f: _key_to_float(lck[f, : nonempty[f]]) for f in range(F) if lowc[f] and not fb[f] and cnt[f] > 0}
    sort_f = [f for f in range(F) if fb[f]]
    sorted_out = {}
    if sort_f:
        for f, e in zip(sort_f, _edges_device(sort_rows(S[sort_f]), max_value_bins)):
            sorted_out[f] = e
    out = []
    for f in range(F):
        if f in sorted_out:
            out.append(sorted_out[f])
        elif cnt[f] == 0:
            out.append(np.zeros(0, np.float32))
        elif f in dist:
            out.append(dist[f][:-1].astype(np.float32))
        else:
            qf = _key_to_float(keys[f])
            e = np.unique(qf[:T])
            e = e[e < qf[T]]
            out.append(e[: max_value_bins - 1])
    return out


def _edges_device(S: torch.Tensor, max_value_bins: int) -> list:
    """``_edges_from_sorted`` for every row of the ascending-sorted sample S
    [F][m] (NaNs last) with the heavy work on the device: distinct values by
    adjacent comparison, the 'lower' quantiles as index gathers; only the
    distinct values of low-cardinality features and [F][<= 256] quantiles
    reach the host (no [F][m] rank / cumsum temporaries)."""
    F, m = S.shape
    dev = S.device
    cnt = (~torch.isnan(S)).sum(1)                                      # non-NaN prefix length
    new = torch.arange(m, device=dev)[None, :] < cnt[:, None]
    new[:, 1:] &= S[:, 1:] != S[:, :-1]
    nuniq = new.sum(1)
    # distinct values of the features with <= max_value_bins of them (row-major
    # nonzero order = ascending within each feature); the selection scan runs
    # over those features only
    low = torch.nonzero(nuniq <= max_value_bins)[:, 0]
    if low.numel():
        fl, pi = torch.nonzero(new.index_select(0, low), as_tuple=True)
        fi, uval = low[fl], S.index_select(0, low)[fl, pi]
    else:
        fi = torch.zeros(0, dtype=torch.int64, device=dev)
        uval = torch.zeros(0, dtype=S.dtype, device=dev)
    cnt_h = cnt.cpu().numpy()
    # numpy 'lower' quantile: index floor((n - 1) q) in float64
    qv = np.linspace(0.0, 1.0, max_value_bins + 1)[1:-1]
    idx = np.floor((np.maximum(cnt_h, 1) - 1)[:, None].astype(np.float64) * qv[None, :]).astype(np.int64)
    Q = torch.gather(S, 1, torch.from_numpy(idx).to(dev))
    mx = torch.gather(S, 1, (cnt - 1).clamp_min(0)[:, None])[:, 0]
    Q, nu, mx = Q.cpu().numpy(), nuniq.cpu().numpy(), mx.cpu().numpy()
    fi, uval = fi.cpu().numpy(), uval.cpu().numpy()
    starts = np.searchsorted(fi, np.arange(F + 1))
    out = []
    for f in range(F):
        if cnt_h[f] == 0:
            out.append(np.zeros(0, np.float32))
        elif nu[f] <= max_value_bins:
            out.append(uval[starts[f]: starts[f + 1]][: nu[f] - 1].astype(np.float32))
        else:
            e = np.unique(Q[f].astype(np.float32))
            e = e[e < mx[f]]
            out.append(e[: max_value_bins - 1])
    return out


MAX_CAT_LEVELS = 255


def categorical_bins(edges: np.ndarray, nvb: np.ndarray, nbt: int, levels: dict) -> tuple:
    """Identity bins for categorical features: ``levels`` maps feature index ->
    number of levels L (codes 0..L-1); a feature with 2 <= L <= 255 gets the
    cut points 0.5, 1.5, ..., L - 1.5 (bin = level code) and is flagged for
    group splits.  The histogram width grows to hold the widest one.  Enum
    columns with more levels keep the ordinal quantile bins of their codes
    (H2O groups levels beyond nbins_cats similarly).  Returns (edges, nvb,
    nbt, cat [F] bool)."""
    F = edges.shape[0]
    cat = np.zeros(F, bool)
    use = {f: L for f, L in levels.items() if 2 <= L <= MAX_CAT_LEVELS}
    if not use:
        return edges, nvb, nbt, cat
    nbt2 = max(nbt, hist_width(max(use.values())))
    if nbt2 > nbt:
        wide = np.full((F, nbt2), np.inf, np.float32)
        wide[:, :nbt] = edges
        edges = wide
    edges = np.array(edges, np.float32, copy=True)
    nvb = np.array(nvb, np.int32, copy=True)
    for f, L in use.items():
        edges[f, :] = np.inf
        edges[f, : L - 1] = np.arange(L - 1, dtype=np.float32) + 0.5
        nvb[f] = L
        cat[f] = True
    return edges, nvb, nbt2, cat


def bin_matrix(X: torch.Tensor, edges: np.ndarray, nvb: np.ndarray, nbt: int, names=None,
               cat: np.ndarray | None = None) -> BinnedMatrix:
    """Bin feature-major float32 ``X`` [F][n] (any stride on dim 1 == 1);
    ``cat``: categorical flags from :func:`categorical_bins`."""
    F, n = X.shape
    npad = max(ROW_ALIGN, int(math.ceil(n / ROW_ALIGN) * ROW_ALIGN))
    dev = X.device
    names = list(names) if names is not None else [f"C{i + 1}" for i in range(F)]
    e_t = torch.from_numpy(np.ascontiguousarray(edges, np.float32)).to(dev)
    nv_t = torch.from_numpy(np.ascontiguousarray(nvb, np.int32)).to(dev)
    if X.is_cuda:
        Xc = X.float().contiguous()
        codes = torch.empty((F, npad), dtype=torch.uint8, device=dev)
        lib = ops.tree_lib()
        ops.check(lib.h2omx_bin_features(ops.P(Xc), Xc.stride(0), n, F, ops.P(e_t), ops.P(nv_t), nbt,
                                         ops.P(codes), npad, ops.stream(dev)), "bin_features")
    else:
        Xn = X.float().numpy()
        codes_np = np.zeros((F, npad), np.uint8)
        for f in range(F):
            m = int(nvb[f]) - 1
            col = Xn[f]
            c = np.searchsorted(edges[f, :m], col, side="left").astype(np.uint8)
            c[np.isnan(col)] = nbt - 1
            codes_np[f, :n] = c
        codes = torch.from_numpy(codes_np)
    return BinnedMatrix(codes=codes, edges=e_t, nvb=nv_t, n=n, npad=npad, nbt=nbt, names=names,
                        cat=None if cat is None else np.asarray(cat, bool))

