"""Frame munging operations behind Rapids (h2o-py ``H2OFrame`` methods).

Row-sharded semantics (every rank holds a contiguous shard of each frame):

* shard-local, element-wise: ``ifelse``, ``na_omit``, ``cut``, ``relevel``,
  ``stratified_split`` (per-row random draw);
* local pass + small collectives: ``scale`` / ``impute`` (global means,
  sds, medians, modes), ``cumsum``/``cumprod``/``cummin``/``cummax`` (the
  ranks' totals are exchanged to offset each shard), ``kfold_column`` and
  ``which`` (global row ids), ``quantile`` (exact: distributed bisection on
  the value with all-reduced counts, no data movement);
* aggregated results (``group_by``, ``unique``, ``table``): each rank
  aggregates its shard, the per-rank partial tables are all-gathered and
  combined; the (small) result frame lives on the leader (rank 0) and the
  other ranks hold empty shards of it;
* ``sort`` / ``merge``: rows are gathered to the leader, which holds the
  result (documented limitation: a distributed sample-sort / hash-join
  exchange is future work).

All numeric work runs on the frame's device (torch ops on the GPU).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.distributed as dist

from .frame import ENUM, INT, REAL, Frame, Vec


# ---------------------------------------------------------------------------
# helpers
# ---------------------------------------------------------------------------
def _ws(comm) -> int:
    return comm.world_size if comm is not None else 1


def _rank(comm) -> int:
    return comm.rank if comm is not None else 0


def _gather_objects(comm, obj) -> list:
    if _ws(comm) == 1:
        return [obj]
    out = [None] * comm.world_size
    dist.all_gather_object(out, obj, group=getattr(comm, "group", None))
    return out


def row_base(n: int, comm) -> int:
    counts = _gather_objects(comm, int(n))
    return int(sum(counts[: _rank(comm)]))


def _allreduce(t: torch.Tensor, comm, op="sum") -> torch.Tensor:
    if _ws(comm) > 1:
        comm.all_reduce_(t, op)
    return t


def _empty_like(fr: Frame) -> Frame:
    return Frame([Vec(v.name, v.data[:0], v.vtype, v.domain) for v in fr.vecs])


def _to_pandas_local(fr: Frame):
    return fr.to_pandas()


def gather_to_leader(fr: Frame, comm) -> Frame | None:
    """All rows on rank 0 (None elsewhere), enum domains unified."""
    if _ws(comm) == 1:
        return fr
    from .distributed import gather_frame

    g = gather_frame(fr, comm)
    return g if _rank(comm) == 0 else None


def _leader_result(fr_or_none: Frame | None, template: Frame, comm) -> Frame:
    if _rank(comm) == 0:
        return fr_or_none
    return _empty_like(template)


# ---------------------------------------------------------------------------
# element-wise / shard-local
# ---------------------------------------------------------------------------
def ifelse(test: Frame, yes, no) -> Frame:
    t = test.vecs[0].as_float()
    cond = torch.nan_to_num(t, nan=0.0) != 0
    na = torch.isnan(t)

    def val(x, i):
        if isinstance(x, Frame):
            v = x.vecs[min(i, x.ncols - 1)]
            return v
        return x

    ncols = max(f.ncols if isinstance(f, Frame) else 1 for f in (test, yes, no))
    out = []
    for i in range(ncols):
        y, n_ = val(yes, i), val(no, i)
        # both categorical with the same domain -> categorical result
        if isinstance(y, Vec) and isinstance(n_, Vec) and y.vtype == ENUM and n_.vtype == ENUM and \
                list(y.domain) == list(n_.domain):
            r = torch.where(cond, y.data, n_.data)
            r = torch.where(na, torch.full_like(r, -1), r)
            out.append(Vec(test.names[min(i, test.ncols - 1)], r, ENUM, list(y.domain)))
            continue
        if isinstance(y, str) or isinstance(n_, str):
            levels = sorted({s for s in (y, n_) if isinstance(s, str)})
            code = {s: i for i, s in enumerate(levels)}
            yc = torch.full_like(t, code[y] if isinstance(y, str) else -1, dtype=torch.int32)
            nc = torch.full_like(t, code[n_] if isinstance(n_, str) else -1, dtype=torch.int32)
            r = torch.where(cond, yc, nc)
            r = torch.where(na, torch.full_like(r, -1), r)
            out.append(Vec(test.names[0], r, ENUM, levels))
            continue
        yt = y.as_float() if isinstance(y, Vec) else torch.full_like(t, float(y))
        nt = n_.as_float() if isinstance(n_, Vec) else torch.full_like(t, float(n_))
        r = torch.where(cond, yt, nt)
        out.append(Vec(test.names[min(i, test.ncols - 1)], torch.where(na, torch.full_like(r, float("nan")), r),
                       REAL))
    return Frame(out)


def na_omit(fr: Frame) -> Frame:
    ok = torch.ones(fr.nrows, dtype=torch.bool, device=fr.device)
    for v in fr.vecs:
        ok &= ~torch.isnan(v.as_float())
    return fr.rows(torch.nonzero(ok).flatten())


def cut(fr: Frame, breaks, labels=None, include_lowest=False, right=True, digits=3) -> Frame:
    x = fr.vecs[0].as_float()
    b = torch.tensor(sorted(float(v) for v in breaks), dtype=torch.float32, device=x.device)
    nb = b.numel() - 1
    if labels is None or len(labels) == 0:
        fmt = lambda v: f"{v:.{digits}g}"  # noqa: E731
        labels = [(f"({fmt(b[i])},{fmt(b[i + 1])}]" if right else f"[{fmt(b[i])},{fmt(b[i + 1])})")
                  for i in range(nb)]
    idx = torch.bucketize(x, b, right=not right) - 1      # right-closed: (b_i, b_i+1]
    if include_lowest:
        edge = b[0] if right else b[-1]
        idx = torch.where(x == edge, torch.full_like(idx, 0 if right else nb - 1), idx)
    bad = (idx < 0) | (idx >= nb) | torch.isnan(x)
    codes = torch.where(bad, torch.full_like(idx, -1), idx).to(torch.int32)
    return Frame([Vec(fr.names[0], codes, ENUM, [str(s) for s in labels])])


def relevel(fr: Frame, level: str) -> Frame:
    v = fr.vecs[0]
    if v.vtype != ENUM or level not in v.domain:
        raise ValueError(f"relevel: {level!r} is not a level of {v.name}")
    dom = [level] + [d for d in v.domain if d != level]
    pos = {d: i for i, d in enumerate(dom)}
    lut = torch.tensor([pos[d] for d in v.domain] + [-1], dtype=torch.int32, device=v.data.device)
    c = v.data.long()
    c = torch.where(c < 0, torch.full_like(c, len(v.domain)), c)
    return Frame([Vec(v.name, lut[c], ENUM, dom)])


def stratified_split(fr: Frame, test_frac: float, seed: int, comm) -> Frame:
    """H2O h2o.random_stratified_split: per class, ~test_frac of rows -> "test"."""
    v = fr.vecs[0]
    g = torch.Generator().manual_seed(int(seed) + 7919 * _rank(comm))
    u = torch.rand(fr.nrows, generator=g, dtype=torch.float64).to(v.data.device)
    codes = v.data.long() if v.vtype == ENUM else torch.bucketize(v.as_float(), torch.unique(v.as_float()))
    out = torch.zeros(fr.nrows, dtype=torch.int32, device=v.data.device)
    for c in torch.unique(codes).tolist():
        m = codes == c
        k = int(m.sum())
        if k == 0:
            continue
        # rank the class rows by their random draw: the lowest test_frac go to test
        r = torch.argsort(torch.argsort(u[m]))
        out[m] = (r < int(round(test_frac * k))).to(torch.int32)
    return Frame([Vec("test_train_split", 1 - out, ENUM, ["test", "train"])])


# ---------------------------------------------------------------------------
# local pass + collectives
# ---------------------------------------------------------------------------
def scale(fr: Frame, center=True, scl=True, comm=None) -> Frame:
    out = []
    for v in fr.vecs:
        x = v.as_float().double()
        ok = ~torch.isnan(x)
        st = torch.stack([ok.double().sum(), torch.where(ok, x, 0).sum(), torch.where(ok, x * x, 0).sum()])
        st = _allreduce(st, comm)
        n, s1, s2 = (float(a) for a in st)
        mean = s1 / max(n, 1)
        sd = math.sqrt(max((s2 - n * mean * mean) / max(n - 1, 1), 0.0))
        y = x - mean if center else x
        if scl:
            y = y / (sd if sd > 0 else 1.0)
        out.append(Vec(v.name, y.float(), REAL))
    return Frame(out)


def cumulative(fr: Frame, how: str, comm=None) -> Frame:
    out = []
    for v in fr.vecs:
        x = v.as_float().double()
        if how == "cumsum":
            loc = torch.cumsum(torch.nan_to_num(x, nan=0.0), 0)
            tot = float(loc[-1]) if loc.numel() else 0.0
            prev = _gather_objects(comm, tot)[: _rank(comm)]
            y = loc + sum(prev)
        elif how == "cumprod":
            loc = torch.cumprod(torch.nan_to_num(x, nan=1.0), 0)
            tot = float(loc[-1]) if loc.numel() else 1.0
            prev = _gather_objects(comm, tot)[: _rank(comm)]
            y = loc * float(np.prod(prev)) if prev else loc
        elif how in ("cummin", "cummax"):
            fill = float("inf") if how == "cummin" else float("-inf")
            xx = torch.nan_to_num(x, nan=fill)
            loc = (torch.cummin if how == "cummin" else torch.cummax)(xx, 0).values
            tot = float(loc[-1]) if loc.numel() else fill
            prev = _gather_objects(comm, tot)[: _rank(comm)]
            if prev:
                p = min(prev) if how == "cummin" else max(prev)
                loc = torch.minimum(loc, torch.tensor(p, dtype=loc.dtype, device=loc.device)) if how == "cummin" \
                    else torch.maximum(loc, torch.tensor(p, dtype=loc.dtype, device=loc.device))
            y = loc
        else:
            raise ValueError(how)
        y = torch.where(torch.isnan(x), torch.full_like(y, float("nan")), y)
        out.append(Vec(v.name, y.float(), REAL))
    return Frame(out)


def kfold_column(fr: Frame, nfolds: int, seed: int, comm=None, how="random") -> Frame:
    n = fr.nrows
    base = row_base(n, comm)
    ids = torch.arange(base, base + n, dtype=torch.int64, device=fr.device)
    if how == "modulo":
        f = ids % nfolds
    else:
        s = int(seed if seed is not None and seed >= 0 else 42)
        # hash of (global row, seed): independent of the sharding
        h = (ids * 0x9E3779B1 + s * 0x85EBCA77) & 0xFFFFFFFF
        h = (h ^ (h >> 16)) * 0x45D9F3B & 0xFFFFFFFF
        h = h ^ (h >> 16)
        f = h % nfolds
    return Frame([Vec("fold", f.to(torch.float32), INT)])


def which(fr: Frame, comm=None) -> Frame:
    x = fr.vecs[0].as_float()
    base = row_base(fr.nrows, comm)
    idx = torch.nonzero(torch.nan_to_num(x, nan=0.0) != 0).flatten() + base
    return Frame([Vec("which", idx.to(torch.float32), INT)])


def quantile(fr: Frame, probs, comm=None, weights: Frame | None = None) -> Frame:
    """Exact type-7 quantiles (H2O "interpolate") per column by distributed
    bisection: each step all-reduces the count of values <= a pivot."""
    rows = []
    for v in fr.vecs:
        x = v.as_float().double()
        x = x[~torch.isnan(x)]
        st = torch.stack([torch.tensor(float(x.numel()), dtype=torch.float64, device=x.device),
                          x.min() if x.numel() else torch.tensor(math.inf, dtype=torch.float64, device=x.device),
                          -x.max() if x.numel() else torch.tensor(math.inf, dtype=torch.float64, device=x.device)])
        cnt = _allreduce(st[:1].clone(), comm)
        mm = _allreduce(st[1:].clone(), comm, "min")
        N = int(cnt[0])
        lo_all, hi_all = float(mm[0]), -float(mm[1])

        def kth(k):   # k-th smallest (0-based) over all ranks
            lo, hi = lo_all, hi_all
            for _ in range(100):
                if lo >= hi:
                    break
                mid = lo + (hi - lo) / 2
                if mid <= lo or mid >= hi:
                    break
                c = _allreduce(torch.tensor([float((x <= mid).sum())], dtype=torch.float64, device=x.device), comm)
                if float(c[0]) >= k + 1:
                    hi = mid
                else:
                    lo = mid
            # snap to the smallest data value >= lo with rank >= k
            cand = x[x >= lo]
            m = torch.tensor([float(cand.min()) if cand.numel() else math.inf], dtype=torch.float64, device=x.device)
            return float(_allreduce(m, comm, "min")[0])

        col = []
        for p in probs:
            if N == 0:
                col.append(float("nan"))
                continue
            h = (N - 1) * float(p)
            k0 = int(math.floor(h))
            a = kth(k0)
            b = kth(min(k0 + 1, N - 1)) if h > k0 else a
            col.append(a + (h - k0) * (b - a))
        rows.append(col)
    dev = fr.device
    vecs = [Vec("Probs", torch.tensor([float(p) for p in probs], dtype=torch.float32, device=dev), REAL)]
    vecs += [Vec(f"{v.name}Quantiles", torch.tensor(r, dtype=torch.float32, device=dev), REAL)
             for v, r in zip(fr.vecs, rows)]
    return Frame(vecs)


def impute(fr: Frame, col: int, method: str = "mean", comm=None, values=None) -> tuple[Frame, list]:
    """H2O h2o.impute on one column (in place); returns (frame, [fill value])."""
    v = fr.vecs[col]
    m = method.lower()
    if v.vtype == ENUM:
        c = v.data.long()
        cnt = torch.zeros(len(v.domain or []) + 1, dtype=torch.float64, device=c.device)
        cnt.index_add_(0, torch.where(c < 0, len(v.domain or []), c), torch.ones_like(c, dtype=torch.float64))
        cnt = _allreduce(cnt, comm)[:-1]
        mode = int(torch.argmax(cnt)) if values is None else int(values[0])
        nv = Vec(v.name, torch.where(v.data < 0, torch.full_like(v.data, mode), v.data), ENUM, v.domain)
        fill = [mode]
    else:
        x = v.as_float()
        if values is not None:
            val = float(values[0])
        elif m == "median":
            val = float(quantile(Frame([v]), [0.5], comm).vecs[1].data[0])
        elif m == "mode":
            ok = x[~torch.isnan(x)]
            u, cnts = torch.unique(ok, return_counts=True)
            part = list(zip(u.tolist(), cnts.tolist()))
            allp = {}
            for lst in _gather_objects(comm, part):
                for a, b in lst:
                    allp[a] = allp.get(a, 0) + b
            val = max(allp.items(), key=lambda t: (t[1], -t[0]))[0] if allp else float("nan")
        else:
            ok = ~torch.isnan(x)
            st = _allreduce(torch.stack([ok.double().sum(), torch.where(ok, x.double(), 0).sum()]), comm)
            val = float(st[1] / st[0].clamp_min(1))
        nv = Vec(v.name, torch.where(torch.isnan(x), torch.full_like(x, val), x), v.vtype, v.domain)
        fill = [val]
    vecs = list(fr.vecs)
    vecs[col] = nv
    return Frame(vecs, key=fr.key), fill


# ---------------------------------------------------------------------------
# aggregations (result on the leader)
# ---------------------------------------------------------------------------
_AGGS = ("nrow", "count", "sum", "mean", "min", "max", "sd", "var", "ss", "mode", "median")


def _group_keys(fr: Frame, gcols: list[int]):
    """Local unique group keys (as tuples of python values) and inverse ids."""
    cols = []
    for i in gcols:
        v = fr.vecs[i]
        cols.append(v.data.long() if v.vtype == ENUM else v.as_float().double())
    if fr.nrows == 0:
        return [], torch.zeros(0, dtype=torch.long, device=fr.device)
    K = torch.stack([c.double() for c in cols], 1)
    K = torch.nan_to_num(K, nan=float("-inf"))        # NA group sorts first
    uk, inv = torch.unique(K, dim=0, return_inverse=True)
    return [tuple(r) for r in uk.cpu().tolist()], inv


def group_by(fr: Frame, gcols: list[int], aggs: list[tuple[str, int, str]], comm=None) -> Frame:
    """``aggs``: (agg, column index, na handling "all"|"rm"|"ignore")."""
    keys, inv = _group_keys(fr, gcols)
    G = len(keys)
    partial = []   # per agg: per group [n, s1, s2, min, max] or value lists (median / mode)
    for agg, ci, na in aggs:
        if agg not in _AGGS:
            raise ValueError(f"group_by: unsupported aggregate {agg!r}")
        v = fr.vecs[ci]
        x = v.as_float().double()
        ok = ~torch.isnan(x)
        if agg in ("median", "mode"):
            vals = [[] for _ in range(G)]
            if G:
                inv_c, x_c = inv.cpu().numpy(), x.cpu().numpy()
                for g, val in zip(inv_c, x_c):
                    if not np.isnan(val):
                        vals[g].append(float(val))
            partial.append(vals)
            continue
        st = torch.zeros((G, 6), dtype=torch.float64, device=x.device)
        if G:
            xo = torch.where(ok, x, torch.zeros_like(x))
            st[:, 0].index_add_(0, inv, ok.double())
            st[:, 1].index_add_(0, inv, xo)
            st[:, 2].index_add_(0, inv, xo * xo)
            st[:, 3] = torch.full((G,), math.inf, dtype=torch.float64, device=x.device).scatter_reduce(
                0, inv, torch.where(ok, x, torch.full_like(x, math.inf)), "amin")
            st[:, 4] = torch.full((G,), -math.inf, dtype=torch.float64, device=x.device).scatter_reduce(
                0, inv, torch.where(ok, x, torch.full_like(x, -math.inf)), "amax")
            st[:, 5].index_add_(0, inv, torch.ones_like(x))                # rows incl. NA
        partial.append(st.cpu().numpy())
    gathered = _gather_objects(comm, (keys, partial))
    if _rank(comm) != 0:
        names = [fr.names[i] for i in gcols] + [_agg_name(a, fr.names[c]) for a, c, _ in aggs]
        return Frame([Vec(n, torch.zeros(0, device=fr.device), REAL) for n in names])
    merged: dict = {}
    for keys_r, part_r in gathered:
        for gi, k in enumerate(keys_r):
            slot = merged.setdefault(k, [None] * len(aggs))
            for ai, (agg, _, _) in enumerate(aggs):
                p = part_r[ai][gi]
                if agg in ("median", "mode"):
                    slot[ai] = (slot[ai] or []) + list(p)
                else:
                    if slot[ai] is None:
                        slot[ai] = np.array(p, np.float64)
                    else:
                        s = slot[ai]
                        slot[ai] = np.array([s[0] + p[0], s[1] + p[1], s[2] + p[2], min(s[3], p[3]),
                                             max(s[4], p[4]), s[5] + p[5]])
    order = sorted(merged)
    dev = fr.device
    out = []
    for j, i in enumerate(gcols):
        v = fr.vecs[i]
        col = [k[j] for k in order]
        if v.vtype == ENUM:
            out.append(Vec(v.name, torch.tensor([int(c) if c != float("-inf") else -1 for c in col],
                                                dtype=torch.int32, device=dev), ENUM, v.domain))
        else:
            out.append(Vec(v.name, torch.tensor([c if c != float("-inf") else float("nan") for c in col],
                                                dtype=torch.float32, device=dev), REAL))
    for ai, (agg, ci, na) in enumerate(aggs):
        res = []
        for k in order:
            s = merged[k][ai]
            if agg in ("median", "mode"):
                if not s:
                    res.append(float("nan"))
                elif agg == "median":
                    res.append(float(np.median(s)))
                else:
                    u, c = np.unique(np.asarray(s), return_counts=True)
                    res.append(float(u[np.argmax(c)]))
                continue
            n, s1, s2, mn, mx, rows = s
            if agg in ("nrow", "count"):
                res.append(rows if na == "all" else n)
            elif agg == "sum":
                res.append(s1)
            elif agg == "mean":
                res.append(s1 / n if n else float("nan"))
            elif agg == "min":
                res.append(mn if n else float("nan"))
            elif agg == "max":
                res.append(mx if n else float("nan"))
            elif agg == "ss":
                res.append(s2)
            else:
                var = (s2 - s1 * s1 / n) / (n - 1) if n > 1 else float("nan")
                res.append(math.sqrt(max(var, 0.0)) if agg == "sd" else var)
        out.append(Vec(_agg_name(agg, fr.names[ci]), torch.tensor(res, dtype=torch.float32, device=dev), REAL))
    return Frame(out)


def _agg_name(agg, col):
    return "nrow" if agg in ("nrow", "count") else f"{agg}_{col}"


def unique(fr: Frame, comm=None, include_nas=False) -> Frame:
    g = group_by(fr, list(range(fr.ncols)), [], comm)
    if not include_nas and g.nrows:
        return na_omit(g)
    return g


def table(fr: Frame, comm=None) -> Frame:
    g = group_by(fr, list(range(fr.ncols)), [("nrow", 0, "all")], comm)
    vecs = list(g.vecs)
    vecs[-1] = Vec("Count", vecs[-1].data, INT)
    return Frame(vecs)


# ---------------------------------------------------------------------------
# leader-resident: sort / merge
# ---------------------------------------------------------------------------
def sort(fr: Frame, cols: list[int], ascending=None, comm=None) -> Frame:
    g = gather_to_leader(fr, comm)
    if g is None:
        return _empty_like(fr)
    asc = list(ascending) if ascending else [True] * len(cols)
    idx = torch.arange(g.nrows, device=g.device)
    # stable sort from the last key to the first; NAs first (H2O)
    for ci, a in reversed(list(zip(cols, asc))):
        x = g.vecs[ci].as_float()[idx].double()
        key = torch.where(torch.isnan(x), torch.full_like(x, -math.inf), x)
        o = torch.sort(key if a else -key, stable=True).indices
        if not a:   # NAs still first
            na = torch.isnan(x[o])
            o = torch.cat([o[na], o[~na]])
        idx = idx[o]
    return g.rows(idx)


def merge(left: Frame, right: Frame, all_x=False, all_y=False, by_x=None, by_y=None, comm=None) -> Frame:
    lg = gather_to_leader(left, comm)
    rg = gather_to_leader(right, comm)
    if _rank(comm) != 0:
        names = left.names + [n for n in right.names if n not in (by_y or [])]
        return Frame([Vec(n, torch.zeros(0, device=left.device), REAL) for n in names])
    import pandas as pd

    L, R = lg.to_pandas(), rg.to_pandas()
    bx = [left.names[i] for i in by_x] if by_x else [c for c in left.names if c in right.names]
    by = [right.names[i] for i in by_y] if by_y else bx
    how = "outer" if (all_x and all_y) else ("left" if all_x else ("right" if all_y else "inner"))
    M = pd.merge(L, R, left_on=bx, right_on=by, how=how, suffixes=("", "0"), sort=True)
    if by != bx:
        M = M.drop(columns=[c for c in by if c not in bx])
    out = Frame.from_pandas(M, device=left.device)
    return out
