"""Model explanations: SHAP contributions and partial dependence.

``predict_contributions(model, frame)`` (H2O ``predict_contributions``):
path-dependent TreeSHAP for GBM / DRF / XGBoost / Isolation-Forest-free
tree ensembles with one tree per iteration (regression and binomial, like
H2O).  Output columns are the predictors plus ``BiasTerm``; each row sums
to the model's raw margin (link space).  On the GPU the contributions come
from csrc/explain_kernels.hip (one thread per row over a flattened path
table); on CPU frames the same path formula runs vectorised in NumPy.

``partial_dependence(model, frame, col, nbins)`` (H2O PartialDependence):
mean / sd / standard error of the model response with ``col`` forced to
each grid value (``nbins`` equally spaced values between the column's min
and max, every level for categorical columns), scored on the device.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .frame.frame import ENUM, Frame, Vec
from .models.base import ModelCategory


# ---------------------------------------------------------------------------
# TreeSHAP
# ---------------------------------------------------------------------------
def tree_paths(trees: np.ndarray, scale: float = 1.0, catbits: np.ndarray | None = None):
    """Flatten every root-to-leaf path: returns (leaves [L][4] int32 =
    {first element, m, value bits, tree}, elems [E][4] float32 = {feature |
    na_ok << 30 | categorical << 29, z, lo, hi}, expected value, max unique
    features, sets [S][8] uint32).  A categorical feature's element keeps the
    set of levels the path allows (intersection of its group splits' sides)
    in ``sets[lo]``."""
    leaves, elems, sets = [], [], []
    expected = 0.0
    maxm = 1
    full = np.full(8, 0xFFFFFFFF, np.uint32)
    for t in range(trees.shape[0]):
        tr = trees[t]
        cb = None if catbits is None else catbits[t]
        # stack entries: (node, {feature: [z, lo, hi, na_ok, level set or None]})
        stack = [(0, {})]
        while stack:
            i, path = stack.pop()
            nd = tr[i]
            if nd["feat"] < 0:
                v = float(nd["value"]) * scale
                m = len(path)
                zprod = 1.0
                start = len(elems)
                for f, (z, lo, hi, na, st) in path.items():
                    if st is not None:
                        elems.append((np.int32(f | (int(na) << 30) | (1 << 29)).view(np.float32), z,
                                      float(len(sets)), 0.0))
                        sets.append(st)
                    else:
                        elems.append((np.int32(f | (int(na) << 30)).view(np.float32), z, lo, hi))
                    zprod *= z
                leaves.append((start, m, np.float32(v).view(np.int32), t))
                expected += v * zprod
                maxm = max(maxm, m)
                continue
            f, thr, left = int(nd["feat"]), float(nd["thr"]), int(nd["left"])
            is_cat = cb is not None and (int(nd["na_left"]) & 2) != 0
            w = float(nd["weight"])
            for child, go_left in ((left, True), (left + 1, False)):
                cw = float(tr[child]["weight"])
                r = cw / w if w > 0 else 0.0
                z, lo, hi, na, st = path.get(f, (1.0, -np.inf, np.inf, True, None))
                if is_cat:
                    side = cb[i] if go_left else ~cb[i]
                    st = (full if st is None else st) & side
                elif go_left:
                    hi = min(hi, thr)
                else:
                    lo = max(lo, thr)
                na = na and (bool(int(nd["na_left"]) & 1) == go_left)
                p2 = dict(path)
                p2[f] = (z * r, lo, hi, na, st)
                stack.append((child, p2))
    lv = np.asarray(leaves, np.int32).reshape(-1, 4)
    el = np.asarray([(e[0], e[1], e[2], e[3]) for e in elems], np.float32).reshape(-1, 4) if elems else \
        np.zeros((0, 4), np.float32)
    if elems:
        el[:, 0] = np.asarray([e[0] for e in elems], np.float32)
    st = np.asarray(sets, np.uint32).reshape(-1, 8) if sets else np.zeros((1, 8), np.uint32)
    return lv, el, expected, maxm, st


def shapley_weights(M: int) -> np.ndarray:
    """w[m][k] = k! (m-1-k)! / m! for 1 <= m <= M, 0 <= k < m (row/col M+1)."""
    w = np.zeros((M + 1, M + 1), np.float64)
    for m in range(1, M + 1):
        for k in range(m):
            w[m, k] = math.exp(math.lgamma(k + 1) + math.lgamma(m - k) - math.lgamma(m + 1))
    return w


def _bucket(maxm: int) -> int:
    return 8 if maxm <= 8 else (16 if maxm <= 16 else 32)


def _shap_numpy(X: np.ndarray, lv, el, maxm, sets=None) -> np.ndarray:
    F, n = X.shape
    out = np.zeros((F, n), np.float64)
    W = shapley_weights(maxm)
    for start, m, vbits, _ in lv:
        v = float(np.int32(vbits).view(np.float32))
        if m == 0:
            continue
        E = el[start: start + m]
        feats = E[:, 0].view(np.int32)
        f = feats & 0x1FFFFFFF
        na_ok = (feats >> 30) & 1
        iscat = (feats >> 29) & 1
        z = E[:, 1].astype(np.float64)
        x = X[f]                                       # [m][n]
        with np.errstate(invalid="ignore"):
            o = np.where(np.isnan(x), na_ok[:, None].astype(np.float64),
                         ((x > E[:, 2:3]) & (x <= E[:, 3:4])).astype(np.float64))
        if sets is not None and iscat.any():
            from .models.tree.structs import bitset_has

            for j in np.nonzero(iscat)[0]:
                c = np.where(np.isnan(x[j]), -1, x[j]).astype(np.int64)
                oor = (c < 0) | (c > 255)
                inside = bitset_has(sets[int(E[j, 2])], c).astype(np.float64)
                o[j] = np.where(np.isnan(x[j]) | oor, float(na_ok[j]), inside)
        P = np.zeros((m + 1, n))
        P[0] = 1.0
        for j in range(m):
            P[1:] = z[j] * P[1:] + o[j] * P[:-1]
            P[0] *= z[j]
        for i in range(m):
            s = np.zeros(n)
            carry = np.zeros(n)
            s1 = np.zeros(n)
            for k in range(m, 0, -1):
                q = P[k] - z[i] * carry
                s1 += q * W[m, k - 1]
                carry = q
            if z[i] > 0:
                s0 = (P[:m] * W[m, :m, None]).sum(0) / z[i]
            else:
                s0 = np.zeros(n)
            s = np.where(o[i] != 0, s1, s0)
            out[f[i]] += v * (o[i] - z[i]) * s
    return out


def predict_contributions(model, frame: Frame) -> Frame:
    ens = getattr(model, "ens", None)
    if ens is None or model.algo not in ("gbm", "drf", "xgboost", "generic"):
        raise NotImplementedError(f"predict_contributions is available for tree models, not {model.algo}")
    if ens.K != 1:
        raise NotImplementedError("predict_contributions supports regression and binomial tree models (as in H2O)")
    frame = model.adapt_frame(frame)
    X = model._matrix(frame) if hasattr(model, "_matrix") else frame.feature_matrix(model.x)
    F, n = X.shape
    nt = ens.ntrees
    scale = 1.0 / nt if (ens.average and nt > 0) else 1.0
    cb = getattr(ens, "catbits", None)
    lv, el, expected, maxm, sets = tree_paths(ens.trees[:nt], scale, None if cb is None else cb[:nt])
    bias = expected + (0.0 if ens.average else float(ens.init_f[0]))
    if X.is_cuda:
        from .ops import P, check, explain_lib, stream

        dev = X.device
        Xc = X.float().contiguous()
        M = _bucket(maxm)
        wt = torch.from_numpy(shapley_weights(M).astype(np.float32)).to(dev)
        lvd = torch.from_numpy(lv).to(dev)
        eld = torch.from_numpy(el if el.size else np.zeros((1, 4), np.float32)).to(dev)
        out = torch.zeros((F, n), dtype=torch.float32, device=dev)
        setd = torch.from_numpy(sets.view(np.int32).copy()).to(dev)
        check(explain_lib().h2omx_tree_shap(P(Xc), Xc.stride(0), n, F, P(lvd), int(lv.shape[0]), P(eld), P(wt),
                                            maxm, P(out), P(setd), stream(dev)), "tree_shap")
    else:
        out = torch.from_numpy(_shap_numpy(X.double().numpy(), lv, el, maxm, sets).astype(np.float32))
    vecs = [Vec(c, out[j], "real") for j, c in enumerate(model.x)]
    vecs.append(Vec("BiasTerm", torch.full((n,), float(bias), dtype=torch.float32, device=out.device), "real"))
    return Frame(vecs)


# ---------------------------------------------------------------------------
# Partial dependence
# ---------------------------------------------------------------------------
def _response(model, P: torch.Tensor, target: str | None) -> torch.Tensor:
    if model.category == ModelCategory.BINOMIAL:
        return P[-1]
    if model.category == ModelCategory.MULTINOMIAL:
        dom = list(model.response_domain)
        return P[dom.index(target) if target is not None else 0]
    return P[0]


def partial_dependence(model, frame: Frame, col: str, nbins: int = 20, target: str | None = None,
                       user_splits=None, comm=None) -> dict:
    """H2O PartialDependence for one column: {col, mean_response,
    stddev_response, std_error_mean_response} per grid value."""
    frame = model.adapt_frame(frame)
    v = frame.vec(col)
    n = frame.nrows
    if v.vtype == ENUM:
        dom = list(model.feature_domains.get(col) or v.domain or [])
        grid = list(range(len(dom)))
        labels = dom
    else:
        if user_splits is not None:
            grid = [float(a) for a in user_splits]
        else:
            x = v.as_float()
            ok = ~torch.isnan(x)
            lo = x[ok].min() if bool(ok.any()) else torch.tensor(0.0)
            hi = x[ok].max() if bool(ok.any()) else torch.tensor(0.0)
            mm = torch.stack([lo.float(), -hi.float()]).to(x.device)
            if comm is not None and comm.world_size > 1:
                comm.all_reduce_(mm, "min")
            lo_v, hi_v = float(mm[0]), float(-mm[1])
            grid = list(np.linspace(lo_v, hi_v, nbins)) if hi_v > lo_v else [lo_v]
        labels = grid
    rows = []
    for g in grid:
        if v.vtype == ENUM:
            nv = Vec(col, torch.full((n,), int(g), dtype=torch.int32, device=v.data.device), ENUM, list(dom))
        else:
            nv = Vec(col, torch.full((n,), float(g), dtype=torch.float32, device=v.data.device), v.vtype)
        fr = Frame([nv if u.name == col else u for u in frame.vecs])
        r = _response(model, model.predict_raw(fr), target).double()
        st = torch.stack([r.sum(), (r * r).sum(), torch.tensor(float(n), dtype=torch.float64, device=r.device)])
        if comm is not None and comm.world_size > 1:
            comm.all_reduce_(st)
        s, s2, cnt = (float(a) for a in st)
        mean = s / max(cnt, 1.0)
        sd = math.sqrt(max(s2 / max(cnt, 1.0) - mean * mean, 0.0) * cnt / max(cnt - 1.0, 1.0))
        rows.append({col: labels[len(rows)], "mean_response": mean, "stddev_response": sd,
                     "std_error_mean_response": sd / math.sqrt(max(cnt, 1.0))})
    return {"column": col, "target": target, "data": rows}
