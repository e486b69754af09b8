"""More H2O model-introspection and explanation APIs.

* ``predict_leaf_node_assignment(model, frame, type)``: for every tree (and
  class), the leaf each row reaches, as an "LRRL" path (``Path``) or a node
  id (``Node_ID``).  Columns are ``T<t>.C<k>``.
* ``staged_predict_proba(model, frame)``: the prediction after each boosting
  iteration (GBM / XGBoost), or the running average of trees (DRF).
* ``feature_frequencies(model, frame)``: how often each feature is tested
  on the paths of each row, summed over the trees.
* ``glm_contributions(model, frame)``: exact linear SHAP values for GLMs,
  beta_j (x_j - mean_j) in link space, with one-hot columns folded back onto
  their categorical column, plus ``BiasTerm``.
* ``ice(model, frame, col)``: per-row individual conditional expectation
  curves (the per-row version of partial dependence).
* ``fairness_metrics(model, frame, protected_columns, reference,
  favorable_class)``: per protected group, the size, AUC, accuracy,
  selected ratio, TPR, FPR and precision.  Also the adverse impact ratio
  (AIR) against the reference group, with a Fisher exact / chi-square
  p-value.
* ``model_correlation(models, frame)``, ``varimp_heatmap(models)``,
  ``residual_analysis(model, frame)`` and ``learning_curve(model)``: the
  data behind H2O's explain plots.
* ``explain(models, frame)``: every applicable piece, as one dict.

All tree walks run as batched device gathers over the ensemble's node table.
Every statistic that aggregates rows is all-reduced when a communicator is given.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .frame.frame import ENUM, Frame, Vec
from .models.base import ModelCategory


def _tree_models(model):
    ens = getattr(model, "ens", None)
    if ens is None:
        raise NotImplementedError(f"{model.algo}: tree models only (GBM / DRF / XGBoost)")
    return ens


def _walk(tree: np.ndarray, X: torch.Tensor, catbits: np.ndarray | None = None):
    """Leaf index and path bits (bit d = went right at depth d) for every row."""
    from .models.tree.structs import TreeWalker

    dev = X.device
    tw = TreeWalker(tree, catbits, dev)
    feat, left = tw.feat, tw.left
    n = X.shape[1]
    idx = torch.zeros(n, dtype=torch.long, device=dev)
    bits = torch.zeros(n, dtype=torch.long, device=dev)
    depth = torch.zeros(n, dtype=torch.long, device=dev)
    rows = torch.arange(n, device=dev)
    used = []
    for _ in range(64):
        f = feat[idx]
        inner = f >= 0
        if not bool(inner.any()):
            break
        v = X[f.clamp_min(0), rows]
        go_left = tw.go_left(idx, v)
        right = inner & ~go_left
        used.append(torch.where(inner, f, torch.full_like(f, -1)))
        bits = bits | (right.long() << depth.clamp(max=62))
        depth = depth + inner.long()
        idx = torch.where(inner, left[idx] + right.long(), idx)
    return idx, bits, depth, used


def _cb(ens, t):
    cb = getattr(ens, "catbits", None)
    return None if cb is None else cb[t]


def _X(model, frame):
    frame = model.adapt_frame(frame)
    return model._matrix(frame) if hasattr(model, "_matrix") else frame.feature_matrix(model.x)


def predict_leaf_node_assignment(model, frame: Frame, type: str = "Path") -> Frame:  # noqa: A002
    ens = _tree_models(model)
    X = _X(model, frame).float()
    vecs = []
    for t in range(ens.ntrees * ens.K):
        idx, bits, depth, _ = _walk(ens.trees[t], X, _cb(ens, t))
        name = f"T{t // ens.K + 1}.C{t % ens.K + 1}"
        if str(type).lower() == "node_id":
            vecs.append(Vec(name, idx.float(), "int"))
            continue
        key = depth * (1 << 40) + bits
        u, inv = torch.unique(key, return_inverse=True)
        dom = []
        for k in u.cpu().tolist():
            d, b = k >> 40, k & ((1 << 40) - 1)
            dom.append("".join("R" if (b >> i) & 1 else "L" for i in range(d)))
        vecs.append(Vec(name, inv.to(torch.int32), ENUM, dom))
    return Frame(vecs)


def staged_predict_proba(model, frame: Frame) -> Frame:
    ens = _tree_models(model)
    X = _X(model, frame).float()
    K, n = ens.K, X.shape[1]
    acc = torch.zeros((K, n), dtype=torch.float64, device=X.device)
    if not ens.average:
        acc += torch.from_numpy(ens.init_f.astype(np.float64)).to(X.device)[:, None]
    vecs = []
    for t in range(ens.ntrees):
        for k in range(K):
            idx, _, _, _ = _walk(ens.trees[t * K + k], X, _cb(ens, t * K + k))
            acc[k] += torch.from_numpy(ens.trees[t * K + k]["value"].astype(np.float64)).to(X.device)[idx]
        margin = (acc / (t + 1)) if ens.average else acc
        P = model._link(margin.float())
        if model.category == ModelCategory.BINOMIAL:
            vecs.append(Vec(f"T{t + 1}.C1", P[-1].float(), "real"))
        else:
            for k in range(P.shape[0]):
                vecs.append(Vec(f"T{t + 1}.C{k + 1}", P[k].float(), "real"))
    return Frame(vecs)


def feature_frequencies(model, frame: Frame) -> Frame:
    ens = _tree_models(model)
    X = _X(model, frame).float()
    F, n = X.shape
    cnt = torch.zeros((F + 1, n), dtype=torch.float32, device=X.device)
    for t in range(ens.ntrees * ens.K):
        _, _, _, used = _walk(ens.trees[t], X, _cb(ens, t))
        for f in used:
            cnt.scatter_add_(0, torch.where(f >= 0, f, torch.full_like(f, F))[None, :],
                             torch.ones((1, n), device=X.device))
    return Frame([Vec(c, cnt[j], "real") for j, c in enumerate(model.x)])


def glm_contributions(model, frame: Frame) -> Frame:
    if model.algo not in ("glm", "gam") or model.family == "multinomial" or model.family == "ordinal":
        raise NotImplementedError("linear contributions: single-output GLMs")
    frame = model.adapt_frame(frame)
    spec = getattr(model, "interaction_spec", None)
    if spec:
        from .models.glm_extras import apply_interactions

        frame = apply_interactions(frame, spec)
    d = model.design
    Xs = d.transform(d.raw_matrix(frame)).double()
    b = torch.from_numpy(model.beta_std[0].astype(np.float64)).to(Xs.device)
    p = Xs.shape[0]
    # standardised design columns are centred at the training means: x_std = (x - mean) / sd
    contrib = b[:p, None] * Xs
    cols, out = [], []
    for c in d.x:
        js = [j for j, (col, _) in enumerate(d.spec) if col == c]
        if not js:
            continue
        cols.append(c)
        out.append(contrib[js].sum(0))
    bias = float(b[p])
    vecs = [Vec(c, v.float(), "real") for c, v in zip(cols, out)]
    vecs.append(Vec("BiasTerm", torch.full((Xs.shape[1],), bias, dtype=torch.float32, device=Xs.device), "real"))
    return Frame(vecs)


def ice(model, frame: Frame, col: str, nbins: int = 20, target: str | None = None, max_rows: int = 1000) -> dict:
    """Per-row ICE curves for up to ``max_rows`` rows: {grid, curves [rows][grid]}."""
    from .explain import _response

    frame = model.adapt_frame(frame)
    n = min(frame.nrows, int(max_rows))
    sub = frame.rows(torch.arange(n, device=frame.device))
    v = sub.vec(col)
    if v.vtype == ENUM:
        dom = list(model.feature_domains.get(col) or v.domain or [])
        grid = list(range(len(dom)))
        labels = dom
    else:
        x = v.as_float()
        ok = ~torch.isnan(x)
        lo, hi = (float(x[ok].min()), float(x[ok].max())) if bool(ok.any()) else (0.0, 0.0)
        grid = list(np.linspace(lo, hi, nbins)) if hi > lo else [lo]
        labels = grid
    curves = []
    for g in grid:
        if v.vtype == ENUM:
            nv = Vec(col, torch.full((n,), int(g), dtype=torch.int32, device=v.data.device), ENUM, list(dom))
        else:
            nv = Vec(col, torch.full((n,), float(g), dtype=torch.float32, device=v.data.device), v.vtype)
        fr = Frame([nv if u.name == col else u for u in sub.vecs])
        curves.append(_response(model, model.predict_raw(fr), target).double().cpu())
    C = torch.stack(curves, 1).numpy()
    return {"column": col, "grid": labels, "curves": C.tolist(), "mean": C.mean(0).tolist()}


def _binary_rates(p1: torch.Tensor, y: torch.Tensor, thr: float):
    pred = (p1 >= thr).double()
    yy = y.double()
    tp = float((pred * yy).sum())
    fp = float((pred * (1 - yy)).sum())
    fn = float(((1 - pred) * yy).sum())
    tn = float(((1 - pred) * (1 - yy)).sum())
    return tp, fp, fn, tn


def fairness_metrics(model, frame: Frame, protected_columns, reference=None, favorable_class=None,
                     comm=None) -> dict:
    """H2O ``model.fairness_metrics``: per-group metrics of a binomial model
    and the adverse impact ratio against the reference group."""
    from scipy import stats as sst

    from .metrics.core import auc_from_scores

    if model.category != ModelCategory.BINOMIAL:
        raise ValueError("fairness_metrics: binomial models")
    frame = model.adapt_frame(frame)
    P = model.predict_raw(frame)
    dom = list(model.response_domain)
    fav = dom.index(favorable_class) if favorable_class in dom else 1
    pf = P[fav].float()
    y = (frame.vec(model.y).data.long() == fav)
    thr = (model.training_metrics or {}).get("max_f1_threshold", 0.5)
    thr = thr if fav == 1 else 1 - thr
    codes = [frame.vec(c).data.long() for c in protected_columns]
    doms = [list(frame.vec(c).domain or []) for c in protected_columns]
    groups = {}
    import itertools

    for combo in itertools.product(*[range(len(d)) for d in doms]):
        mask = torch.ones(frame.nrows, dtype=torch.bool, device=pf.device)
        for c, k in zip(codes, combo):
            mask &= c == k
        name = tuple(d[k] for d, k in zip(doms, combo))
        tp, fp, fn, tn = _binary_rates(pf[mask], y[mask], thr)
        st = torch.tensor([tp, fp, fn, tn], dtype=torch.float64)
        if comm is not None and comm.world_size > 1:
            st = torch.from_numpy(comm.all_reduce_numpy(st.numpy()))
        tp, fp, fn, tn = (float(a) for a in st)
        total = tp + fp + fn + tn
        if total == 0:
            continue
        yy = y[mask]
        try:
            auc = float(auc_from_scores(pf[mask], yy.float(), comm=comm)) if 0 < float(yy.float().mean()) < 1 else \
                float("nan")
        except Exception:  # noqa: BLE001
            auc = float("nan")
        groups[name] = {"total": total, "relativeSize": 0.0, "auc": auc, "accuracy": (tp + tn) / total,
                        "selected": tp + fp, "selectedRatio": (tp + fp) / total,
                        "tpr": tp / max(tp + fn, 1e-300), "fpr": fp / max(fp + tn, 1e-300),
                        "precision": tp / max(tp + fp, 1e-300) if tp + fp > 0 else float("nan")}
    if not groups:
        raise ValueError("fairness_metrics: no rows in any protected group")
    biggest = max(groups, key=lambda g: groups[g]["total"])
    ref = tuple(reference) if reference is not None else biggest
    if ref not in groups:
        raise ValueError(f"fairness_metrics: reference {reference} has no rows")
    N = sum(g["total"] for g in groups.values())
    R = groups[ref]
    rows = []
    for name, g in groups.items():
        g["relativeSize"] = g["total"] / N
        g["AIR_selectedRatio"] = g["selectedRatio"] / R["selectedRatio"] if R["selectedRatio"] > 0 else float("nan")
        table = [[g["selected"], g["total"] - g["selected"]], [R["selected"], R["total"] - R["selected"]]]
        if name == ref:
            pv = 1.0
        elif N < 1e5:
            pv = float(sst.fisher_exact(np.array(table, dtype=np.float64).round().astype(np.int64))[1])
        else:
            pv = float(sst.chi2_contingency(np.array(table) + 0.5)[1])
        g["p.value"] = pv
        rows.append({**{c: v for c, v in zip(protected_columns, name)}, **g})
    return {"overview": rows, "reference": list(ref), "favorable_class": dom[fav], "threshold": thr}


def model_correlation(models, frame: Frame) -> dict:
    """Pearson correlation of the models' predictions (class-1 probability
    for binomial models)."""
    from .explain import _response

    preds = [_response(m, m.predict_raw(frame), None).double().cpu().numpy() for m in models]
    C = np.corrcoef(np.stack(preds))
    return {"model_ids": [m.model_id for m in models], "correlation": C.tolist()}


def varimp_heatmap(models) -> dict:
    cols = sorted({v for m in models for v, *_ in m.varimp()})
    M = np.zeros((len(cols), len(models)))
    for j, m in enumerate(models):
        d = {v: s for v, _, s, _ in m.varimp()}
        for i, c in enumerate(cols):
            M[i, j] = d.get(c, 0.0)
    return {"variables": cols, "model_ids": [m.model_id for m in models], "scaled_importance": M.tolist()}


def residual_analysis(model, frame: Frame) -> dict:
    if model.category != ModelCategory.REGRESSION:
        raise ValueError("residual_analysis: regression models")
    fr = model.adapt_frame(frame)
    f = model.predict_raw(fr)[0].double()
    y = fr.vec(model.y).as_float().double()
    ok = ~torch.isnan(y)
    r = (y - f)[ok]
    return {"fitted": f[ok].cpu().tolist(), "residuals": r.cpu().tolist(),
            "rmse": float(torch.sqrt((r * r).mean())) if r.numel() else float("nan")}


def learning_curve(model) -> list:
    return list(model.scoring_history or [])


def explain(models, frame: Frame, columns=None, top_n_features: int = 5) -> dict:
    """H2O ``h2o.explain`` data: variable importance, partial dependence and
    ICE for the top features, SHAP summary (tree models), residuals
    (regression), model correlation and varimp heatmap (several models)."""
    from .explain import partial_dependence, predict_contributions

    models = models if isinstance(models, (list, tuple)) else [models]
    m0 = models[0]
    out: dict = {"models": [m.model_id for m in models]}
    vi = m0.varimp()
    out["varimp"] = vi
    cols = columns or [v for v, *_ in vi[:top_n_features]] or list(m0.x)[:top_n_features]
    out["pdp"] = [partial_dependence(m0, frame, c) for c in cols]
    out["ice"] = [ice(m0, frame, c, max_rows=100) for c in cols]
    if getattr(m0, "ens", None) is not None and m0.ens.K == 1:
        sh = predict_contributions(m0, frame)
        out["shap_summary"] = {c: float(sh.vec(c).data.abs().mean()) for c in m0.x}
    if m0.category == ModelCategory.REGRESSION:
        ra = residual_analysis(m0, frame)
        out["residual_analysis"] = {"rmse": ra["rmse"]}
    out["learning_curve"] = learning_curve(m0)
    if len(models) > 1:
        out["model_correlation"] = model_correlation(models, frame)
        out["varimp_heatmap"] = varimp_heatmap(models)
    return out
