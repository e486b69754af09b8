"""Top-level H2O utilities that are not tied to one estimator.

* ``make_metrics(predicted, actuals, domain=None, distribution=None,
  weights=None)``: H2O ``h2o.make_metrics``.  It computes model metrics
  from a prediction frame and an actual-response frame: binomial (class-1
  probability column), multinomial (one probability column per class) or
  regression.
* ``permutation_importance(model, frame, metric="AUTO", n_repeats=1,
  seed=-1)``: H2O ``model.permutation_importance``.  Each feature's
  importance is the increase in a loss-type metric (or the decrease in AUC /
  AUCPR) after that column is shuffled.  Scores come from device-side
  scoring passes.
* ``train_segments(estimator_cls, params, segment_columns, x, y,
  training_frame)``: H2O ``h2o.train_segments``.  It trains one model per
  combination of the segment columns' levels and returns a status table
  (segment levels, model id, status, errors).
"""
from __future__ import annotations

import itertools

import numpy as np
import torch

from .frame.frame import DKV, ENUM, Frame, Vec
from .metrics import binomial_metrics, multinomial_metrics, regression_metrics
from .models.base import ModelCategory


def make_metrics(predicted: Frame, actuals: Frame, domain=None, distribution=None, weights: Frame | None = None,
                 comm=None) -> dict:
    av = actuals.vecs[0]
    w = weights.vecs[0].as_float() if weights is not None else None
    if domain is None and av.vtype == ENUM:
        domain = list(av.domain or [])
    if domain:
        dom = list(domain)
        if av.vtype == ENUM:
            pos = {s: i for i, s in enumerate(dom)}
            lut = torch.tensor([pos.get(s, -1) for s in (av.domain or [])] + [-1], dtype=torch.long,
                               device=av.data.device)
            c = av.data.long()
            y = lut[torch.where(c >= 0, c, torch.full_like(c, lut.numel() - 1))]
        else:
            y = av.as_float().long()
        ok = y >= 0
        if len(dom) == 2:
            p1 = predicted.vecs[-1].as_float()
            m = binomial_metrics(p1[ok], y[ok].float(), None if w is None else w[ok], comm)
            m["model_category"] = ModelCategory.BINOMIAL
            return m
        cols = [predicted.vec(d) if d in predicted.names else predicted.vecs[-len(dom) + k]
                for k, d in enumerate(dom)]
        P = torch.stack([c.as_float() for c in cols])
        m = multinomial_metrics(P[:, ok], y[ok], None if w is None else w[ok], comm)
        m["model_category"] = ModelCategory.MULTINOMIAL
        return m
    pr = predicted.vecs[0].as_float()
    y = av.as_float()
    ok = ~torch.isnan(y) & ~torch.isnan(pr)
    dist = str(distribution or "gaussian").lower()
    m = regression_metrics(pr[ok], y[ok], None if w is None else w[ok], comm,
                           dist if dist in ("poisson", "gamma", "laplace") else "gaussian")
    m["model_category"] = ModelCategory.REGRESSION
    return m


_HIGHER_BETTER = ("AUC", "AUCPR")


def _metric_key(model, metric):
    m = str(metric or "AUTO").upper()
    if m == "AUTO":
        return {ModelCategory.BINOMIAL: "logloss", ModelCategory.MULTINOMIAL: "logloss"}.get(model.category, "RMSE")
    return {"LOGLOSS": "logloss", "MAE": "mae", "RMSLE": "rmsle", "MEAN_PER_CLASS_ERROR": "mean_per_class_error"}.get(
        m, m)


def permutation_importance(model, frame: Frame, metric="AUTO", n_repeats: int = 1, seed: int = -1,
                           features=None) -> list[dict]:
    """Rows {variable, relative_importance, scaled_importance, percentage}
    sorted by importance (mean over ``n_repeats`` shuffles)."""
    key = _metric_key(model, metric)
    comm = getattr(model, "comm", None)
    base = model._metrics(frame, model.predict_raw(frame), comm).get(key)
    if base is None:
        raise ValueError(f"permutation_importance: metric {metric!r} is not reported for this model")
    g = torch.Generator().manual_seed(int(seed) if seed is not None and seed >= 0 else 42)
    feats = list(features or model.x)
    imp = {}
    for f in feats:
        deltas = []
        for _ in range(max(1, int(n_repeats))):
            perm = torch.randperm(frame.nrows, generator=g).to(frame.device)
            v = frame.vec(f)
            nv = Vec(v.name, v.data[perm], v.vtype, v.domain)
            fr = Frame([nv if u.name == f else u for u in frame.vecs])
            val = model._metrics(fr, model.predict_raw(fr), comm).get(key)
            d = (base - val) if key in _HIGHER_BETTER else (val - base)
            deltas.append(float(d))
        imp[f] = float(np.mean(deltas))
    mx = max((abs(v) for v in imp.values()), default=0.0)
    tot = sum(max(v, 0.0) for v in imp.values())
    rows = [{"variable": f, "relative_importance": v, "scaled_importance": v / mx if mx > 0 else 0.0,
             "percentage": max(v, 0.0) / tot if tot > 0 else 0.0} for f, v in imp.items()]
    rows.sort(key=lambda r: -r["relative_importance"])
    return rows


def train_segments(estimator_cls, params: dict, segment_columns, x=None, y=None, training_frame: Frame = None,
                   validation_frame: Frame | None = None, segment_models_id: str | None = None, comm=None) -> dict:
    """One model per segment (levels of the categorical ``segment_columns``).
    With a communicator, every rank holds a shard of each segment and the
    models train data-parallel, one segment after another."""
    segs = [segment_columns] if isinstance(segment_columns, str) else list(segment_columns)
    for s in segs:
        if training_frame.vec(s).vtype != ENUM:
            raise ValueError(f"train_segments: segment column {s!r} must be categorical")
    doms = [list(training_frame.vec(s).domain or []) for s in segs]
    sid = segment_models_id or f"segment_models_{id(training_frame) & 0xFFFFFF:x}"
    rows = []
    base_x = [c for c in (x or training_frame.names) if c not in segs and c != y]
    for combo in itertools.product(*[range(len(d)) for d in doms]):
        mask = torch.ones(training_frame.nrows, dtype=torch.bool, device=training_frame.device)
        for s, k in zip(segs, combo):
            mask &= training_frame.vec(s).data.long() == k
        n_local = int(mask.sum())
        n = n_local
        if comm is not None and comm.world_size > 1:
            n = int(comm.all_reduce_numpy(np.array([float(n_local)]))[0])
        levels = {s: d[k] for s, d, k in zip(segs, doms, combo)}
        row = dict(levels)
        if n == 0:
            continue
        mid = f"{sid}_" + "_".join(str(v) for v in levels.values())
        try:
            sub = training_frame.rows(torch.nonzero(mask).flatten())
            vsub = None
            if validation_frame is not None:
                vm = torch.ones(validation_frame.nrows, dtype=torch.bool, device=validation_frame.device)
                for s, lv in levels.items():
                    vd = list(validation_frame.vec(s).domain or [])
                    vm &= validation_frame.vec(s).data.long() == (vd.index(lv) if lv in vd else -2)
                vsub = validation_frame.rows(torch.nonzero(vm).flatten())
            m = estimator_cls(**dict(params, model_id=mid)).train(x=base_x, y=y, training_frame=sub,
                                                                   validation_frame=vsub, comm=comm)
            row.update(model=m.model_id, status="SUCCEEDED", errors=None, rows=n)
        except Exception as e:  # noqa: BLE001  (H2O reports per-segment failures in the table)
            row.update(model=None, status="FAILED", errors=f"{type(e).__name__}: {e}", rows=n)
        rows.append(row)
    out = {"segment_models_id": sid, "segment_columns": segs, "segments": rows}
    DKV.put(sid, out)
    return out
