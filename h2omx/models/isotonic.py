"""Isotonic Regression (H2O ``H2OIsotonicRegressionEstimator``).

Fits the monotone non-decreasing step function of one predictor that
minimises the weighted squared error (pool-adjacent-violators).  Each rank
first collapses its shard to (unique x, Σw·y, Σw) — a sort + segment sum
on the device — the per-rank summaries are all-gathered (the H2O MRTask
reduce), merged and pooled on the host.  Prediction interpolates linearly
between the fitted thresholds; outside them ``out_of_bounds="clip"`` uses
the end values and ``"NA"`` returns NaN.
"""
from __future__ import annotations

import numpy as np
import torch

from ..frame.frame import Frame
from .base import Model, ModelBuilder, ModelCategory


def pav(x: np.ndarray, y: np.ndarray, w: np.ndarray):
    """Pool adjacent violators over x-sorted unique points -> (thresholds, values)."""
    blocks_y, blocks_w, blocks_lo, blocks_hi = [], [], [], []
    for xi, yi, wi in zip(x, y, w):
        blocks_y.append(yi)
        blocks_w.append(wi)
        blocks_lo.append(xi)
        blocks_hi.append(xi)
        while len(blocks_y) > 1 and blocks_y[-2] > blocks_y[-1]:
            w2 = blocks_w[-2] + blocks_w[-1]
            y2 = (blocks_y[-2] * blocks_w[-2] + blocks_y[-1] * blocks_w[-1]) / w2
            lo = blocks_lo[-2]
            hi = blocks_hi[-1]
            for lst in (blocks_y, blocks_w, blocks_lo, blocks_hi):
                lst.pop()
            blocks_y[-1], blocks_w[-1], blocks_lo[-1], blocks_hi[-1] = y2, w2, lo, hi
    thr, val = [], []
    for yb, lo, hi in zip(blocks_y, blocks_lo, blocks_hi):
        thr.append(lo)
        val.append(yb)
        if hi != lo:
            thr.append(hi)
            val.append(yb)
    return np.asarray(thr, np.float64), np.asarray(val, np.float64)


class IsotonicRegressionModel(Model):
    algo = "isotonicregression"
    algo_full_name = "Isotonic Regression"

    def __init__(self, builder, model_id, thresholds, values):
        super().__init__(builder, model_id)
        self.thresholds_x = thresholds
        self.thresholds_y = values

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        x = frame.vec(self.x[0]).as_float()
        dev = x.device
        tx = torch.from_numpy(self.thresholds_x).to(dev)
        ty = torch.from_numpy(self.thresholds_y).to(dev)
        xd = x.double()
        i = torch.searchsorted(tx, xd).clamp(1, max(tx.numel() - 1, 1))
        if tx.numel() == 1:
            out = ty[0].expand_as(xd).clone()
        else:
            x0, x1 = tx[i - 1], tx[i]
            y0, y1 = ty[i - 1], ty[i]
            t = torch.where(x1 > x0, (xd - x0) / (x1 - x0).clamp_min(1e-300), torch.zeros_like(xd))
            out = y0 + t.clamp(0, 1) * (y1 - y0)
        lo, hi = tx[0], tx[-1]
        if str(self.params["out_of_bounds"]).lower() == "clip":
            out = torch.where(xd < lo, ty[0], torch.where(xd > hi, ty[-1], out))
        else:
            out = torch.where((xd < lo) | (xd > hi), torch.full_like(out, float("nan")), out)
        out = torch.where(torch.isnan(xd), torch.full_like(out, float("nan")), out)
        return out.float()[None, :]

    def summary(self):
        return {"model_id": self.model_id, "number_of_thresholds": int(self.thresholds_x.size)}

    def to_json(self):
        j = super().to_json()
        j["output"]["thresholds_x"] = self.thresholds_x.tolist()
        j["output"]["thresholds_y"] = self.thresholds_y.tolist()
        return j


class H2OIsotonicRegressionEstimator(ModelBuilder):
    algo = "isotonicregression"
    DEFAULTS = dict(out_of_bounds="NA", custom_metric_func=None)

    def _fit(self, train: Frame, valid, model_id):
        if len(self.x) != 1:
            raise ValueError("isotonicregression takes exactly one predictor column")
        if self.category != ModelCategory.REGRESSION:
            raise ValueError("isotonicregression needs a numeric response")
        x = train.vec(self.x[0]).as_float().double()
        y = train.vec(self.y).as_float().double()
        w = (train.vec(self.params["weights_column"]).as_float().double() if self.params.get("weights_column")
             else torch.ones_like(x))
        ok = ~torch.isnan(x) & ~torch.isnan(y) & (w > 0)
        x, y, w = x[ok], y[ok], w[ok]
        ux, inv = torch.unique(x, sorted=True, return_inverse=True)
        sw = torch.zeros_like(ux).index_add_(0, inv, w)
        swy = torch.zeros_like(ux).index_add_(0, inv, w * y)
        S = torch.stack([ux, swy, sw], 1)
        comm = self.comm
        if comm is not None and comm.world_size > 1:
            S = comm.all_gather_cat(S)
        S = S.cpu().numpy()
        if S.shape[0] == 0:
            raise ValueError("isotonicregression: no complete rows")
        ux, inv = np.unique(S[:, 0], return_inverse=True)
        swy = np.bincount(inv, weights=S[:, 1])
        sw = np.bincount(inv, weights=S[:, 2])
        thr, val = pav(ux, swy / sw, sw)
        return IsotonicRegressionModel(self, model_id, thr, val)
