"""Target Encoding (H2O ``H2OTargetEncoderEstimator`` equivalent).

Replaces each categorical column by the (blended) mean of the response
over the rows sharing its level.  Statistics are per-level sums built with
one ``scatter_add`` per column on the rank's shard and combined across ranks
with a single all-reduce per column (the MRTask reduce of H2O's
``TargetEncoderModel``).

Encoding of level ``l`` with ``n_l`` rows and response sum ``s_l`` (prior
``p = sum y / n``):

* ``blending=False``: ``s_l / n_l`` (unseen / NA level -> prior);
* ``blending=True``:  ``lambda * s_l / n_l + (1 - lambda) * p`` with
  ``lambda = 1 / (1 + exp((inflection_point - n_l) / smoothing))``.

``data_leakage_handling`` for the training frame (``transform(...,
as_training=True)``): ``None`` uses all rows, ``LeaveOneOut`` removes the
row's own response from its level's sums, ``KFold`` uses the sums of the
other folds (``fold_column``).  ``noise`` adds uniform(-noise, noise) to
training encodings (seeded).  Binomial responses encode P(y = second
level); multinomial responses get one column per class except the first
(``<col>_<class>_te``); regression encodes the mean.
"""
from __future__ import annotations

import math

import torch

from ..frame.frame import ENUM, REAL, Frame, Vec
from .base import Model, ModelBuilder, ModelCategory


class TargetEncoderModel(Model):
    algo = "targetencoder"
    algo_full_name = "TargetEncoder"

    def __init__(self, builder, model_id, stats, prior, classes, columns):
        super().__init__(builder, model_id)
        self.stats = stats          # col -> (sums [L+1][C] float64, counts [L+1] float64, per-fold or None)
        self.prior = prior          # [C] float64
        self.classes = classes      # output class labels (None for regression / binomial)
        self.columns = columns

    def _encode(self, num, den, prior):
        p_ = self.params
        with torch.no_grad():
            mean = torch.where(den[:, None] > 0, num / den.clamp_min(1e-300)[:, None], prior[None, :])
            if p_["blending"]:
                k, f = float(p_["inflection_point"]), max(float(p_["smoothing"]), 1e-12)
                lam = 1.0 / (1.0 + torch.exp((k - den) / f))
                mean = lam[:, None] * mean + (1.0 - lam[:, None]) * prior[None, :]
        return mean

    def transform(self, frame: Frame, as_training: bool = False, noise: float | None = None,
                  blending: bool | None = None, inflection_point=None, smoothing=None) -> Frame:
        """Encoded frame: the original columns (categoricals kept unless
        ``keep_original_categorical_columns`` is false) plus ``<col>_te``."""
        p_ = dict(self.params)
        for k, v in (("blending", blending), ("inflection_point", inflection_point), ("smoothing", smoothing)):
            if v is not None:
                self.params[k] = v
        try:
            return self._transform(frame, as_training, noise)
        finally:
            self.params.update({k: p_[k] for k in ("blending", "inflection_point", "smoothing")})

    def _transform(self, frame, as_training, noise):
        p_ = self.params
        frame = self.adapt_frame(frame)
        dev = frame.device
        leak = str(p_["data_leakage_handling"] or "None").lower() if as_training else "none"
        if noise is None:
            noise = float(p_["noise"]) if as_training else 0.0
        out = [v for v in frame.vecs if p_["keep_original_categorical_columns"] or v.name not in self.columns]
        y = None
        if leak in ("leaveoneout", "leave_one_out"):
            y = _response_matrix(frame.vec(self.y), self.category, len(self.prior)).to(dev)
        g = torch.Generator(device="cpu").manual_seed(int(p_["seed"]) if p_["seed"] not in (None, -1) else 1234)
        prior = self.prior.to(dev)
        for c in self.columns:
            sums, cnts, folds = self.stats[c]
            sums, cnts = sums.to(dev), cnts.to(dev)
            codes = frame.vec(c).data.long()
            L = cnts.numel() - 1
            idx = torch.where((codes >= 0) & (codes < L), codes, torch.full_like(codes, L))   # NA / unseen -> L
            if leak in ("kfold", "k_fold") and folds is not None:
                fcol = p_["fold_column"]
                fid = frame.vec(fcol).as_float().long().to(dev)
                fs, fc, fold_values = folds
                fpos = torch.searchsorted(fold_values.to(dev), fid).clamp_max(fold_values.numel() - 1)
                num = sums[idx] - fs.to(dev)[fpos, idx]
                den = cnts[idx] - fc.to(dev)[fpos, idx]
                enc = self._encode(num, den, prior)
            elif y is not None:
                num = sums[idx] - y
                den = cnts[idx] - 1.0
                enc = self._encode(num, den, prior)
            else:
                enc = self._encode(sums, cnts, prior)[idx]
            # NA / unseen levels use the prior whatever the level statistics say
            enc = torch.where((idx == L)[:, None], prior[None, :].expand_as(enc), enc)
            if noise > 0:
                enc = enc + (torch.rand(enc.shape, generator=g) * 2 - 1).to(dev, enc.dtype) * noise
            names = _out_names(c, self.classes)
            for j, nm in enumerate(names):
                out.append(Vec(nm, enc[:, j].float(), REAL))
        return Frame(out)

    def predict(self, frame: Frame) -> Frame:
        return self.transform(frame)

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        fr = self.transform(frame)
        cols = [n for c in self.columns for n in _out_names(c, self.classes)]
        return torch.stack([fr.vec(n).data for n in cols]) if cols else torch.zeros((0, frame.nrows))

    def model_performance(self, frame=None):
        return self.training_metrics

    def summary(self):
        return {"model_id": self.model_id, "encoded_columns": self.columns,
                "prior": [float(v) for v in self.prior]}

    def to_json(self):
        j = super().to_json()
        j["output"]["model_category"] = "TargetEncoder"
        j["output"]["te_column_name_to_missing_values_presence"] = [
            {"column": c, "missing": bool(self.stats[c][1][-1] > 0)} for c in self.columns]
        return j


def _out_names(col, classes):
    if classes is None:
        return [f"{col}_te"]
    return [f"{col}_{k}_te" for k in classes]


def _response_matrix(yv: Vec, category, C) -> torch.Tensor:
    """[n][C] float64 targets: binomial P(y=1), multinomial one-hot of classes 1..K-1, regression y."""
    if category == ModelCategory.REGRESSION:
        return yv.as_float().double()[:, None]
    codes = yv.data.long()
    if category == ModelCategory.BINOMIAL:
        return (codes == 1).double()[:, None]
    cls = torch.arange(1, C + 1, device=codes.device)
    return (codes[:, None] == cls[None, :]).double()


class H2OTargetEncoderEstimator(ModelBuilder):
    algo = "targetencoder"
    DEFAULTS = dict(columns_to_encode=None, keep_original_categorical_columns=True, blending=False,
                    inflection_point=10.0, smoothing=20.0, data_leakage_handling="None", noise=0.01)

    def _resolve_columns(self, frame, x, y):
        x, y = super()._resolve_columns(frame, x, y)
        cte = self.params.get("columns_to_encode")
        if cte:
            flat = [c if isinstance(c, str) else c[0] for c in cte]
            x = [c for c in flat if c in frame.names]
        return [c for c in x if frame.vec(c).vtype == ENUM], y

    def _fit(self, train: Frame, valid, model_id):
        if self.y is None:
            raise ValueError("targetencoder needs a response column")
        p_ = self.params
        comm = self.comm
        dev = train.device
        yv = train.vec(self.y)
        if self.category == ModelCategory.MULTINOMIAL:
            classes = list(self.response_domain[1:])
        else:
            classes = None
        C = 1 if classes is None else len(classes)
        Y = _response_matrix(yv, self.category, C).to(dev)
        ok = ~torch.isnan(Y).any(1)
        if self.category != ModelCategory.REGRESSION:
            ok &= yv.data >= 0
        Y = torch.where(ok[:, None], Y, torch.zeros_like(Y))
        w = ok.double()
        tot = torch.cat([(Y * w[:, None]).sum(0), w.sum()[None]])
        if comm is not None and comm.world_size > 1:
            comm.all_reduce_(tot)
        prior = (tot[:C] / tot[C].clamp_min(1.0)).cpu()
        kfold = str(p_["data_leakage_handling"] or "None").lower() in ("kfold", "k_fold")
        if kfold and not p_.get("fold_column"):
            raise ValueError("targetencoder: data_leakage_handling='KFold' needs fold_column")
        fold_values = None
        if kfold:
            fid = train.vec(p_["fold_column"]).as_float().long()
            fv = torch.unique(fid)
            if comm is not None and comm.world_size > 1:
                fv = torch.unique(comm.all_gather_cat(fv))
            fold_values = fv.sort().values
        stats = {}
        for c in self.x:
            dom = self.feature_domains.get(c) or []
            L = len(dom)
            codes = train.vec(c).data.long()
            idx = torch.where(codes >= 0, codes, torch.full_like(codes, L))
            sums = torch.zeros((L + 1, C), dtype=torch.float64, device=dev)
            cnts = torch.zeros((L + 1,), dtype=torch.float64, device=dev)
            sums.index_add_(0, idx, Y * w[:, None])
            cnts.index_add_(0, idx, w)
            folds = None
            if kfold:
                F = fold_values.numel()
                fpos = torch.searchsorted(fold_values.to(dev), fid.to(dev))
                flat = fpos * (L + 1) + idx
                fs = torch.zeros((F * (L + 1), C), dtype=torch.float64, device=dev).index_add_(0, flat, Y * w[:, None])
                fc = torch.zeros((F * (L + 1),), dtype=torch.float64, device=dev).index_add_(0, flat, w)
                if comm is not None and comm.world_size > 1:
                    comm.all_reduce_(fs)
                    comm.all_reduce_(fc)
                folds = (fs.view(F, L + 1, C).cpu(), fc.view(F, L + 1).cpu(), fold_values.cpu())
            if comm is not None and comm.world_size > 1:
                comm.all_reduce_(sums)
                comm.all_reduce_(cnts)
            stats[c] = (sums.cpu(), cnts.cpu(), folds)
        model = TargetEncoderModel(self, model_id, stats, prior, classes, list(self.x))
        model.training_metrics = {"nobs": float(tot[C]), "prior": [float(v) for v in prior]}
        if not math.isfinite(float(p_["inflection_point"])) or float(p_["smoothing"]) <= 0:
            raise ValueError("targetencoder: inflection_point must be finite and smoothing > 0")
        return model
