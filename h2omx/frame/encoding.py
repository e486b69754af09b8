"""H2O ``categorical_encoding`` schemes applied before an algorithm sees the
predictors (hex/Model.java CategoricalEncodingScheme).

Schemes that an algorithm implements natively stay with the algorithm:

* ``AUTO`` / ``Enum``: GBM / DRF group splits on the level codes
  (models/tree_models.py); GLM / DeepLearning / K-Means expand the levels
  internally (``OneHotInternal``); XGBoost's AUTO is one-hot, as in H2O.
* ``SortByResponse`` in the tree builders (levels reordered by mean
  response); other algorithms get the same reordering as a transform.

The others are frame transformations fitted on the training frame and stored
on the model, so scoring frames are encoded identically
(:meth:`CategoricalEncoder.transform`, called from ``Model.adapt_frame``):

* ``OneHotExplicit``: one 0/1 column ``c.level`` per level plus
  ``c.missing(NA)``;
* ``Binary``: the level index + 1 (0 = NA) written in ``ceil(log2(L + 1))``
  0/1 columns ``c:0`` (least significant bit) ...;
* ``Eigen``: one column ``c.Eigen``: each level's entry of the top
  eigenvector of the column's centred one-hot covariance (k = 1);
* ``LabelEncoder``: the level index as a numeric column (ordinal splits);
* ``EnumLimited``: the ``max_categorical_levels`` (default 10) most frequent
  levels kept, every other level merged into ``other``; the column stays
  categorical and the algorithm's native handling applies.

Unknown scheme names raise.  Levels unseen at training time encode like NA.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .frame import ENUM, REAL, Frame, Vec

SCHEMES = {"auto": "auto", "enum": "enum", "onehotinternal": "onehotinternal", "onehotexplicit": "onehotexplicit",
           "binary": "binary", "eigen": "eigen", "labelencoder": "labelencoder", "sortbyresponse": "sortbyresponse",
           "enumlimited": "enumlimited"}
TRANSFORMS = ("onehotexplicit", "binary", "eigen", "labelencoder", "enumlimited", "sortbyresponse")


def normalize_scheme(name) -> str:
    key = str(name or "AUTO").replace("_", "").lower()
    if key not in SCHEMES:
        raise ValueError(f"unknown categorical_encoding {name!r} (one of AUTO, Enum, OneHotInternal, OneHotExplicit, "
                         "Binary, Eigen, LabelEncoder, SortByResponse, EnumLimited)")
    return SCHEMES[key]


class CategoricalEncoder:
    """Fitted per-column encodings; ``x_out`` is the predictor list the
    algorithm trains on."""

    def __init__(self, scheme: str, x: list, types: dict, domains: dict, max_levels: int = 10, y: str | None = None):
        self.scheme = scheme
        self.y = y
        self.x_in = list(x)
        self.types, self.domains = dict(types), {c: list(d or []) for c, d in domains.items()}
        self.max_levels = int(max_levels)
        self.spec: dict = {}          # column -> scheme data
        self.x_out: list = []
        self.out_types: dict = {}
        self.out_domains: dict = {}

    # -- fitting -------------------------------------------------------------
    def fit(self, frame: Frame, comm=None) -> "CategoricalEncoder":
        for c in self.x_in:
            if self.types.get(c) != ENUM:
                self.x_out.append(c)
                self.out_types[c] = self.types.get(c)
                self.out_domains[c] = self.domains.get(c)
                continue
            dom = self.domains.get(c) or []
            L = len(dom)
            if self.scheme == "onehotexplicit":
                names = [f"{c}.{lv}" for lv in dom] + [f"{c}.missing(NA)"]
                self.spec[c] = {"names": names}
                self._numeric(names)
            elif self.scheme == "binary":
                nb = max(1, math.ceil(math.log2(L + 1)))
                names = [f"{c}:{k}" for k in range(nb)]
                self.spec[c] = {"names": names, "bits": nb}
                self._numeric(names)
            elif self.scheme == "labelencoder":
                self.spec[c] = {"names": [c]}
                self._numeric([c])
            elif self.scheme == "eigen":
                counts = self._counts(frame, c, L, comm)
                p = counts / max(counts.sum(), 1.0)
                cov = np.diag(p) - np.outer(p, p)
                w, v = np.linalg.eigh(cov) if L else (np.zeros(0), np.zeros((0, 0)))
                vec = v[:, int(np.argmax(w))] if L else np.zeros(0)
                if L and vec[int(np.argmax(np.abs(vec)))] < 0:
                    vec = -vec            # deterministic sign
                self.spec[c] = {"names": [f"{c}.Eigen"], "values": vec.astype(np.float64)}
                self._numeric([f"{c}.Eigen"])
            elif self.scheme == "sortbyresponse":
                # levels reordered by mean response (NaN-free rows), unseen-in-training last
                yv = frame.vec(self.y) if self.y is not None else None
                if yv is None:
                    raise ValueError("categorical_encoding SortByResponse needs a response column")
                yval = yv.as_float().double()
                codes = self.codes_in_training_domain(frame, c)
                ok = (codes >= 0) & ~torch.isnan(yval)
                sums = torch.bincount(codes[ok], weights=yval[ok], minlength=L)[:L].cpu().numpy()
                cnt = torch.bincount(codes[ok], minlength=L)[:L].double().cpu().numpy()
                if comm is not None and comm.world_size > 1:
                    sums, cnt = comm.all_reduce_numpy(sums), comm.all_reduce_numpy(cnt)
                order = sorted(range(L), key=lambda i: (sums[i] / cnt[i] if cnt[i] > 0 else float("inf"), i))
                lut = np.empty(L, np.int64)
                lut[order] = np.arange(L)
                self.spec[c] = {"names": [c], "lut": lut, "domain": [dom[i] for i in order]}
                self.x_out.append(c)
                self.out_types[c] = ENUM
                self.out_domains[c] = [dom[i] for i in order]
            elif self.scheme == "enumlimited":
                counts = self._counts(frame, c, L, comm)
                keep = sorted(np.argsort(-counts, kind="stable")[: self.max_levels].tolist())
                new_dom = [dom[i] for i in keep]
                if L > len(keep):
                    new_dom.append("other")
                lut = np.full(L, len(new_dom) - 1 if L > len(keep) else -1, np.int64)
                for j, i in enumerate(keep):
                    lut[i] = j
                self.spec[c] = {"names": [c], "lut": lut, "domain": new_dom}
                self.x_out.append(c)
                self.out_types[c] = ENUM
                self.out_domains[c] = new_dom
            else:
                raise ValueError(f"categorical_encoding {self.scheme!r} is not a frame transform")
        return self

    def _numeric(self, names):
        for n in names:
            self.x_out.append(n)
            self.out_types[n] = REAL
            self.out_domains[n] = None

    def _counts(self, frame: Frame, c: str, L: int, comm) -> np.ndarray:
        codes = self.codes_in_training_domain(frame, c)
        cnt = torch.bincount(codes[codes >= 0], minlength=L)[:L].double().cpu().numpy()
        if comm is not None and comm.world_size > 1:
            cnt = comm.all_reduce_numpy(cnt)
        return cnt

    # -- applying --------------------------------------------------------------
    def codes_in_training_domain(self, frame: Frame, c: str) -> torch.Tensor:
        """Level codes of ``c`` mapped onto the training domain (-1 = NA / unseen)."""
        v = frame.vec(c)
        dom = self.domains.get(c) or []
        if v.vtype != ENUM:
            raise ValueError(f"column {c!r} must be categorical")
        if list(v.domain or []) == dom:
            return v.data.long()
        idx = {d: i for i, d in enumerate(dom)}
        lut = torch.tensor([idx.get(d, -1) for d in (v.domain or [])] + [-1], dtype=torch.long, device=v.data.device)
        codes = v.data.long()
        return lut[torch.where(codes >= 0, codes, torch.full_like(codes, lut.numel() - 1))]

    def transform(self, frame: Frame) -> Frame:
        if getattr(frame, "_encoded_by", None) is self:
            return frame
        new = {}
        for c, sp in self.spec.items():
            if c not in frame.names:
                continue
            codes = self.codes_in_training_domain(frame, c)
            dev = codes.device
            L = len(self.domains.get(c) or [])
            if self.scheme == "onehotexplicit":
                cols = []
                for j in range(L):
                    cols.append((codes == j).float())
                cols.append((codes < 0).float())
                new[c] = [Vec(nm, t, REAL) for nm, t in zip(sp["names"], cols)]
            elif self.scheme == "binary":
                val = torch.where(codes >= 0, codes + 1, torch.zeros_like(codes))
                new[c] = [Vec(nm, ((val >> k) & 1).float(), REAL) for k, nm in enumerate(sp["names"])]
            elif self.scheme == "labelencoder":
                f = codes.float()
                new[c] = [Vec(c, torch.where(codes >= 0, f, torch.full_like(f, float("nan"))), REAL)]
            elif self.scheme == "eigen":
                vals = torch.from_numpy(np.append(sp["values"], np.nan).astype(np.float32)).to(dev)
                new[c] = [Vec(sp["names"][0], vals[torch.where(codes >= 0, codes, torch.full_like(codes, L))],
                              REAL)]
            elif self.scheme in ("enumlimited", "sortbyresponse"):
                lut = torch.from_numpy(np.append(sp["lut"], -1)).to(dev)
                mapped = lut[torch.where(codes >= 0, codes, torch.full_like(codes, L))].to(torch.int32)
                new[c] = [Vec(c, mapped, ENUM, list(sp["domain"]))]
        vecs = []
        for v in frame.vecs:
            vecs.extend(new.get(v.name, [v]))
        out = Frame(vecs, key=frame.key)
        out._encoded_by = self
        return out

    # -- persistence (MOJO payload) -----------------------------------------
    def to_json(self) -> dict:
        spec = {}
        for c, sp in self.spec.items():
            d = dict(sp)
            for k in ("lut", "values"):
                if k in d:
                    d[k] = np.asarray(d[k]).tolist()
            spec[c] = d
        return {"scheme": self.scheme, "x_in": self.x_in, "types": self.types, "domains": self.domains,
                "max_levels": self.max_levels, "y": self.y, "spec": spec, "x_out": self.x_out,
                "out_types": self.out_types, "out_domains": self.out_domains}

    @classmethod
    def from_json(cls, j: dict) -> "CategoricalEncoder":
        ce = cls(j["scheme"], j["x_in"], j["types"], j["domains"], j.get("max_levels", 10), j.get("y"))
        for c, d in j["spec"].items():
            d = dict(d)
            if "lut" in d:
                d["lut"] = np.asarray(d["lut"], np.int64)
            if "values" in d:
                d["values"] = np.asarray(d["values"], np.float64)
            ce.spec[c] = d
        ce.x_out, ce.out_types, ce.out_domains = list(j["x_out"]), dict(j["out_types"]), dict(j["out_domains"])
        return ce
