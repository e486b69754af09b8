"""Columnar frames (H2O Frame / Vec equivalents) and the distributed key store.

A :class:`Frame` is an ordered set of :class:`Vec` columns of equal length,
resident on one device (the rank's GPU, or CPU).  In a multi-rank cluster
each rank holds a contiguous row shard of every frame under the same key
(H2O's row-chunked distribution; SURVEY.md §2.3 "Data parallel").
Categorical columns store int32 level codes (-1 = NA) against a sorted
domain, exactly like H2O enum Vecs; numeric columns store float32 (NaN = NA).
"""
from __future__ import annotations

import itertools
import threading
import uuid
from dataclasses import dataclass, field

import numpy as np
import torch

REAL, INT, ENUM, STRING, TIME = "real", "int", "enum", "string", "time"


@dataclass
class Vec:
    name: str
    data: torch.Tensor             # float32 (numeric) or int32 codes (enum)
    vtype: str = REAL
    domain: list | None = None

    @property
    def nrows(self) -> int:
        return int(self.data.shape[0])

    @property
    def is_categorical(self) -> bool:
        return self.vtype == ENUM

    def as_float(self) -> torch.Tensor:
        if self.vtype == ENUM:
            f = self.data.float()
            return torch.where(self.data < 0, torch.full_like(f, float("nan")), f)
        return self.data.float()

    def summary(self) -> dict:
        x = self.as_float()
        na = torch.isnan(x)
        v = x[~na]
        out = {"label": self.name, "type": self.vtype, "missing_count": int(na.sum()), "domain": self.domain}
        if v.numel():
            out.update(mins=[float(v.min())], maxs=[float(v.max())], mean=float(v.double().mean()),
                       sigma=float(v.double().std()) if v.numel() > 1 else 0.0,
                       zero_count=int((v == 0).sum()))
        else:
            out.update(mins=[float("nan")], maxs=[float("nan")], mean=float("nan"), sigma=float("nan"), zero_count=0)
        return out


class Frame:
    _counter = itertools.count()

    def __init__(self, vecs: list[Vec], key: str | None = None):
        if vecs:
            n = vecs[0].nrows
            for v in vecs:
                if v.nrows != n:
                    raise ValueError(f"column {v.name} has {v.nrows} rows, expected {n}")
        self.vecs = list(vecs)
        self.key = key or f"frame_{next(self._counter)}_{uuid.uuid4().hex[:8]}"

    # -- construction ----------------------------------------------------------
    @classmethod
    def from_numpy(cls, data, names=None, device="cpu", categorical=(), key=None) -> "Frame":
        """``data``: dict name -> 1-D array, or a 2-D array [n][p] (row-major)."""
        if isinstance(data, dict):
            items = list(data.items())
        else:
            arr = np.asarray(data)
            if arr.ndim == 1:
                arr = arr[:, None]
            names = names or [f"C{i + 1}" for i in range(arr.shape[1])]
            items = [(n, arr[:, i]) for i, n in enumerate(names)]
        vecs = []
        for name, col in items:
            col = np.asarray(col)
            if col.dtype.kind in "OUS" or name in categorical:
                vecs.append(_enum_vec(name, col, device))
            else:
                vt = INT if col.dtype.kind in "iub" else REAL
                vecs.append(Vec(name, torch.as_tensor(col.astype(np.float32), device=device), vt))
        return cls(vecs, key=key)

    @classmethod
    def from_pandas(cls, df, device="cpu", key=None) -> "Frame":
        data = {}
        cats = []
        for c in df.columns:
            s = df[c]
            if str(s.dtype) in ("object", "category", "bool", "string"):
                data[c] = s.astype(str).where(~s.isna(), None).to_numpy(dtype=object)
                cats.append(c)
            else:
                data[c] = s.to_numpy()
        return cls.from_numpy(data, device=device, categorical=cats, key=key)

    @classmethod
    def from_tensor(cls, X: torch.Tensor, names=None, y: torch.Tensor | None = None, y_name="response",
                    y_categorical=False, key=None) -> "Frame":
        """Feature-major tensor [F][n] (+ optional response) -> Frame (no copy)."""
        F = X.shape[0]
        names = names or [f"C{i + 1}" for i in range(F)]
        vecs = [Vec(n, X[i], REAL) for i, n in enumerate(names)]
        if y is not None:
            if y_categorical:
                codes = y.to(torch.int32)
                k = int(codes.max().item()) + 1 if codes.numel() else 0
                vecs.append(Vec(y_name, codes, ENUM, [str(i) for i in range(k)]))
            else:
                vecs.append(Vec(y_name, y.float(), REAL))
        return cls(vecs, key=key)

    # -- properties --------------------------------------------------------------
    @property
    def names(self) -> list[str]:
        return [v.name for v in self.vecs]

    @property
    def columns(self) -> list[str]:
        return self.names

    @property
    def nrows(self) -> int:
        return self.vecs[0].nrows if self.vecs else 0

    @property
    def ncols(self) -> int:
        return len(self.vecs)

    @property
    def shape(self):
        return (self.nrows, self.ncols)

    @property
    def device(self):
        return self.vecs[0].data.device if self.vecs else torch.device("cpu")

    @property
    def types(self) -> dict:
        return {v.name: v.vtype for v in self.vecs}

    def vec(self, name: str) -> Vec:
        for v in self.vecs:
            if v.name == name:
                return v
        raise KeyError(f"column '{name}' not in frame {self.key}")

    def __getitem__(self, item):
        if isinstance(item, str):
            return Frame([self.vec(item)])
        if isinstance(item, int):
            return Frame([self.vecs[item]])
        if isinstance(item, (list, tuple)):
            return Frame([self.vec(c) if isinstance(c, str) else self.vecs[c] for c in item])
        if isinstance(item, slice):
            return self.rows(torch.arange(self.nrows)[item])
        if torch.is_tensor(item):
            return self.rows(item)
        raise TypeError(item)

    def rows(self, idx: torch.Tensor) -> "Frame":
        idx = idx.to(self.device)
        if idx.dtype == torch.bool:
            idx = torch.nonzero(idx).flatten()
        return Frame([Vec(v.name, v.data.index_select(0, idx), v.vtype, v.domain) for v in self.vecs])

    def to(self, device) -> "Frame":
        return Frame([Vec(v.name, v.data.to(device), v.vtype, v.domain) for v in self.vecs], key=self.key)

    def cbind(self, other: "Frame") -> "Frame":
        return Frame(self.vecs + other.vecs)

    def drop(self, cols) -> "Frame":
        cols = {cols} if isinstance(cols, str) else set(cols)
        return Frame([v for v in self.vecs if v.name not in cols])

    def asfactor(self, col: str) -> "Frame":
        v = self.vec(col)
        if v.vtype == ENUM:
            return self
        x = v.data.cpu().numpy()
        vals = np.where(np.isnan(x), np.nan, x)
        nv = _enum_vec(v.name, np.array([None if np.isnan(a) else _num_label(a) for a in vals], dtype=object),
                       v.data.device)
        return Frame([nv if u.name == col else u for u in self.vecs], key=self.key)

    def split_frame(self, ratios=(0.75,), seed: int = 1234) -> list["Frame"]:
        g = torch.Generator().manual_seed(seed)
        u = torch.rand(self.nrows, generator=g)
        edges = np.cumsum([0.0] + list(ratios) + [1.0 - sum(ratios)])
        out = []
        for lo, hi in zip(edges[:-1], edges[1:]):
            m = (u >= lo) & (u < hi)
            out.append(self.rows(m))
        return out

    # -- model matrices -------------------------------------------------------------
    def feature_matrix(self, cols: list[str]) -> torch.Tensor:
        """Feature-major float32 [F][n] (enum columns as their codes, NA -> NaN)."""
        if not cols:
            return torch.zeros((0, self.nrows), device=self.device)
        return torch.stack([self.vec(c).as_float() for c in cols]).contiguous()

    def summary(self) -> list[dict]:
        return [v.summary() for v in self.vecs]

    def to_pandas(self):
        import pandas as pd

        d = {}
        for v in self.vecs:
            if v.vtype == ENUM:
                codes = v.data.cpu().numpy()
                dom = np.array(list(v.domain) + [None], dtype=object)
                d[v.name] = dom[np.where(codes < 0, len(v.domain), codes)]
            else:
                d[v.name] = v.data.cpu().numpy()
        return pd.DataFrame(d)

    def head(self, n=10):
        return self[: min(n, self.nrows)]

    def __repr__(self):
        return f"Frame(key={self.key!r}, rows={self.nrows}, cols={self.names})"


def _num_label(a: float) -> str:
    return str(int(a)) if float(a).is_integer() else repr(float(a))


def _enum_vec(name: str, col: np.ndarray, device) -> Vec:
    mask = np.array([c is None or (isinstance(c, float) and np.isnan(c)) for c in col])
    vals = np.array(["" if m else str(c) for c, m in zip(col, mask)], dtype=object)
    domain = sorted(set(vals[~mask].tolist()))
    lut = {d: i for i, d in enumerate(domain)}
    codes = np.array([-1 if m else lut[v] for v, m in zip(vals, mask)], dtype=np.int32)
    return Vec(name, torch.as_tensor(codes, device=device), ENUM, domain)


class DKV:
    """Distributed key-value store of frames, models and jobs (per rank)."""

    _lock = threading.RLock()
    _store: dict = {}

    @classmethod
    def put(cls, key: str, obj):
        with cls._lock:
            cls._store[key] = obj
        return key

    @classmethod
    def get(cls, key: str, default=None):
        with cls._lock:
            return cls._store.get(key, default)

    @classmethod
    def remove(cls, key: str):
        with cls._lock:
            return cls._store.pop(key, None)

    @classmethod
    def keys(cls, kind=None):
        with cls._lock:
            if kind is None:
                return list(cls._store)
            return [k for k, v in cls._store.items() if isinstance(v, kind)]

    @classmethod
    def clear(cls):
        with cls._lock:
            cls._store.clear()
