"""Frame utilities behind H2O's ``h2o.create_frame``, ``h2o.interaction``
and ``H2OFrame.insert_missing_values`` (REST ``/3/CreateFrame``,
``/3/Interaction``, ``/3/MissingInserter``).

Every function works on the calling rank's row shard.  ``create_frame``
generates each rank's share of the rows; its column layout and categorical
domains come from the global seed, so all ranks agree.  ``interaction``
builds the level vocabulary from all-gathered level counts, so every shard
gets the same domain.
"""
from __future__ import annotations

import itertools

import numpy as np
import torch

from .distributed import _gather_objects
from .frame import ENUM, Frame, Vec


def create_frame(rows: int = 10000, cols: int = 10, *, randomize: bool = True, real_range: float = 100.0,
                 categorical_fraction: float = 0.2, factors: int = 100, integer_fraction: float = 0.2,
                 integer_range: int = 100, binary_fraction: float = 0.1, binary_ones_fraction: float = 0.02,
                 time_fraction: float = 0.0, string_fraction: float = 0.0, missing_fraction: float = 0.01,
                 has_response: bool = False, response_factors: int = 2, positive_response: bool = False,
                 seed: int = 1234, value: float = 0.0, comm=None, device="cpu") -> Frame:
    """Random frame with H2O CreateFrame's column mix (real / categorical /
    integer / binary / time columns, NA fraction, optional response first)."""
    world = comm.world_size if comm is not None else 1
    rank = comm.rank if comm is not None else 0
    n = rows // world + (1 if rank < rows % world else 0)
    rng = np.random.default_rng(seed)
    fr_ = np.array([categorical_fraction, integer_fraction, binary_fraction, time_fraction, string_fraction])
    if fr_.sum() > 1.0 + 1e-9:
        raise ValueError("create_frame: column fractions sum to more than 1")
    counts = np.floor(fr_ * cols).astype(int)
    kinds = (["enum"] * counts[0] + ["int"] * counts[1] + ["bin"] * counts[2] + ["time"] * counts[3]
             + ["str"] * counts[4])
    kinds += ["real"] * (cols - len(kinds))
    rng.shuffle(kinds)
    g = torch.Generator().manual_seed(int(seed) * 1000003 + rank)
    vecs = []
    if has_response:
        if response_factors > 1:
            yv = torch.randint(0, response_factors, (n,), generator=g).to(torch.int32)
            vecs.append(Vec("response", yv.to(device), ENUM, [str(i) for i in range(response_factors)]))
        else:
            r = torch.rand(n, generator=g, dtype=torch.float64) * real_range
            r = r if positive_response else r * 2 - real_range
            vecs.append(Vec("response", r.float().to(device), "real"))
    for j, k in enumerate(kinds):
        name = f"C{j + 1}"
        if k in ("enum", "str"):
            pre = f"c{j}.l" if k == "enum" else f"s{j}_"
            lv = [f"{pre}{i}" for i in range(max(1, factors))]
            v = Vec(name, torch.randint(0, len(lv), (n,), generator=g).to(torch.int32), ENUM, lv)
        elif k == "int":
            v = Vec(name, torch.randint(-integer_range, integer_range + 1, (n,), generator=g).float(), "int")
        elif k == "bin":
            v = Vec(name, (torch.rand(n, generator=g) < binary_ones_fraction).float(), "int")
        elif k == "time":
            ms = torch.randint(0, 50 * 365 * 86400, (n,), generator=g).double() * 1000.0
            v = Vec(name, ms.float(), "time")
        else:
            d = ((torch.rand(n, generator=g, dtype=torch.float64) * 2 - 1) * real_range).float() if randomize \
                else torch.full((n,), float(value))
            v = Vec(name, d, "real")
        if missing_fraction > 0:
            v = _with_na(v, torch.rand(n, generator=g) < missing_fraction)
        vecs.append(Vec(v.name, v.data.to(device), v.vtype, v.domain))
    return Frame(vecs)


def _with_na(v: Vec, mask: torch.Tensor) -> Vec:
    mask = mask.to(v.data.device)
    if v.vtype == ENUM:
        return Vec(v.name, torch.where(mask, torch.full_like(v.data, -1), v.data), ENUM, v.domain)
    d = v.data.float()
    return Vec(v.name, torch.where(mask, torch.full_like(d, float("nan")), d), v.vtype)


def insert_missing_values(frame: Frame, fraction: float = 0.1, seed: int | None = None, comm=None) -> Frame:
    """Replace a ``fraction`` of the entries of every column with NA (in place
    on the frame, as H2O's MissingInserter)."""
    rank = comm.rank if comm is not None else 0
    g = torch.Generator().manual_seed((int(seed) if seed is not None and seed >= 0 else 42) * 7919 + rank)
    new = [_with_na(v, torch.rand(frame.nrows, generator=g) < float(fraction)) for v in frame.vecs]
    frame.vecs[:] = new
    return frame


def interaction(frame: Frame, factors, pairwise: bool = False, max_factors: int = 100, min_occurrence: int = 1,
                comm=None) -> Frame:
    """Categorical interaction columns (H2O ``h2o.interaction``).  With
    ``pairwise`` there is one column per pair of factors, otherwise one column
    for all of them.  Levels are "a_b" strings.  Only the ``max_factors``
    most frequent levels that occur at least ``min_occurrence`` times
    (counted over all ranks) are kept; all others become "other"."""
    factors = [frame.names[f] if isinstance(f, int) else f for f in factors]
    for f in factors:
        if frame.vec(f).vtype != ENUM:
            raise ValueError(f"interaction: column {f!r} is not categorical")
    groups = list(itertools.combinations(factors, 2)) if pairwise else [tuple(factors)]
    out = []
    for grp in groups:
        vs = [frame.vec(c) for c in grp]
        codes = torch.zeros(frame.nrows, dtype=torch.int64, device=frame.device)
        na = torch.zeros(frame.nrows, dtype=torch.bool, device=frame.device)
        mult = 1
        for v in reversed(vs):
            c = v.data.long()
            na |= c < 0
            codes = codes + c.clamp_min(0) * mult
            mult *= max(1, len(v.domain or []))
        u, cnt = torch.unique(codes[~na], return_counts=True)
        merged: dict[int, int] = {}
        for d in _gather_objects(comm, dict(zip(u.cpu().tolist(), cnt.cpu().tolist()))):
            for k, c in d.items():
                merged[k] = merged.get(k, 0) + c
        keep = sorted((k for k, c in merged.items() if c >= int(min_occurrence)), key=lambda k: (-merged[k], k))
        keep = sorted(keep[: int(max_factors)])

        def label(code):
            parts, rem = [], code
            for v in reversed(vs):
                L = max(1, len(v.domain or []))
                parts.append(v.domain[rem % L])
                rem //= L
            return "_".join(reversed(parts))

        dom = [label(k) for k in keep]
        other = len(dom) < len(merged)
        if other:
            dom.append("other")
        new = torch.full_like(codes, len(keep) if other else -1)
        if keep:
            keys = torch.tensor(keep, dtype=torch.int64, device=frame.device)
            pos = torch.searchsorted(keys, codes).clamp(max=len(keep) - 1)
            new = torch.where(keys[pos] == codes, pos, new)
        new = torch.where(na, torch.full_like(new, -1), new)
        out.append(Vec("_".join(grp), new.to(torch.int32), ENUM, dom))
    return Frame(out)
