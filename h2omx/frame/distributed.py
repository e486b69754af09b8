"""Cross-rank frame helpers: every rank holds a row shard of a frame under
the same key, so categorical domains and column statistics are combined
with collectives (H2O's distributed Vec rollups)."""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.distributed as dist

from .frame import ENUM, Frame, Vec


def _gather_objects(comm, obj):
    if comm is None or comm.world_size == 1:
        return [obj]
    out = [None] * comm.world_size
    dist.all_gather_object(out, obj)
    return out


def unify_domains(frame: Frame, comm) -> Frame:
    """Give every enum column the sorted union of the shards' domains and
    remap local codes to it (each rank's parser saw only its byte range)."""
    if comm is None or comm.world_size == 1:
        return frame
    enums = [v for v in frame.vecs if v.vtype == ENUM]
    local = {v.name: list(v.domain or []) for v in enums}
    allds = _gather_objects(comm, local)
    kinds = _gather_objects(comm, [v.vtype == ENUM for v in frame.vecs])
    if any(k != kinds[0] for k in kinds):
        raise ValueError("column types differ between shards; parse with explicit column types")
    new_vecs = []
    for v in frame.vecs:
        if v.vtype != ENUM:
            new_vecs.append(v)
            continue
        union = sorted(set().union(*[set(d.get(v.name) or []) for d in allds]))
        pos = {s: i for i, s in enumerate(union)}
        lut = torch.tensor([pos[s] for s in (v.domain or [])] + [-1], dtype=torch.int32, device=v.data.device)
        codes = v.data.long()
        codes = torch.where(codes < 0, torch.full_like(codes, len(v.domain or [])), codes)
        new_vecs.append(Vec(v.name, lut[codes].to(torch.int32), ENUM, union))
    return Frame(new_vecs, key=frame.key)


def global_nrows(frame: Frame, comm) -> int:
    n = frame.nrows
    if comm is None or comm.world_size == 1:
        return n
    return int(comm.all_reduce_numpy(np.array([float(n)]))[0])


def column_summaries(frame: Frame, comm) -> list[dict]:
    """H2O rollup stats (min, max, mean, sigma, NA / zero counts) over all shards."""
    rows = []
    stats = []
    for v in frame.vecs:
        x = v.as_float().double()
        na = torch.isnan(x)
        ok = x[~na]
        n = float(ok.numel())
        s1 = float(ok.sum()) if n else 0.0
        s2 = float((ok * ok).sum()) if n else 0.0
        mn = float(ok.min()) if n else math.inf
        mx = float(ok.max()) if n else -math.inf
        stats.append([n, s1, s2, float(na.sum()), float((ok == 0).sum()) if n else 0.0, mn, -mx])
    a = np.array(stats, dtype=np.float64).reshape(-1, 7)
    if comm is not None and comm.world_size > 1 and a.size:
        sums = comm.all_reduce_numpy(np.ascontiguousarray(a[:, :5]))
        mins = comm.all_reduce_numpy(np.ascontiguousarray(a[:, 5:]), "min")
        a = np.concatenate([sums, mins], 1)
    for v, (n, s1, s2, nas, zeros, mn, negmx) in zip(frame.vecs, a):
        mean = s1 / n if n else float("nan")
        var = (s2 - n * mean * mean) / (n - 1) if n > 1 else 0.0
        rows.append({"label": v.name, "type": v.vtype, "domain": v.domain, "missing_count": int(nas),
                     "zero_count": int(zeros), "mins": [mn if n else float("nan")],
                     "maxs": [-negmx if n else float("nan")], "mean": mean,
                     "sigma": math.sqrt(max(var, 0.0)) if n else float("nan"),
                     "domain_cardinality": len(v.domain or [])})
    return rows


def gather_frame(frame: Frame, comm, max_rows: int | None = None) -> Frame:
    """Concatenate all shards on every rank (small frames only: downloads,
    leaderboards, previews)."""
    if comm is None or comm.world_size == 1:
        return frame
    vecs = []
    for v in frame.vecs:
        d = v.data if max_rows is None else v.data[:max_rows]
        vecs.append(Vec(v.name, comm.all_gather_cat(d.contiguous()), v.vtype, v.domain))
    return Frame(vecs, key=frame.key)
