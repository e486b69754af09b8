"""Cluster operations: the functions every rank runs, in the same order,
when the leader's REST layer issues a command (see cluster.Cluster.run).

Each op works on the rank's own row shard and combines results with the
shared communicator; the leader's return value is what the REST layer
reports.  Arguments are JSON-serialisable (frame / model keys, parameter
dicts) because they travel over the command bus.
"""
from __future__ import annotations

import base64
import os
import tempfile

import numpy as np
import torch

from ..frame.distributed import column_summaries, gather_frame, global_nrows, unify_domains
from ..frame.frame import DKV, ENUM, Frame, Vec


def _dev(cl):
    return cl.comm.device


def _frame(key) -> Frame:
    fr = DKV.get(key)
    if not isinstance(fr, Frame):
        raise KeyError(f"frame {key!r} not found")
    return fr


def _model(key):
    from ..models.base import Model

    m = DKV.get(key)
    if not isinstance(m, Model):
        raise KeyError(f"model {key!r} not found")
    return m


# ---------------------------------------------------------------------------
def op_import_files(cl, paths, dest, sep=None, header=None, col_types=None, col_names=None):
    from ..frame.parse import import_shard, sample_setup

    files = []
    for p in paths:
        if os.path.isdir(p):
            files += sorted(os.path.join(p, f) for f in os.listdir(p) if not f.startswith("."))
        else:
            files.append(p)
    # the leader fixes names / types / separator so every shard parses alike
    setup = None
    if cl.rank == 0:
        setup = sample_setup(files[0], sep, header)
        if col_types:
            setup["column_types"] = ["Enum" if str(t).lower() in ("enum", "categorical", "factor") else
                                     ("String" if str(t).lower() == "string" else "Numeric") for t in col_types]
        if col_names:
            setup["column_names"] = list(col_names)
    if cl.world_size > 1:
        setup = cl.comm.broadcast_object(setup, 0)
    parts = [import_shard(f, cl.rank, cl.world_size, setup if i == 0 else dict(setup, check_header=setup["check_header"]),
                          device=_dev(cl)) for i, f in enumerate(files)]
    fr = parts[0] if len(parts) == 1 else _rbind(parts)
    fr = unify_domains(fr, cl.comm)
    fr.key = dest
    DKV.put(dest, fr)
    return {"key": dest, "rows": global_nrows(fr, cl.comm), "cols": fr.ncols}


def _rbind(frames):
    from ..frame.distributed import unify_domains as _u  # noqa: F401

    vecs = []
    for j, v0 in enumerate(frames[0].vecs):
        if v0.vtype == ENUM:
            union = sorted(set().union(*[set(f.vecs[j].domain or []) for f in frames]))
            pos = {s: i for i, s in enumerate(union)}
            datas = []
            for f in frames:
                v = f.vecs[j]
                lut = torch.tensor([pos[s] for s in (v.domain or [])] + [-1], dtype=torch.int32, device=v.data.device)
                c = v.data.long()
                datas.append(lut[torch.where(c < 0, torch.full_like(c, len(v.domain or [])), c)])
            vecs.append(Vec(v0.name, torch.cat(datas).to(torch.int32), ENUM, union))
        else:
            vecs.append(Vec(v0.name, torch.cat([f.vecs[j].data for f in frames]), v0.vtype))
    return Frame(vecs)


def op_parse_blob(cl, blob_key, dest, sep=None, header=None, col_types=None, col_names=None):
    """Parse an uploaded file (/3/PostFile): the leader stored its bytes under
    ``blob/<key>`` in the command-bus store (or the local blob table)."""
    data = _get_blob(cl, blob_key)
    fd, path = tempfile.mkstemp(suffix=".csv")
    try:
        with os.fdopen(fd, "wb") as fh:
            fh.write(data)
        return op_import_files(cl, [path], dest, sep, header, col_types, col_names)
    finally:
        os.unlink(path)


_BLOBS: dict[str, bytes] = {}


def put_blob(cl, key: str, data: bytes):
    _BLOBS[key] = data
    if cl.world_size > 1 and cl.store is not None:
        cl.store.set(f"blob/{key}", base64.b64encode(data))


def _get_blob(cl, key):
    if key in _BLOBS:
        return _BLOBS[key]
    if cl.store is not None:
        return base64.b64decode(cl.store.get(f"blob/{key}"))
    raise KeyError(key)


def blob_setup(cl, key, sep=None, header=None) -> dict:
    """ParseSetup on the leader's copy of the data (column names / types)."""
    from ..frame.parse import parse_setup

    if key in _BLOBS:
        fd, path = tempfile.mkstemp(suffix=".csv")
        with os.fdopen(fd, "wb") as fh:
            fh.write(_BLOBS[key][: 1 << 22])
        try:
            return parse_setup(path, sep, header)
        finally:
            os.unlink(path)
    return parse_setup(key, sep, header)


def op_synthetic(cl, kind, rows, dest, cols=None, seed=42):
    """Device-generated synthetic frames (HIGGS / Airlines / wide Gaussian
    shapes from BASELINE.md); each rank generates its share of ``rows``."""
    from ..frame import synthetic

    per = rows // cl.world_size + (1 if cl.rank < rows % cl.world_size else 0)
    s = seed + 1000003 * cl.rank
    if kind == "wide_gaussian":
        X, y = synthetic.wide_gaussian(per, int(cols or 100), seed=s, device=_dev(cl))
    else:
        X, y = getattr(synthetic, kind)(per, seed=s, device=_dev(cl))
    fr = Frame.from_tensor(X.contiguous(), y=y, y_name="response", y_categorical=True)
    fr.vecs[-1].domain = ["0", "1"]
    fr.key = dest
    DKV.put(dest, fr)
    return {"key": dest, "rows": global_nrows(fr, cl.comm), "cols": fr.ncols}


def _resolve_params(params: dict) -> dict:
    out = {}
    for k, v in params.items():
        if k in ("user_points",) and isinstance(v, str):
            out[k] = _frame(v)
        else:
            out[k] = v
    return out


def op_train(cl, algo, params, x=None, y=None, training_frame=None, validation_frame=None, model_id=None):
    from ..models import ESTIMATORS

    cls = ESTIMATORS.get(algo)
    if cls is None:
        raise ValueError(f"unknown algorithm {algo!r}")
    p = _resolve_params(dict(params))
    p["model_id"] = model_id
    est = cls(**p)
    if algo == "generic":                      # MOJO import: no training frame
        return est.train(comm=cl.comm if cl.world_size > 1 else None).model_id
    tr = _frame(training_frame)
    va = _frame(validation_frame) if validation_frame else None
    comm = cl.comm if cl.world_size > 1 else None
    m = est.train(x=x, y=y, training_frame=tr, validation_frame=va, comm=comm)
    return m.model_id


def op_predict(cl, model, frame, dest, kind="predict", leaf_type="Path"):
    m = _model(model)
    fr = _frame(frame)
    if kind == "contributions":
        pf = m.predict_contributions(fr)
    elif kind == "leaf_nodes":
        pf = m.predict_leaf_node_assignment(fr, leaf_type)
    elif kind == "staged_proba":
        pf = m.staged_predict_proba(fr)
    elif kind == "feature_frequencies":
        pf = m.feature_frequencies(fr)
    else:
        pf = m.predict(fr)
    pf.key = dest
    DKV.put(dest, pf)
    return {"key": dest, "rows": global_nrows(pf, cl.comm)}


def op_partial_dependence(cl, model, frame, cols, nbins=20, targets=(None,)):
    from ..explain import partial_dependence

    m = _model(model)
    fr = _frame(frame)
    comm = cl.comm if cl.world_size > 1 else None
    return [partial_dependence(m, fr, c, nbins=nbins, target=t, comm=comm) for c in cols for t in targets]


def op_model_metrics(cl, model, frame):
    m = _model(model)
    fr = _frame(frame)
    old = m.comm
    m.comm = cl.comm if cl.world_size > 1 else None
    try:
        if m.category == "Clustering":
            return m.model_performance(fr)
        return m._metrics(fr, m.predict_raw(fr), m.comm)
    finally:
        m.comm = old


def op_frame_summary(cl, key):
    fr = _frame(key)
    return {"rows": global_nrows(fr, cl.comm), "columns": column_summaries(fr, cl.comm)}


def op_frame_rows(cl, key, n=10, offset=0):
    fr = _frame(key)
    g = gather_frame(fr, cl.comm, max_rows=offset + n)
    out = []
    for v in g.vecs:
        d = v.data[offset: offset + n].cpu()
        if v.vtype == ENUM:
            out.append([v.domain[i] if i >= 0 else None for i in d.tolist()])
        else:
            out.append([None if np.isnan(a) else float(a) for a in d.double().numpy()])
    return out


def op_frame_download(cl, key):
    fr = gather_frame(_frame(key), cl.comm)
    return fr.to_pandas().to_csv(index=False)


def op_delete(cl, key):
    DKV.remove(key)
    return True


def op_delete_all(cl, retain=None):
    keep = set(retain or [])
    for k in list(DKV.keys()):
        if k not in keep:
            DKV.remove(k)
    return True


def op_split_frame(cl, key, ratios, dests, seed=-1):
    fr = _frame(key)
    parts = fr.split_frame(tuple(ratios), seed=(seed if seed is not None and seed >= 0 else 1234) + 7919 * cl.rank)
    out = []
    for p, d in zip(parts, dests):
        p.key = d
        DKV.put(d, p)
        out.append({"key": d, "rows": global_nrows(p, cl.comm)})
    return out


def op_rapids(cl, ast, session_id=None):
    from ..api.rapids import evaluate

    return evaluate(ast, cl)


def op_automl(cl, spec):
    from ..automl import run_automl

    return run_automl(spec, comm=cl.comm if cl.world_size > 1 else None)


def op_grid(cl, algo, params, hyper_params, search_criteria=None, x=None, y=None, training_frame=None,
            validation_frame=None, grid_id=None):
    from ..grid import run_grid

    return run_grid(algo, _resolve_params(dict(params)), hyper_params, search_criteria, x, y, training_frame,
                    validation_frame, grid_id, comm=cl.comm if cl.world_size > 1 else None)


def op_grid_sorted(cl, grid_id, sort_by=None, decreasing=None):
    g = DKV.get(grid_id)
    if g is None:
        raise KeyError(grid_id)
    return g.get_grid(sort_by, decreasing).to_json()


def op_save_model(cl, model, path):
    from ..mojo import save_model

    if cl.rank == 0:
        return save_model(_model(model), path)
    return path


def op_load_model(cl, path):
    from ..mojo import load_model

    m = load_model(path)
    DKV.put(m.model_id, m)
    return m.model_id


def op_create_frame(cl, dest, spec):
    from ..frame.tools import create_frame

    fr = create_frame(comm=cl.comm if cl.world_size > 1 else None, device=_dev(cl), **spec)
    fr.key = dest
    DKV.put(dest, fr)
    return {"key": dest, "rows": global_nrows(fr, cl.comm), "cols": fr.ncols}


def op_interaction(cl, source, dest, factors, pairwise=False, max_factors=100, min_occurrence=1):
    from ..frame.tools import interaction

    fr = interaction(_frame(source), factors, pairwise, max_factors, min_occurrence,
                     comm=cl.comm if cl.world_size > 1 else None)
    fr.key = dest
    DKV.put(dest, fr)
    return {"key": dest, "rows": global_nrows(fr, cl.comm), "cols": fr.ncols}


def op_insert_missing(cl, key, fraction=0.1, seed=-1):
    from ..frame.tools import insert_missing_values

    insert_missing_values(_frame(key), fraction, seed, comm=cl.comm if cl.world_size > 1 else None)
    return {"key": key}


def op_frame_export(cl, key, path, force=False):
    """h2o.export_file: the leader writes the gathered frame as CSV."""
    fr = gather_frame(_frame(key), cl.comm)
    if cl.rank == 0:
        if os.path.exists(path) and not force:
            raise FileExistsError(f"{path} exists (use force=True)")
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        fr.to_pandas().to_csv(path, index=False)
    return path


def op_w2v_synonyms(cl, model, word, count=20):
    return _model(model).find_synonyms(word, int(count))


def op_w2v_transform(cl, model, frame, dest, aggregate_method="NONE"):
    m = _model(model)
    out = m.transform(_frame(frame), aggregate_method)
    out.key = dest
    DKV.put(dest, out)
    return {"key": dest, "rows": global_nrows(out, cl.comm)}


def op_network_test(cl, sizes=(1 << 10, 1 << 16, 1 << 20, 1 << 24), reps=5):
    """Collective latency / bandwidth over the cluster's communicator (H2O
    NetworkTest): all-reduce of fp32 buffers of each size, timed on the leader."""
    import time

    dev = _dev(cl)
    out = []
    for nbytes in sizes:
        t = torch.ones(max(1, int(nbytes) // 4), dtype=torch.float32, device=dev)
        cl.comm.all_reduce_(t)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        cl.comm.barrier()
        t0 = time.perf_counter()
        for _ in range(int(reps)):
            cl.comm.all_reduce_(t)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dt = cl.comm.max_scalar((time.perf_counter() - t0) / int(reps))
        w = cl.world_size
        bus = 2.0 * (w - 1) / w * t.numel() * 4 / dt if w > 1 and dt > 0 else 0.0
        out.append({"bytes": int(t.numel() * 4), "microseconds": dt * 1e6, "bus_bandwidth_GBps": bus / 1e9})
    return {"world_size": cl.world_size, "backend": _backend_name(cl), "results": out}


def _backend_name(cl):
    import torch.distributed as dist

    return dist.get_backend() if cl.world_size > 1 and dist.is_initialized() else "local"


def op_make_metrics(cl, predictions, actuals, domain=None, distribution=None, weights=None):
    from ..tools import make_metrics

    return make_metrics(_frame(predictions), _frame(actuals), domain, distribution,
                        _frame(weights) if weights else None, comm=cl.comm if cl.world_size > 1 else None)


def op_permutation_importance(cl, model, frame, metric="AUTO", n_repeats=1, seed=-1, features=None):
    from ..tools import permutation_importance

    m = _model(model)
    old = m.comm
    m.comm = cl.comm if cl.world_size > 1 else None
    try:
        return permutation_importance(m, _frame(frame), metric, n_repeats, seed, features)
    finally:
        m.comm = old


def op_train_segments(cl, algo, params, segment_columns, x=None, y=None, training_frame=None,
                      validation_frame=None, segment_models_id=None):
    from ..models import ESTIMATORS
    from ..tools import train_segments

    return train_segments(ESTIMATORS[algo], _resolve_params(dict(params)), segment_columns, x, y,
                          _frame(training_frame), _frame(validation_frame) if validation_frame else None,
                          segment_models_id, comm=cl.comm if cl.world_size > 1 else None)


def op_fault(cl, rank=-1, kind="raise"):
    """Test-only fault injection: rank ``rank`` fails the command."""
    if rank in (-1, cl.rank):
        raise RuntimeError(f"injected fault on rank {cl.rank}")
    return True


OPS = {name[3:]: fn for name, fn in list(globals().items()) if name.startswith("op_")}


def register_all(cl):
    for name, fn in OPS.items():
        cl.register(name, fn)
