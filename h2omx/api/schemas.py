"""JSON shapes of the H2O REST v3 API (``water.api.schemas3``), produced
from h2omx objects: TwoDimTable, FrameV3, ModelMetrics*, ModelV3 fragments.

The h2o-py / h2o-R clients read these documents; the field names follow
H2O's schema classes.  (No client is installed in this environment, so the
shapes are pinned by tests/test_rest_api.py through h2omx.client, which
issues the same requests h2o-py does.)
"""
from __future__ import annotations

import math

import numpy as np

H2O_VERSION = "3.46.0.6"


def _num(v):
    if v is None:
        return None
    if isinstance(v, (np.floating, float)):
        f = float(v)
        return f if math.isfinite(f) else ("NaN" if math.isnan(f) else ("Infinity" if f > 0 else "-Infinity"))
    if isinstance(v, (np.integer,)):
        return int(v)
    return v


def meta(schema_name: str, schema_type: str, version: int = 3) -> dict:
    return {"schema_version": version, "schema_name": schema_name, "schema_type": schema_type}


def two_dim_table(name: str, col_names: list, col_types: list, rows: list[list], description: str = "",
                  col_formats: list | None = None) -> dict:
    """H2O TwoDimTableV3: ``data`` is COLUMN-major (one list per column)."""
    ncol = len(col_names)
    cols = [[_num(r[j]) if j < len(r) else None for r in rows] for j in range(ncol)]
    fm = col_formats or ["%s" if t == "string" else ("%d" if t in ("int", "long") else "%.5f") for t in col_types]
    return {
        "__meta": meta("TwoDimTableV3", "TwoDimTable"),
        "name": name,
        "description": description,
        "columns": [{"__meta": meta("ColumnSpecsBase", "Iced"), "name": n, "type": t, "format": f, "description": n}
                    for n, t, f in zip(col_names, col_types, fm)],
        "rowcount": len(rows),
        "data": cols,
    }


def key_ref(name: str, kind: str) -> dict:
    url = {"Key<Frame>": f"/3/Frames/{name}", "Key<Model>": f"/3/Models/{name}"}.get(kind, "")
    return {"__meta": meta("KeyV3", "Iced"), "name": name, "type": kind, "URL": url}


# ---------------------------------------------------------------------------
def frame_json(key: str, summary: dict, preview: list | None = None, row_offset: int = 0, row_count: int = 10,
               full: bool = True) -> dict:
    cols = []
    for j, c in enumerate(summary["columns"]):
        ent = {
            "__meta": meta("ColV3", "Vec"),
            "label": c["label"],
            "type": c["type"],
            "missing_count": c["missing_count"],
            "zero_count": c["zero_count"],
            "positive_infinity_count": 0,
            "negative_infinity_count": 0,
            "mins": [_num(x) for x in c["mins"]],
            "maxs": [_num(x) for x in c["maxs"]],
            "mean": _num(c["mean"]),
            "sigma": _num(c["sigma"]),
            "domain": c["domain"],
            "domain_cardinality": c.get("domain_cardinality", 0),
            "precision": -1,
            "data": None,
            "string_data": None,
        }
        if preview is not None:
            vals = preview[j]
            if c["type"] == "enum":
                dom = c["domain"] or []
                ent["data"] = [float(dom.index(v)) if v is not None else "NaN" for v in vals]
            else:
                ent["data"] = [_num(v) if v is not None else "NaN" for v in vals]
        cols.append(ent)
    return {
        "__meta": meta("FrameV3", "Frame"),
        "frame_id": key_ref(key, "Key<Frame>"),
        "byte_size": 0,
        "is_text": False,
        "rows": summary["rows"],
        "row_offset": row_offset,
        "row_count": min(row_count, summary["rows"]),
        "column_offset": 0,
        "column_count": len(cols),
        "total_column_count": len(cols),
        "num_columns": len(cols),
        "columns": cols if full else None,
        "chunk_summary": None,
        "distribution_summary": None,
    }


def frame_base_json(key: str, rows: int, cols: int) -> dict:
    return {"__meta": meta("FrameBaseV3", "Frame"), "frame_id": key_ref(key, "Key<Frame>"), "rows": rows,
            "columns": cols, "byte_size": 0, "is_text": False}


# ---------------------------------------------------------------------------
def metrics_json(m: dict | None, category: str, model_key: str | None = None, frame_key: str | None = None,
                 domain: list | None = None) -> dict | None:
    if m is None:
        return None
    kind = {"Binomial": "ModelMetricsBinomial", "Multinomial": "ModelMetricsMultinomial",
            "Regression": "ModelMetricsRegression", "Clustering": "ModelMetricsClustering"}.get(category,
                                                                                           "ModelMetrics")
    out = {"__meta": meta(kind + "V3", kind), "model_category": category,
           "model": key_ref(model_key, "Key<Model>") if model_key else None,
           "frame": key_ref(frame_key, "Key<Frame>") if frame_key else None,
           "description": None, "scoring_time": 0, "predictions": None}
    for k, v in m.items():
        if k in ("confusion_matrix", "hit_ratio_table", "withinss", "size"):
            continue
        out[k] = _num(v) if not isinstance(v, (list, dict)) else v
    if category == "Binomial":
        out["pr_auc"] = out.get("AUCPR")
        dom = domain or ["0", "1"]
        cm = m.get("confusion_matrix")
        if cm is not None:
            (tn, fp), (fn, tp) = cm
            rows = [[dom[0], tn, fp, fp / max(tn + fp, 1e-300), f"({int(fp)}/{int(tn + fp)})"],
                    [dom[1], fn, tp, fn / max(fn + tp, 1e-300), f"({int(fn)}/{int(fn + tp)})"],
                    ["Total", tn + fn, fp + tp, (fp + fn) / max(tn + fp + fn + tp, 1e-300),
                     f"({int(fp + fn)}/{int(tn + fp + fn + tp)})"]]
            out["cm"] = {"__meta": meta("ConfusionMatrixV3", "ConfusionMatrix"),
                         "table": two_dim_table("Confusion Matrix (Act/Pred) for max f1 @ threshold = "
                                                f"{m.get('max_f1_threshold', 0.5)}",
                                                ["", dom[0], dom[1], "Error", "Rate"],
                                                ["string", "double", "double", "double", "string"], rows)}
        out["max_criteria_and_metric_scores"] = two_dim_table(
            "Maximum Metrics", ["metric", "threshold", "value", "idx"], ["string", "double", "double", "long"],
            [["max f1", m.get("max_f1_threshold"), m.get("max_f1"), 0]])
    elif category == "Multinomial":
        dom = domain or []
        cm = m.get("confusion_matrix")
        if cm is not None:
            K = len(cm)
            rows = []
            for i in range(K):
                tot = sum(cm[i])
                err = (tot - cm[i][i]) / tot if tot else 0.0
                rows.append([dom[i] if i < len(dom) else str(i)] + list(cm[i]) + [err])
            out["cm"] = {"__meta": meta("ConfusionMatrixV3", "ConfusionMatrix"),
                         "table": two_dim_table("Confusion Matrix", [""] + list(dom) + ["Error"],
                                                ["string"] + ["double"] * K + ["double"], rows)}
        hr = m.get("hit_ratio_table")
        if hr is not None:
            out["hit_ratio_table"] = two_dim_table("Top-K Hit Ratios", ["k", "hit_ratio"], ["int", "double"],
                                                   [[i + 1, v] for i, v in enumerate(hr)])
    elif category == "Clustering":
        out["tot_withinss"] = _num(m.get("tot_withinss"))
        out["totss"] = _num(m.get("totss"))
        out["betweenss"] = _num(m.get("betweenss"))
        ws, sz = m.get("withinss") or [], m.get("size") or []
        out["centroid_stats"] = two_dim_table("Centroid Statistics", ["centroid", "size", "within_cluster_sum_of_squares"],
                                              ["int", "double", "double"],
                                              [[i + 1, s, w] for i, (s, w) in enumerate(zip(sz, ws))])
    return out


def model_json(model) -> dict:
    from ..models.base import _jsonable

    j = model.to_json()
    out = j["output"]
    cat = model.category
    dom = model.response_domain
    out["training_metrics"] = metrics_json(model.training_metrics, cat, model.model_id, None, dom)
    out["validation_metrics"] = metrics_json(model.validation_metrics, cat, model.model_id, None, dom)
    out["cross_validation_metrics"] = metrics_json(model.cross_validation_metrics, cat, model.model_id, None, dom)
    vi = model.varimp()
    out["variable_importances"] = two_dim_table(
        "Variable Importances", ["variable", "relative_importance", "scaled_importance", "percentage"],
        ["string", "double", "double", "double"], [list(r) for r in vi]) if vi else None
    summ = model.summary()
    out["model_summary"] = two_dim_table("Model Summary", list(summ.keys()),
                                         ["string" if isinstance(v, str) else "double" for v in summ.values()],
                                         [[_jsonable(v) if not isinstance(v, (list, dict)) else str(v)
                                           for v in summ.values()]])
    sh = model.scoring_history or []
    if sh:
        keys = list(sh[0].keys())
        out["scoring_history"] = two_dim_table("Scoring History", keys, ["double"] * len(keys),
                                               [[r.get(k) for k in keys] for r in sh])
    else:
        out["scoring_history"] = None
    out["cross_validation_models"] = [key_ref(m.model_id, "Key<Model>") for m in model.cv_models] or None
    out["model_category"] = cat
    params = [{"__meta": meta("ModelParameterSchemaV3", "Iced"), "name": p["name"], "label": p["name"],
               "actual_value": p["actual_value"], "default_value": None, "input_value": p["actual_value"],
               "type": type(p["actual_value"]).__name__} for p in j["parameters"]]
    return {
        "__meta": meta("ModelSchemaV3", "Model"),
        "model_id": key_ref(model.model_id, "Key<Model>"),
        "algo": model.algo,
        "algo_full_name": j["algo_full_name"],
        "response_column_name": model.y,
        "data_frame": None,
        "timestamp": 0,
        "have_pojo": False,
        "have_mojo": True,
        "parameters": params,
        "output": out,
    }


def cloud_json(cluster, started_ms: int, node_infos: list[dict]) -> dict:
    import time

    return {
        "__meta": meta("CloudV3", "Iced"),
        "skip_ticks": False,
        "version": H2O_VERSION,
        "branch_name": "rel-h2omx",
        "last_commit_hash": "h2omx",
        "describe": "h2omx MI355X-native H2O cluster",
        "compiled_by": "h2omx",
        "compiled_on": "",
        "build_number": "1",
        "build_age": "0 days",
        "build_too_old": False,
        "node_idx": 0,
        "cloud_name": cluster.cfg.cloud_name,
        "cloud_size": cluster.world_size,
        "cloud_uptime_millis": int(time.time() * 1000) - started_ms,
        "cloud_internal_timezone": "UTC",
        "datafile_parser_timezone": "UTC",
        "cloud_healthy": True,
        "bad_nodes": 0,
        "consensus": True,
        "locked": True,
        "is_client": False,
        "nodes": node_infos,
        "internal_security_enabled": False,
        "leader_idx": 0,
        "web_ip": None,
        # h2omx extension: GPU peer topology + collective transport of the cloud
        # (runtime/topology.py); the operator copies it into the H2O CR status
        "h2omx_topology": _topology(cluster),
    }


def _topology(cluster) -> dict:
    from ..runtime.topology import cloud_summary

    return cloud_summary(getattr(cluster, "topology", None), getattr(cluster, "comm", None))
