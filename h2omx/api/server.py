"""H2O REST API served by the leader node (port 54321).

Implements the routes the h2o-py / h2o-R clients use to connect, load data,
build models, score and download MOJOs:

  GET  /3/Cloud  /3/About  /3/Capabilities  /3/Metadata/endpoints  /3/InitID
  POST /4/sessions           DELETE /4/sessions/{id}
  GET  /3/ImportFiles        POST /3/ImportFilesMulti   POST /3/PostFile
  POST /3/ParseSetup         POST /3/Parse
  GET  /3/Frames[/{id}[/summary|/columns/{c}/summary]]  DELETE /3/Frames/{id}
  GET  /3/DownloadDataset    POST /3/SplitFrame
  GET  /3/ModelBuilders[/{algo}]   POST /3/ModelBuilders/{algo}[/parameters]
  GET  /3/Jobs[/{id}]        POST /3/Jobs/{id}/cancel
  GET  /3/Models[/{id}]      DELETE /3/Models/{id}     GET /3/Models/{id}/mojo
  POST /99/Models.bin/{id}   POST /99/Models.upload.bin   GET /99/Models.fetch.bin/{id}
  POST /3/Predictions/models/{m}/frames/{f}   POST /4/Predictions/models/{m}/frames/{f}
  POST /3/ModelMetrics/models/{m}/frames/{f}
  POST /3/Predictions/...?predict_contributions=true  (TreeSHAP)
  POST /3/PartialDependence  GET /3/PartialDependence/{id}
  POST /99/Grid/{algo}       GET /99/Grids[/{id}]
  POST /99/AutoMLBuilder     GET /99/AutoML/{id}    GET /99/Leaderboards/{id}
  POST /99/Rapids            DELETE /3/DKV[/{key}]  POST /3/Shutdown
  GET  /3/Logs/nodes/{n}/files/{name}   GET /3/Timeline   GET /metrics

Requests are parsed like H2O does: query string for GET, form-encoded (or
JSON) bodies for POST, parameter values in H2O's string syntax (``[a,b]``
lists, ``true``/``false``).  Operations on sharded data go through the
cluster command bus so every rank participates.
"""
from __future__ import annotations

import io
import json
import logging
import math
import os
import re
import threading
import time
import uuid
import zipfile
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, unquote, urlparse

import numpy as np

from ..frame.frame import DKV, Frame
from ..runtime.jobs import JobRegistry
from . import schemas as S

log = logging.getLogger("h2omx.api")
LOG_BUFFER: list[str] = []



# model categories each builder produces (GET /3/ModelBuilders "can_build")
_CAN_BUILD = {"kmeans": ["Clustering"], "pca": ["DimReduction"], "svd": ["DimReduction"], "glrm": ["DimReduction"],
              "aggregator": ["DimReduction"], "isolationforest": ["AnomalyDetection"],
              "extendedisolationforest": ["AnomalyDetection"], "coxph": ["CoxPH"], "rulefit": ["Binomial", "Regression"], "word2vec": ["WordEmbedding"],
              "targetencoder": ["TargetEncoder"], "isotonicregression": ["Regression"], "adaboost": ["Binomial"],
              "upliftdrf": ["BinomialUplift"], "infogram": ["Binomial", "Multinomial", "Regression"],
              "psvm": ["Binomial"]}

class _BufferHandler(logging.Handler):
    def emit(self, record):
        LOG_BUFFER.append(self.format(record))
        if len(LOG_BUFFER) > 5000:
            del LOG_BUFFER[:1000]


_bh = _BufferHandler()
_bh.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s"))
logging.getLogger("h2omx").addHandler(_bh)
logging.getLogger("h2omx").setLevel(logging.INFO)


class ApiError(Exception):
    def __init__(self, status: int, msg: str, exc_type: str = "IllegalArgumentException"):
        super().__init__(msg)
        self.status = status
        self.msg = msg
        self.exc_type = exc_type


# ---------------------------------------------------------------------------
# H2O parameter-string parsing
# ---------------------------------------------------------------------------
def parse_list(v) -> list:
    if isinstance(v, list):
        return v
    if v is None:
        return []
    s = str(v).strip()
    if s in ("", "null", "[]"):
        return []
    if s.startswith("["):
        try:
            return json.loads(s)
        except ValueError:
            s = s[1:-1]
    return [p.strip().strip('"').strip("'") for p in s.split(",") if p.strip()]


def coerce(value, default):
    """Convert an H2O REST string into the Python type of ``default``."""
    if not isinstance(value, str):
        return value
    s = value.strip()
    if s in ("null", "None"):
        return None
    if isinstance(default, bool):
        return s.lower() in ("true", "1")
    if isinstance(default, int) and not isinstance(default, bool):
        try:
            return int(float(s))
        except ValueError:
            return default
    if isinstance(default, float):
        try:
            return float(s)
        except ValueError:
            return default
    if isinstance(default, list):
        items = parse_list(s)
        if default and isinstance(default[0], (int, float)):
            return [type(default[0])(float(x)) for x in items]
        return items
    if default is None:
        if s.startswith("[") or s.startswith("{"):
            try:
                return json.loads(s)
            except ValueError:
                return parse_list(s)
        if s.lower() in ("true", "false"):
            return s.lower() == "true"
        try:
            return int(s)
        except ValueError:
            pass
        try:
            return float(s)
        except ValueError:
            return s.strip('"')
    return s.strip('"')


_REST_ALIASES = {"lambda": "lambda_", "alpha": "alpha"}


def _predict_kind(params) -> str:
    """/3/Predictions flags (H2O PredictionsHandler): contributions, leaf node
    assignment, staged probabilities or feature frequencies instead of scores."""
    for flag, kind in (("predict_contributions", "contributions"), ("leaf_node_assignment", "leaf_nodes"),
                       ("predict_staged_proba", "staged_proba"), ("feature_frequencies", "feature_frequencies")):
        if str(params.get(flag, "false")).lower() == "true":
            return kind
    return "predict"


class H2OApi:
    """Route table + handlers; transport-independent (tests call ``handle``)."""

    def __init__(self, cluster, shutdown_cb=None):
        self.cluster = cluster
        self.jobs = JobRegistry()
        self.peer_lost: str | None = None
        wd = getattr(cluster, "watchdog", None)
        if wd is not None:
            wd.on_lost(self._on_peer_lost)
        self.sessions: dict[str, float] = {}
        self.started_ms = int(time.time() * 1000)
        self.shutdown_cb = shutdown_cb
        self.counters = {"requests": 0, "models_built": 0, "rows_parsed": 0}
        self.timeline: list[dict] = []
        self.automl: dict[str, object] = {}
        self.grid_results: dict[str, dict] = {}
        self.pdp_results: dict[str, list] = {}
        self.routes = []
        R = self._route
        R("GET", r"/3/Cloud", self.cloud)
        R("HEAD", r"/3/Cloud", self.cloud)
        R("GET", r"/3/About", self.about)
        R("GET", r"/3/Capabilities(/.*)?", self.capabilities)
        R("GET", r"/3/Metadata/endpoints", self.endpoints)
        R("GET", r"/3/InitID", self.init_id)
        R("POST", r"/4/sessions", self.new_session)
        R("DELETE", r"/4/sessions/(?P<sid>[^/]+)", self.end_session)
        R("GET", r"/3/ImportFiles", self.import_files)
        R("POST", r"/3/ImportFiles", self.import_files)
        R("POST", r"/3/ImportFilesMulti", self.import_files_multi)
        R("POST", r"/3/PostFile(\.bin)?", self.post_file)
        R("POST", r"/3/ParseSetup", self.parse_setup)
        R("POST", r"/3/Parse", self.parse)
        R("GET", r"/3/Frames", self.frames)
        R("GET", r"/3/Frames/(?P<fid>[^/]+)", self.frame)
        R("GET", r"/3/Frames/(?P<fid>[^/]+)/summary", self.frame)
        R("GET", r"/3/Frames/(?P<fid>[^/]+)/light", self.frame)
        R("GET", r"/3/Frames/(?P<fid>[^/]+)/columns/(?P<col>[^/]+)/summary", self.frame_column)
        R("DELETE", r"/3/Frames/(?P<fid>[^/]+)", self.delete_key)
        R("GET", r"/3/DownloadDataset(\.bin)?", self.download_dataset)
        R("POST", r"/3/SplitFrame", self.split_frame)
        R("GET", r"/3/ModelBuilders", self.model_builders)
        R("GET", r"/3/ModelBuilders/(?P<algo>[^/]+)", self.model_builders)
        R("POST", r"/3/ModelBuilders/(?P<algo>[^/]+)/parameters", self.validate_params)
        R("POST", r"/3/ModelBuilders/(?P<algo>[^/]+)", self.build_model)
        R("GET", r"/3/Jobs", self.jobs_list)
        R("GET", r"/3/Jobs/(?P<jid>[^/]+)", self.job)
        R("POST", r"/3/Jobs/(?P<jid>[^/]+)/cancel", self.job_cancel)
        R("GET", r"/3/Models", self.models)
        R("GET", r"/3/Models/(?P<mid>[^/]+)", self.model)
        R("DELETE", r"/3/Models/(?P<mid>[^/]+)", self.delete_key)
        R("GET", r"/3/Models/(?P<mid>[^/]+)/mojo", self.mojo)
        R("GET", r"/3/Models\.mojo/(?P<mid>[^/]+)", self.mojo)
        R("POST", r"/99/Models\.bin/(?P<mid>[^/]*)", self.save_model)
        R("GET", r"/99/Models\.fetch\.bin/(?P<mid>[^/]+)", self.mojo)
        R("POST", r"/99/Models\.upload\.bin/(?P<mid>[^/]*)", self.upload_model)
        R("POST", r"/99/Models\.mojo/(?P<mid>[^/]*)", self.save_model)
        R("POST", r"/3/Predictions/models/(?P<mid>[^/]+)/frames/(?P<fid>[^/]+)", self.predict)
        R("POST", r"/4/Predictions/models/(?P<mid>[^/]+)/frames/(?P<fid>[^/]+)", self.predict_async)
        R("POST", r"/3/ModelMetrics/models/(?P<mid>[^/]+)/frames/(?P<fid>[^/]+)", self.model_metrics)
        R("GET", r"/3/ModelMetrics/models/(?P<mid>[^/]+)/frames/(?P<fid>[^/]+)", self.model_metrics)
        R("POST", r"/99/Grid/(?P<algo>[^/]+)", self.grid_build)
        R("GET", r"/99/Grids", self.grids)
        R("GET", r"/99/Grids/(?P<gid>[^/]+)", self.grid_get)
        R("POST", r"/99/AutoMLBuilder", self.automl_build)
        R("GET", r"/99/AutoML/(?P<aid>[^/]+)", self.automl_get)
        R("GET", r"/99/Leaderboards/(?P<aid>[^/]+)", self.leaderboard)
        R("POST", r"/3/PartialDependence/?", self.partial_dependence)
        R("GET", r"/3/PartialDependence/(?P<pid>[^/]+)", self.partial_dependence_get)
        R("POST", r"/99/Rapids", self.rapids)
        R("DELETE", r"/3/DKV", self.delete_all)
        R("DELETE", r"/3/DKV/(?P<key>[^/]+)", self.delete_key)
        R("POST", r"/3/Shutdown", self.shutdown)
        R("GET", r"/3/Logs/nodes/(?P<node>[^/]+)/files/(?P<name>[^/]+)", self.logs)
        R("GET", r"/3/Logs/download", self.logs)
        R("GET", r"/3/Timeline", self.timeline_get)
        R("GET", r"/3/NodePersistentStorage/.*", self.nps)
        R("GET", r"/metrics", self.prometheus)
        R("POST", r"/3/LogAndEcho", self.log_and_echo)
        R("POST", r"/3/Frames/(?P<fid>[^/]+)/export", self.frame_export)
        R("POST", r"/3/CreateFrame", self.create_frame)
        R("POST", r"/3/Interaction", self.interaction)
        R("POST", r"/3/MissingInserter", self.missing_inserter)
        R("GET", r"/3/Word2VecSynonyms", self.w2v_synonyms)
        R("GET", r"/3/Word2VecTransform", self.w2v_transform)
        R("GET", r"/3/NetworkTest", self.network_test)
        R("GET", r"/3/Typeahead/files", self.typeahead_files)
        R("POST", r"/3/GarbageCollect", self.garbage_collect)
        R("GET", r"/3/JStack", self.jstack)
        R("GET", r"/3/ModelMetrics", self.model_metrics_all)
        R("POST", r"/3/ModelMetrics/predictions_frame/(?P<pf>[^/]+)/actuals_frame/(?P<af>[^/]+)", self.make_metrics)
        R("POST", r"/3/PermutationVarImp", self.permutation_varimp)
        R("POST", r"/99/SegmentModelsBuilders/(?P<algo>[^/]+)", self.segment_models)
        R("GET", r"/3/SegmentModels/(?P<sid>[^/]+)", self.segment_models_get)
        if os.environ.get("H2OMX_ENABLE_FAULT_INJECTION") == "1":
            R("POST", r"/99/h2omx/fault", self.inject_fault)

    def _route(self, method, pattern, fn):
        self.routes.append((method, re.compile("^" + pattern + "$"), fn))

    # -- dispatch -------------------------------------------------------------
    def handle(self, method: str, path: str, params: dict, body: bytes = b"", headers=None):
        """Returns (status, content_type, payload bytes|dict)."""
        self.counters["requests"] += 1
        t0 = time.time()
        path = path.rstrip("/") or "/"
        if path.endswith(".json"):
            path = path[:-5]
        for m, rx, fn in self.routes:
            if m != method and not (method == "HEAD" and m == "GET"):
                continue
            mt = rx.match(path)
            if mt:
                try:
                    out = fn(params=params, body=body, headers=headers or {}, **mt.groupdict())
                    status, ctype, payload = (200, "application/json", out) if not isinstance(out, tuple) else out
                except ApiError as e:
                    status, ctype, payload = e.status, "application/json", _error_json(e.status, e.msg, e.exc_type,
                                                                                      path)
                except KeyError as e:
                    status, ctype, payload = 404, "application/json", _error_json(404, f"Object not found: {e}",
                                                                                 "H2OKeyNotFoundArgumentException",
                                                                                 path)
                except Exception as e:  # noqa: BLE001
                    log.exception("request %s %s failed", method, path)
                    status, ctype, payload = 500, "application/json", _error_json(500, f"{type(e).__name__}: {e}",
                                                                                 type(e).__name__, path)
                self.timeline.append({"method": method, "path": path, "status": status,
                                      "ms": round((time.time() - t0) * 1000, 3)})
                if len(self.timeline) > 1000:
                    del self.timeline[:200]
                return status, ctype, payload
        return 404, "application/json", _error_json(404, f"Resource {path} not found", "H2ONotFoundArgumentException",
                                                    path)

    # -- cloud / session ------------------------------------------------------
    def _node_infos(self):
        import torch

        infos = []
        for r in range(self.cluster.world_size):
            ent = {"__meta": S.meta("NodeV3", "Iced"), "h2o": f"rank{r}", "ip_port": f"rank{r}:54321",
                   "healthy": self.peer_lost is None, "last_ping": int(time.time() * 1000),
                   "pid": os.getpid() if r == 0 else -1,
                   "num_cpus": os.cpu_count() or 1, "cpus_allowed": os.cpu_count() or 1, "nthreads": 16,
                   "sys_load": 0.0, "my_cpu_pct": -1, "sys_cpu_pct": -1, "mem_value_size": 0, "pojo_mem": 0,
                   "free_mem": 0, "max_mem": 0, "swap_mem": 0, "num_keys": len(DKV.keys()), "free_disk": 0,
                   "max_disk": 0, "rpcs_active": 0, "fjthrds": [], "fjqueue": [], "tcps_active": 0,
                   "open_fds": -1, "gflops": 0.0, "mem_bw": 0.0}
            if self.cluster.comm.device.type == "cuda" and r == self.cluster.rank:
                p = torch.cuda.get_device_properties(self.cluster.comm.device)
                ent["gpu"] = {"name": p.name, "total_memory": p.total_memory,
                              "multi_processor_count": p.multi_processor_count}
                ent["max_mem"] = p.total_memory
            infos.append(ent)
        return infos

    def _on_peer_lost(self, reason: str) -> None:
        self.peer_lost = reason
        self.jobs.fail_running(reason)

    def cloud(self, **_):
        out = S.cloud_json(self.cluster, self.started_ms, self._node_infos())
        if self.peer_lost is not None:
            out["cloud_healthy"] = False
            out["bad_nodes"] = max(1, int(out.get("bad_nodes") or 0))
        return out

    def about(self, **_):
        import torch

        from .. import __version__

        ents = [("Build git branch", "h2omx"), ("Build project version", S.H2O_VERSION),
                ("h2omx version", __version__), ("Built by", "h2omx"), ("PyTorch", torch.__version__),
                ("Backend", "ROCm/HIP gfx950 + RCCL" if torch.cuda.is_available() else "CPU")]
        return {"__meta": S.meta("AboutV3", "Iced"), "entries": [{"name": a, "value": b} for a, b in ents]}

    def capabilities(self, **_):
        from ..models import ESTIMATORS

        caps = [{"name": a} for a in list(ESTIMATORS) + ["stackedensemble", "automl"]]
        return {"__meta": S.meta("CapabilitiesV3", "Iced"), "capabilities": caps}

    def endpoints(self, **_):
        rs = [{"http_method": m, "url_pattern": rx.pattern.strip("^$"), "handler_method": fn.__name__}
              for m, rx, fn in self.routes]
        return {"__meta": S.meta("MetadataV3", "Iced"), "routes": rs}

    def init_id(self, **_):
        sid = f"_sid_{uuid.uuid4().hex[:8]}"
        self.sessions[sid] = time.time()
        return {"__meta": S.meta("InitIDV3", "Iced"), "session_key": sid}

    def new_session(self, **_):
        sid = f"_sid_{uuid.uuid4().hex[:8]}"
        self.sessions[sid] = time.time()
        return {"__meta": S.meta("SessionIdV4", "Iced", 4), "session_key": sid}

    def end_session(self, sid, **_):
        self.sessions.pop(sid, None)
        return {"__meta": S.meta("SessionIdV4", "Iced", 4), "session_key": sid}

    # -- data import ----------------------------------------------------------
    def import_files(self, params, **_):
        path = params.get("path")
        if not path:
            raise ApiError(400, "path is required")
        return self._import_paths([path])

    def import_files_multi(self, params, **_):
        return self._import_paths(parse_list(params.get("paths")))

    def _import_paths(self, paths):
        files, fails = [], []
        for p in paths:
            p2 = p[len("file://"):] if p.startswith("file://") else p
            if os.path.isdir(p2):
                for f in sorted(os.listdir(p2)):
                    if not f.startswith("."):
                        files.append(os.path.join(p2, f))
            elif os.path.exists(p2):
                files.append(p2)
            else:
                fails.append(p)
        if not files and fails:
            raise ApiError(400, f"File {fails[0]} does not exist")
        return {"__meta": S.meta("ImportFilesV3", "Iced"), "path": paths[0] if paths else None, "files": files,
                "destination_frames": files, "fails": fails, "dels": []}

    def post_file(self, params, body, headers, **_):
        from ..runtime.ops import put_blob

        dest = params.get("destination_frame") or f"upload_{uuid.uuid4().hex[:10]}"
        data = _multipart_payload(body, headers)
        put_blob(self.cluster, dest, data)
        return {"__meta": S.meta("PostFileV3", "Iced"), "destination_frame": dest, "total_bytes": len(data)}

    def _source(self, src: str):
        from ..runtime.ops import _BLOBS

        return ("blob", src) if src in _BLOBS else ("file", src)

    def parse_setup(self, params, **_):
        from ..runtime.ops import blob_setup

        srcs = parse_list(params.get("source_frames"))
        if not srcs:
            raise ApiError(400, "source_frames is required")
        sep = params.get("separator")
        sep_c = chr(int(sep)) if sep not in (None, "", "null") and str(sep).lstrip("-").isdigit() and int(sep) > 0 else None
        hdr = params.get("check_header")
        header = None if hdr in (None, "", "0") else (str(hdr) == "1")
        first = srcs[0]
        if os.path.isdir(first):
            first = os.path.join(first, sorted(f for f in os.listdir(first) if not f.startswith("."))[0])
        st = blob_setup(self.cluster, first, sep_c, header)
        types = ["Enum" if t == "Enum" else "Numeric" for t in st["column_types"]]
        base = os.path.basename(srcs[0].rstrip("/"))
        dest = re.sub(r"[^A-Za-z0-9_]", "_", os.path.splitext(base)[0]) + ".hex"
        return {"__meta": S.meta("ParseSetupV3", "Iced"),
                "source_frames": [S.key_ref(s, "Key<Frame>") for s in srcs],
                "parse_type": "CSV", "separator": st["separator"], "single_quotes": False,
                "check_header": st["check_header"], "number_columns": st["number_columns"],
                "column_names": st["column_names"], "column_types": types, "na_strings": None,
                "destination_frame": dest, "header_lines": 1 if st["check_header"] == 1 else 0,
                "chunk_size": 4194304, "total_filtered_column_count": st["number_columns"],
                "data": None, "warnings": [], "skipped_columns": None}

    def parse(self, params, **_):
        srcs = parse_list(params.get("source_frames"))
        if not srcs:
            raise ApiError(400, "source_frames is required")
        dest = params.get("destination_frame") or (os.path.splitext(os.path.basename(srcs[0]))[0] + ".hex")
        sep = params.get("separator")
        sep_c = chr(int(sep)) if sep not in (None, "", "null") and str(sep).lstrip("-").isdigit() and int(sep) > 0 else None
        hdr = params.get("check_header")
        header = None if hdr in (None, "", "0") else (str(hdr) == "1")
        ctypes_ = parse_list(params.get("column_types")) or None
        cnames = parse_list(params.get("column_names")) or None
        types = None
        if ctypes_:
            types = ["enum" if str(t).lower() in ("enum", "categorical", "factor") else
                     ("string" if str(t).lower() == "string" else "numeric") for t in ctypes_]
        cl = self.cluster
        blobs = [s for s in srcs if self._source(s)[0] == "blob"]

        def work(job):
            if blobs:
                res = cl.run("parse_blob", blob_key=blobs[0], dest=dest, sep=sep_c, header=header, col_types=types,
                             col_names=cnames)
            else:
                res = cl.run("import_files", paths=srcs, dest=dest, sep=sep_c, header=header, col_types=types,
                             col_names=cnames)
            self.counters["rows_parsed"] += res["rows"]
            return res

        blocking = str(params.get("blocking", "false")).lower() == "true"
        job = self.jobs.submit(f"Parse {', '.join(srcs)}", dest, "Key<Frame>", work, sync=blocking)
        return {"__meta": S.meta("ParseV3", "Iced"), "destination_frame": S.key_ref(dest, "Key<Frame>"),
                "job": job.to_json(), "rows": 0, "vec_ids": []}

    # -- frames ---------------------------------------------------------------
    def frames(self, **_):
        out = []
        for k in DKV.keys(Frame):
            fr = DKV.get(k)
            out.append(S.frame_base_json(k, fr.nrows, fr.ncols))
        return {"__meta": S.meta("FramesListV3", "Frames"), "frames": out}

    def frame(self, fid, params, **_):
        fid = unquote(fid)
        if not isinstance(DKV.get(fid), Frame):
            raise KeyError(fid)
        n = int(params.get("row_count", 10) or 10)
        off = int(params.get("row_offset", 0) or 0)
        summ = self.cluster.run("frame_summary", key=fid)
        prev = self.cluster.run("frame_rows", key=fid, n=n, offset=off)
        return {"__meta": S.meta("FramesV3", "Frames"), "frames": [S.frame_json(fid, summ, prev, off, n)]}

    def frame_column(self, fid, col, params, **_):
        fid, col = unquote(fid), unquote(col)
        summ = self.cluster.run("frame_summary", key=fid)
        cols = [c for c in summ["columns"] if c["label"] == col]
        if not cols:
            raise KeyError(col)
        summ = dict(summ, columns=cols)
        return {"__meta": S.meta("FramesV3", "Frames"), "frames": [S.frame_json(fid, summ, None)]}

    def download_dataset(self, params, **_):
        fid = params.get("frame_id")
        csv = self.cluster.run("frame_download", key=fid)
        return 200, "text/csv", csv.encode()

    def split_frame(self, params, **_):
        fid = params.get("dataset")
        ratios = [float(x) for x in parse_list(params.get("ratios"))]
        dests = parse_list(params.get("destination_frames")) or [f"{fid}_part{i}" for i in range(len(ratios) + 1)]
        seed = int(params.get("seed", -1) or -1)
        job = self.jobs.submit("SplitFrame", dests[0], "Key<Frame>",
                               lambda j: self.cluster.run("split_frame", key=fid, ratios=ratios, dests=dests,
                                                          seed=seed), sync=True)
        return {"__meta": S.meta("SplitFrameV3", "Iced"), "key": S.key_ref(job.key, "Key<Job>"),
                "dataset": S.key_ref(fid, "Key<Frame>"), "ratios": ratios,
                "destination_frames": [S.key_ref(d, "Key<Frame>") for d in dests], "job": job.to_json()}

    # -- model building -------------------------------------------------------
    def model_builders(self, algo=None, **_):
        from ..models import ESTIMATORS

        out = {}
        for name, cls in ESTIMATORS.items():
            if algo and name != algo:
                continue
            params = [{"name": k, "default_value": _jsonable(v), "type": type(v).__name__, "label": k,
                       "level": "critical" if k in ("training_frame", "response_column") else "secondary"}
                      for k, v in {**cls.COMMON, **cls.DEFAULTS}.items()]
            can = _CAN_BUILD.get(name, ["Binomial", "Multinomial", "Regression"])
            out[name] = {"algo": name, "algo_full_name": name, "can_build": can, "visibility": "Stable",
                         "parameters": params}
        if algo and not out:
            raise ApiError(404, f"Unknown algo {algo}")
        return {"__meta": S.meta("ModelBuildersV3", "Iced"), "model_builders": out}

    def _builder_args(self, algo, params):
        from ..models import ESTIMATORS

        cls = ESTIMATORS.get(algo)
        if cls is None:
            raise ApiError(404, f"Unknown algo {algo}")
        known = {**cls.COMMON, **cls.DEFAULTS}
        args, msgs = {}, []
        tf = params.get("training_frame")
        y = params.get("response_column")
        vf = params.get("validation_frame")
        ignored = parse_list(params.get("ignored_columns"))
        skip = {"training_frame", "response_column", "validation_frame", "ignored_columns", "_exclude_fields",
                "model_id"}
        for k, v in params.items():
            if k in skip:
                continue
            kk = _REST_ALIASES.get(k, k)
            if kk not in known:
                msgs.append({"message_type": "WARN", "field_name": k,
                             "message": f"parameter {k} is not used by h2omx {algo}; ignored"})
                continue
            args[kk] = coerce(v, known[kk])
        if ignored:
            args["ignored_columns"] = ignored
        if not tf:
            raise ApiError(412, "training_frame is required")
        if not isinstance(DKV.get(tf), Frame):
            raise ApiError(404, f"training_frame {tf} not found", "H2OKeyNotFoundArgumentException")
        return args, tf, (y if y not in ("", None) else None), (vf if vf not in ("", None) else None), msgs

    def validate_params(self, algo, params, **_):
        _, _, _, _, msgs = self._builder_args(algo, params)
        return {"__meta": S.meta("ModelParametersSchemaV3", "Iced"), "messages": msgs, "error_count": 0}

    def build_model(self, algo, params, **_):
        if algo == "generic":
            return self._build_generic(params)
        args, tf, y, vf, msgs = self._builder_args(algo, params)
        model_id = params.get("model_id") or f"{algo.upper()}_model_h2omx_{uuid.uuid4().hex[:10]}"
        fr = DKV.get(tf)
        ign = set(args.pop("ignored_columns", []) or [])
        skip = {y, args.get("weights_column"), args.get("fold_column"), args.get("offset_column")}
        x = [c for c in fr.names if c not in ign and c not in skip]

        def work(job):
            mid = self.cluster.run("train", algo=algo, params=args, x=x, y=y, training_frame=tf,
                                   validation_frame=vf, model_id=model_id)
            self.counters["models_built"] += 1
            # deviations from H2O's semantics the builder reported (model.warnings)
            job.warnings.extend(getattr(DKV.get(mid), "warnings", None) or [])
            return mid

        blocking = str(params.get("_blocking", "false")).lower() == "true"
        job = self.jobs.submit(f"{algo} model build", model_id, "Key<Model>", work, sync=blocking)
        return {"__meta": S.meta(f"{algo.upper()}V3", "ModelBuilder"), "algo": algo, "job": job.to_json(),
                "messages": msgs, "error_count": 0, "parameters": {k: _jsonable(v) for k, v in args.items()}}

    def _build_generic(self, params):
        """POST /3/ModelBuilders/generic: import a MOJO from ``path`` or an
        uploaded / imported file key (``model_key``) on every rank."""
        src = params.get("path") or params.get("model_key")
        if not src:
            raise ApiError(412, "generic: path or model_key is required")
        src = src.get("name") if isinstance(src, dict) else str(src)
        model_id = params.get("model_id") or f"Generic_model_h2omx_{uuid.uuid4().hex[:10]}"

        def work(job):
            mid = self.cluster.run("train", algo="generic", params={"path": src}, model_id=model_id)
            self.counters["models_built"] += 1
            return mid

        job = self.jobs.submit("generic model import", model_id, "Key<Model>", work, sync=True)
        return {"__meta": S.meta("GenericV3", "ModelBuilder"), "algo": "generic", "job": job.to_json(),
                "messages": [], "error_count": 0, "parameters": {"path": src}}

    # -- grid search ------------------------------------------------------------
    def grid_build(self, algo, params, **_):
        """POST /99/Grid/{algo}: model parameters plus ``hyper_parameters`` (JSON
        map of lists), ``search_criteria`` (JSON) and ``grid_id``."""
        from ..models import ESTIMATORS

        params = dict(params)
        hp_raw = params.pop("hyper_parameters", None)
        sc_raw = params.pop("search_criteria", None)
        grid_id = params.pop("grid_id", None) or f"Grid_{algo.upper()}_{uuid.uuid4().hex[:8]}"
        hp = _json_arg(hp_raw) or {}
        sc = _json_arg(sc_raw) or {}
        if not isinstance(hp, dict) or not hp:
            raise ApiError(412, "hyper_parameters must be a non-empty map of parameter -> list of values")
        args, tf, y, vf, msgs = self._builder_args(algo, params)
        known = {**ESTIMATORS[algo].COMMON, **ESTIMATORS[algo].DEFAULTS}
        hyper = {}
        for k, vals in hp.items():
            kk = _REST_ALIASES.get(k, k)
            if kk not in known:
                raise ApiError(412, f"hyper parameter {k} is not a parameter of {algo}")
            vals = vals if isinstance(vals, list) else [vals]
            hyper[kk] = [coerce(v, known[kk]) for v in vals]
        fr = DKV.get(tf)
        ign = set(args.pop("ignored_columns", []) or [])
        skip = {y, args.get("weights_column"), args.get("fold_column"), args.get("offset_column")}
        x = [c for c in fr.names if c not in ign and c not in skip]

        def work(job):
            res = self.cluster.run("grid", algo=algo, params=args, hyper_params=hyper, search_criteria=sc, x=x, y=y,
                                   training_frame=tf, validation_frame=vf, grid_id=grid_id)
            self.grid_results[grid_id] = res
            self.counters["models_built"] += len(res.get("model_ids", []))
            return res

        job = self.jobs.submit(f"{algo} grid search", grid_id, "Key<Grid>", work)
        return {"__meta": S.meta(f"{algo.upper()}GridSearchV99", "Grid", 99), "job": job.to_json(),
                "messages": msgs, "hyper_parameters": _jsonable(hyper), "search_criteria": sc}

    def grids(self, **_):
        return {"__meta": S.meta("GridsV99", "Grids", 99),
                "grids": [self._grid_json(g, r) for g, r in self.grid_results.items()]}

    def grid_get(self, gid, params=None, **_):
        gid = unquote(gid)
        res = self.grid_results.get(gid)
        if res is None:
            raise KeyError(gid)
        params = params or {}
        sort_by = params.get("sort_by")
        dec = params.get("decreasing")
        if sort_by:
            res = self.cluster.run("grid_sorted", grid_id=gid, sort_by=sort_by,
                                   decreasing=None if dec in (None, "") else str(dec).lower() == "true")
        return self._grid_json(gid, res)

    @staticmethod
    def _grid_json(gid, res):
        rows = res.get("summary_table") or []
        cols = list(rows[0].keys()) if rows else ["model_ids"]
        table = S.two_dim_table("Hyper-Parameter Search Summary", cols,
                                ["string" if c == "model_ids" else "double" for c in cols],
                                [[r.get(c) for c in cols] for r in rows])
        return {"__meta": S.meta("GridSchemaV99", "Grid", 99), **{k: v for k, v in res.items() if k != "summary_table"},
                "summary_table": table}

    # -- jobs -----------------------------------------------------------------
    def jobs_list(self, **_):
        return {"__meta": S.meta("JobsV3", "Iced"), "jobs": [j.to_json() for j in self.jobs.all()]}

    def job(self, jid, **_):
        j = self.jobs.get(unquote(jid))
        if j is None:
            raise KeyError(jid)
        return {"__meta": S.meta("JobsV3", "Iced"), "jobs": [j.to_json()]}

    def job_cancel(self, jid, **_):
        if not self.jobs.cancel(unquote(jid)):
            raise KeyError(jid)
        return {"__meta": S.meta("JobsV3", "Iced"), "jobs": [self.jobs.get(unquote(jid)).to_json()]}

    # -- models ---------------------------------------------------------------
    def models(self, **_):
        from ..models.base import Model

        out = []
        for k in DKV.keys(Model):
            m = DKV.get(k)
            out.append({"model_id": S.key_ref(k, "Key<Model>"), "algo": m.algo,
                        "response_column_name": m.y})
        return {"__meta": S.meta("ModelsV3", "Models"), "models": out}

    def _get_model(self, mid):
        from ..models.base import Model

        m = DKV.get(unquote(mid))
        if not isinstance(m, Model):
            raise KeyError(mid)
        return m

    def model(self, mid, **_):
        return {"__meta": S.meta("ModelsV3", "Models"), "models": [S.model_json(self._get_model(mid))]}

    def mojo(self, mid, **_):
        from ..mojo import mojo_bytes

        m = self._get_model(mid)
        return 200, "application/zip", mojo_bytes(m)

    def save_model(self, mid, params, **_):
        path = params.get("dir") or params.get("path") or "."
        m = self._get_model(mid)
        target = path if path.endswith(".zip") else os.path.join(path, m.model_id + ".zip")
        os.makedirs(os.path.dirname(os.path.abspath(target)), exist_ok=True)
        out = self.cluster.run("save_model", model=m.model_id, path=target)
        return {"__meta": S.meta("ModelExportV3", "Iced"), "dir": out, "model_id": S.key_ref(m.model_id, "Key<Model>")}

    def upload_model(self, mid, params, body, headers, **_):
        import tempfile

        data = _multipart_payload(body, headers)
        d = tempfile.mkdtemp(prefix="h2omx_model_")
        path = os.path.join(d, "model.zip")
        with open(path, "wb") as f:
            f.write(data)
        if self.cluster.world_size > 1:
            raise ApiError(400, "upload_model on multi-node clusters: use /99/Models.bin with a shared path")
        out = self.cluster.run("load_model", path=path)
        return {"__meta": S.meta("ModelsV3", "Models"), "models": [S.model_json(self._get_model(out))]}

    # -- scoring --------------------------------------------------------------
    def _predict(self, mid, fid, params):
        m = self._get_model(mid)
        fid = unquote(fid)
        if not isinstance(DKV.get(fid), Frame):
            raise KeyError(fid)
        dest = params.get("predictions_frame") or f"prediction_{uuid.uuid4().hex[:10]}"
        kind = _predict_kind(params)
        self.cluster.run("predict", model=m.model_id, frame=fid, dest=dest, kind=kind,
                         leaf_type=params.get("leaf_node_assignment_type") or "Path")
        return m, dest

    def predict(self, mid, fid, params, **_):
        m, dest = self._predict(mid, fid, params)
        mm = None
        if _predict_kind(params) != "predict":
            return {"__meta": S.meta("ModelMetricsListSchemaV3", "Iced"), "model_metrics": [],
                    "predictions_frame": S.key_ref(dest, "Key<Frame>")}
        if m.y is not None and m.y in DKV.get(unquote(fid)).names:
            mm = S.metrics_json(self.cluster.run("model_metrics", model=m.model_id, frame=unquote(fid)), m.category,
                                m.model_id, unquote(fid), m.response_domain)
        if mm is not None:
            mm["predictions"] = S.frame_base_json(dest, 0, 0)
        return {"__meta": S.meta("ModelMetricsListSchemaV3", "Iced"),
                "model_metrics": [mm] if mm else [], "predictions_frame": S.key_ref(dest, "Key<Frame>")}

    def predict_async(self, mid, fid, params, **_):
        dest = params.get("predictions_frame") or f"prediction_{uuid.uuid4().hex[:10]}"
        params = dict(params, predictions_frame=dest)
        job = self.jobs.submit("Prediction", dest, "Key<Frame>", lambda j: self._predict(mid, fid, params))
        return {"__meta": S.meta("JobV4", "Job", 4), "key": S.key_ref(job.key, "Key<Job>"), "job": job.to_json(),
                **job.to_json()}

    def model_metrics(self, mid, fid, params, **_):
        m = self._get_model(mid)
        fid = unquote(fid)
        res = self.cluster.run("model_metrics", model=m.model_id, frame=fid)
        return {"__meta": S.meta("ModelMetricsListSchemaV3", "Iced"),
                "model_metrics": [S.metrics_json(res, m.category, m.model_id, fid, m.response_domain)]}

    # -- partial dependence -------------------------------------------------------
    def partial_dependence(self, params, **_):
        mid = params.get("model_id")
        fid = params.get("frame_id")
        m = self._get_model(mid)
        if not isinstance(DKV.get(fid), Frame):
            raise KeyError(fid)
        cols = parse_list(params.get("cols")) or list(m.x)
        nbins = int(params.get("nbins", 20))
        targets = parse_list(params.get("targets")) or [None]
        dest = params.get("destination_key") or f"PartialDependence_{uuid.uuid4().hex[:10]}"

        def work(job):
            res = self.cluster.run("partial_dependence", model=m.model_id, frame=fid, cols=cols, nbins=nbins,
                                   targets=targets)
            self.pdp_results[dest] = res
            return res

        job = self.jobs.submit("PartialDependence", dest, "Key<PartialDependence>", work)
        return {"__meta": S.meta("PartialDependenceV3", "PartialDependence"), "job": job.to_json(),
                "model_id": S.key_ref(m.model_id, "Key<Model>"), "frame_id": S.key_ref(fid, "Key<Frame>"),
                "destination_key": S.key_ref(dest, "Key<PartialDependence>"), "cols": cols, "nbins": nbins}

    def partial_dependence_get(self, pid, **_):
        pid = unquote(pid)
        res = self.pdp_results.get(pid)
        if res is None:
            raise KeyError(pid)
        tables = []
        for r in res:
            col = r["column"]
            names = [col, "mean_response", "stddev_response", "std_error_mean_response"]
            tables.append(S.two_dim_table(f"PartialDependence: {col}" + (f" class {r['target']}" if r["target"]
                                                                         else ""), names,
                                          ["string" if isinstance(r["data"][0][col], str) else "double"]
                                          + ["double"] * 3 if r["data"] else ["double"] * 4,
                                          [[d[c] for c in names] for d in r["data"]]))
        return {"__meta": S.meta("PartialDependenceV3", "PartialDependence"),
                "destination_key": S.key_ref(pid, "Key<PartialDependence>"), "partial_dependence_data": tables}

    # -- AutoML ---------------------------------------------------------------
    def automl_build(self, params, body, **_):
        spec = params
        if body and body.strip().startswith(b"{"):
            spec = json.loads(body.decode())
        bc = spec.get("build_control", {}) or {}
        project = bc.get("project_name") or f"AutoML_{uuid.uuid4().hex[:8]}"
        bc["project_name"] = project
        spec["build_control"] = bc

        def work(job):
            res = self.cluster.run("automl", spec=spec)
            self.automl[project] = res
            return res

        job = self.jobs.submit(f"AutoML {project}", project, "Key<AutoML>", work)
        return {"__meta": S.meta("AutoMLBuildSpecV99", "Iced", 99), "job": job.to_json(), "build_control": bc}

    def automl_get(self, aid, **_):
        aid = unquote(aid)
        res = self.automl.get(aid)
        if res is None:
            raise KeyError(aid)
        lb = res["leaderboard"]
        return {"__meta": S.meta("AutoMLV99", "AutoML", 99), "automl_id": S.key_ref(aid, "Key<AutoML>"),
                "project_name": aid, "leader": S.key_ref(lb[0]["model_id"], "Key<Model>") if lb else None,
                "leaderboard": {"models": [S.key_ref(r["model_id"], "Key<Model>") for r in lb]},
                "leaderboard_table": _lb_table(res), "event_log_table": S.two_dim_table(
                    "Event Log", ["timestamp", "level", "stage", "message"], ["string"] * 4,
                    [[str(e.get("t")), "Info", e.get("stage", ""), e.get("msg", "")] for e in res.get("events", [])]),
                "modeling_steps": res.get("steps", [])}

    def leaderboard(self, aid, **_):
        aid = unquote(aid)
        res = self.automl.get(aid)
        if res is None:
            raise KeyError(aid)
        return {"__meta": S.meta("LeaderboardV99", "Leaderboard", 99), "project_name": aid,
                "models": [S.key_ref(r["model_id"], "Key<Model>") for r in res["leaderboard"]],
                "sort_metric": res.get("sort_metric"), "table": _lb_table(res)}

    # -- misc -----------------------------------------------------------------
    def rapids(self, params, body, **_):
        ast = params.get("ast")
        if ast is None and body:
            try:
                ast = json.loads(body.decode()).get("ast")
            except ValueError:
                pass
        if not ast:
            raise ApiError(400, "ast is required")
        res = self.cluster.run("rapids", ast=ast, session_id=params.get("session_id"))
        return {"__meta": S.meta("RapidsSchemaV3", "Iced", 99), **res}

    def delete_key(self, params, fid=None, mid=None, key=None, **_):
        k = unquote(fid or mid or key)
        if DKV.get(k) is None:
            raise KeyError(k)
        self.cluster.run("delete", key=k)
        return {"__meta": S.meta("RemoveV3", "Iced")}

    def delete_all(self, params, **_):
        retain = parse_list(params.get("retained_keys"))
        self.cluster.run("delete_all", retain=retain)
        return {"__meta": S.meta("RemoveAllV3", "Iced")}

    def shutdown(self, **_):
        if self.shutdown_cb is not None:
            threading.Timer(0.2, self.shutdown_cb).start()
        return {"__meta": S.meta("ShutdownV3", "Iced")}

    def logs(self, params, node=None, name=None, **_):
        return {"__meta": S.meta("LogsV3", "Iced"), "nodeidx": node, "name": name, "log": "\n".join(LOG_BUFFER[-2000:])}

    def timeline_get(self, **_):
        return {"__meta": S.meta("TimelineV3", "Iced"), "self": "rank0", "now": int(time.time() * 1000),
                "events": list(self.timeline[-200:])}

    # -- frame tools / word2vec / diagnostics ----------------------------------
    def frame_export(self, fid, params, **_):
        fid = unquote(fid)
        if not isinstance(DKV.get(fid), Frame):
            raise KeyError(fid)
        path = params.get("path")
        if not path:
            raise ApiError(400, "path is required")
        force = str(params.get("force", "false")).lower() == "true"
        job = self.jobs.submit("Export", fid, "Key<Frame>",
                               lambda j: self.cluster.run("frame_export", key=fid, path=path, force=force), sync=True)
        return {"__meta": S.meta("FramesV3", "Frames"), "job": job.to_json(), "path": path}

    def create_frame(self, params, **_):
        dest = params.get("dest") or f"frame_{uuid.uuid4().hex[:10]}"
        spec = {}
        casts = {"rows": int, "cols": int, "seed": int, "factors": int, "integer_range": int, "response_factors": int,
                 "real_range": float, "categorical_fraction": float, "integer_fraction": float,
                 "binary_fraction": float, "binary_ones_fraction": float, "time_fraction": float,
                 "string_fraction": float, "missing_fraction": float, "value": float}
        for k, cast in casts.items():
            if params.get(k) not in (None, ""):
                spec[k] = cast(params[k])
        for k in ("randomize", "has_response", "positive_response"):
            if params.get(k) not in (None, ""):
                spec[k] = str(params[k]).lower() == "true"
        if spec.get("seed", 0) < 0:
            spec["seed"] = int(time.time() * 1000) & 0x7FFFFFFF
        job = self.jobs.submit("CreateFrame", dest, "Key<Frame>",
                               lambda j: self.cluster.run("create_frame", dest=dest, spec=spec), sync=True)
        return {"__meta": S.meta("CreateFrameV3", "Iced"), "dest": S.key_ref(dest, "Key<Frame>"),
                "key": S.key_ref(job.key, "Key<Job>"), "job": job.to_json(), **job.to_json()}

    def interaction(self, params, **_):
        src = params.get("source_frame")
        if not isinstance(DKV.get(src), Frame):
            raise KeyError(src)
        dest = params.get("dest") or f"interaction_{uuid.uuid4().hex[:10]}"
        factors = parse_list(params.get("factor_columns"))
        factors = [int(f) if str(f).lstrip("-").isdigit() else f for f in factors]
        kw = dict(pairwise=str(params.get("pairwise", "false")).lower() == "true",
                  max_factors=int(params.get("max_factors", 100)), min_occurrence=int(params.get("min_occurrence", 1)))
        job = self.jobs.submit("Interaction", dest, "Key<Frame>",
                               lambda j: self.cluster.run("interaction", source=src, dest=dest, factors=factors, **kw),
                               sync=True)
        return {"__meta": S.meta("InteractionV3", "Iced"), "dest": S.key_ref(dest, "Key<Frame>"),
                "key": S.key_ref(job.key, "Key<Job>"), "job": job.to_json(), **job.to_json()}

    def missing_inserter(self, params, **_):
        fid = params.get("dataset")
        if not isinstance(DKV.get(fid), Frame):
            raise KeyError(fid)
        frac = float(params.get("fraction", 0.1))
        seed = int(params.get("seed", -1) or -1)
        job = self.jobs.submit("MissingInserter", fid, "Key<Frame>",
                               lambda j: self.cluster.run("insert_missing", key=fid, fraction=frac, seed=seed),
                               sync=True)
        return {"__meta": S.meta("MissingInserterV3", "Iced"), "dataset": S.key_ref(fid, "Key<Frame>"),
                "key": S.key_ref(job.key, "Key<Job>"), "job": job.to_json(), **job.to_json()}

    def w2v_synonyms(self, params, **_):
        m = self._get_model(params.get("model"))
        syn = self.cluster.run("w2v_synonyms", model=m.model_id, word=params.get("word"),
                               count=int(params.get("count", 20)))
        return {"__meta": S.meta("Word2VecSynonymsV3", "Iced"), "model": S.key_ref(m.model_id, "Key<Model>"),
                "word": params.get("word"), "count": int(params.get("count", 20)),
                "synonyms": list(syn.keys()), "scores": list(syn.values())}

    def w2v_transform(self, params, **_):
        m = self._get_model(params.get("model"))
        fid = params.get("words_frame")
        if not isinstance(DKV.get(fid), Frame):
            raise KeyError(fid)
        dest = f"w2v_transform_{uuid.uuid4().hex[:10]}"
        self.cluster.run("w2v_transform", model=m.model_id, frame=fid, dest=dest,
                         aggregate_method=params.get("aggregate_method", "NONE"))
        return {"__meta": S.meta("Word2VecTransformV3", "Iced"), "model": S.key_ref(m.model_id, "Key<Model>"),
                "words_frame": S.key_ref(fid, "Key<Frame>"), "vectors_frame": S.key_ref(dest, "Key<Frame>")}

    def network_test(self, **_):
        res = self.cluster.run("network_test")
        rows = [[r["bytes"], r["microseconds"], r["bus_bandwidth_GBps"]] for r in res["results"]]
        table = S.two_dim_table(f"Collective test ({res['backend']}, {res['world_size']} ranks)",
                                ["bytes", "microseconds", "bus_bandwidth_GBps"], ["long", "double", "double"], rows)
        return {"__meta": S.meta("NetworkTestV3", "Iced"), "table": table, **res}

    def typeahead_files(self, params, **_):
        src = params.get("src") or ""
        limit = int(params.get("limit", 1000) or 1000)
        d, pre = (src, "") if os.path.isdir(src) else (os.path.dirname(src) or ".", os.path.basename(src))
        try:
            names = sorted(n for n in os.listdir(d) if n.startswith(pre))
        except OSError:
            names = []
        return {"__meta": S.meta("TypeaheadV3", "Iced"), "src": src, "limit": limit,
                "matches": [os.path.join(d, n) for n in names[:limit]]}

    def garbage_collect(self, **_):
        import gc

        import torch

        gc.collect()
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        return {"__meta": S.meta("GarbageCollectV3", "Iced")}

    def jstack(self, **_):
        import sys
        import traceback

        traces = []
        for tid, frame in sys._current_frames().items():
            traces.append(f"thread {tid}\n" + "".join(traceback.format_stack(frame)))
        return {"__meta": S.meta("JStackV3", "Iced"),
                "traces": [{"node": "rank0", "time": int(time.time() * 1000), "thread_traces": traces}]}

    def model_metrics_all(self, **_):
        from ..models.base import Model

        out = []
        for k in DKV.keys(Model):
            m = DKV.get(k)
            if m.training_metrics:
                out.append(S.metrics_json(m.training_metrics, m.category, m.model_id, None, m.response_domain))
        return {"__meta": S.meta("ModelMetricsListSchemaV3", "Iced"), "model_metrics": out}

    def make_metrics(self, pf, af, params, **_):
        pf, af = unquote(pf), unquote(af)
        for k in (pf, af):
            if not isinstance(DKV.get(k), Frame):
                raise KeyError(k)
        dom = parse_list(params.get("domain")) or None
        mm = self.cluster.run("make_metrics", predictions=pf, actuals=af, domain=dom,
                              distribution=params.get("distribution"), weights=params.get("weights_frame"))
        cat = mm.pop("model_category")
        return {"__meta": S.meta("ModelMetricsMakerSchemaV3", "Iced"), "predictions_frame": S.key_ref(pf, "Key<Frame>"),
                "actuals_frame": S.key_ref(af, "Key<Frame>"),
                "model_metrics": S.metrics_json(mm, cat, None, af, dom)}

    def permutation_varimp(self, params, **_):
        m = self._get_model(params.get("model_id"))
        fid = params.get("frame_id")
        if not isinstance(DKV.get(fid), Frame):
            raise KeyError(fid)
        rows = self.cluster.run("permutation_importance", model=m.model_id, frame=fid,
                                metric=params.get("metric", "AUTO"), n_repeats=int(params.get("n_repeats", 1)),
                                seed=int(params.get("seed", -1)), features=parse_list(params.get("features")) or None)
        table = S.two_dim_table("Permutation Variable Importance",
                                ["Variable", "Relative Importance", "Scaled Importance", "Percentage"],
                                ["string", "double", "double", "double"],
                                [[r["variable"], r["relative_importance"], r["scaled_importance"], r["percentage"]]
                                 for r in rows])
        return {"__meta": S.meta("PermutationVarImpV3", "Iced"), "permutation_varimp": table}

    def segment_models(self, algo, params, **_):
        params = dict(params)
        segs = parse_list(params.pop("segment_columns", None))
        sid = params.pop("segment_models_id", None) or f"segment_models_{uuid.uuid4().hex[:8]}"
        args, tf, y, vf, msgs = self._builder_args(algo, params)
        fr = DKV.get(tf)
        ign = set(args.pop("ignored_columns", []) or [])
        x = [c for c in fr.names if c not in ign and c != y and c not in segs]

        def work(job):
            return self.cluster.run("train_segments", algo=algo, params=args, segment_columns=segs, x=x, y=y,
                                    training_frame=tf, validation_frame=vf, segment_models_id=sid)

        job = self.jobs.submit(f"{algo} segment models", sid, "Key<SegmentModels>", work, sync=True)
        return {"__meta": S.meta("SegmentModelsParametersV3", "Iced"), "job": job.to_json(),
                "segment_models_id": S.key_ref(sid, "Key<SegmentModels>"), "messages": msgs}

    def segment_models_get(self, sid, **_):
        res = DKV.get(unquote(sid))
        if not isinstance(res, dict):
            raise KeyError(sid)
        return {"__meta": S.meta("SegmentModelsV3", "Iced"), **res}

    def nps(self, **_):
        return {"__meta": S.meta("NodePersistentStorageV3", "Iced"), "entries": []}

    def log_and_echo(self, params, **_):
        log.info("client: %s", params.get("message"))
        return {"__meta": S.meta("LogAndEchoV3", "Iced"), "message": params.get("message")}

    def inject_fault(self, params, **_):
        """Test-only (H2OMX_ENABLE_FAULT_INJECTION=1): make rank ``rank`` fail a
        cluster command; the leader must report it instead of hanging."""
        self.cluster.run("fault", rank=int(params.get("rank", -1)))
        return {"__meta": S.meta("FaultV99", "Iced", 99), "ok": True}

    def prometheus(self, **_):
        comm = self.cluster.comm.stats
        lines = [
            "# TYPE h2omx_requests_total counter", f"h2omx_requests_total {self.counters['requests']}",
            "# TYPE h2omx_models_built_total counter", f"h2omx_models_built_total {self.counters['models_built']}",
            "# TYPE h2omx_rows_parsed_total counter", f"h2omx_rows_parsed_total {self.counters['rows_parsed']}",
            "# TYPE h2omx_cloud_size gauge", f"h2omx_cloud_size {self.cluster.world_size}",
            "# TYPE h2omx_allreduce_calls_total counter", f"h2omx_allreduce_calls_total {comm['all_reduce_calls']}",
            "# TYPE h2omx_allreduce_bytes_total counter", f"h2omx_allreduce_bytes_total {comm['all_reduce_bytes']}",
            "# TYPE h2omx_allreduce_seconds_total counter", f"h2omx_allreduce_seconds_total {comm['all_reduce_s']}",
            "# TYPE h2omx_allgather_calls_total counter", f"h2omx_allgather_calls_total {comm['all_gather_calls']}",
            "# TYPE h2omx_broadcast_calls_total counter", f"h2omx_broadcast_calls_total {comm['broadcast_calls']}",
            "# TYPE h2omx_dkv_keys gauge", f"h2omx_dkv_keys {len(DKV.keys())}",
        ]
        try:
            import torch

            if torch.cuda.is_available():
                lines += ["# TYPE h2omx_gpu_memory_allocated_bytes gauge",
                          f"h2omx_gpu_memory_allocated_bytes {torch.cuda.memory_allocated()}"]
        except Exception:  # noqa: BLE001
            pass
        return 200, "text/plain; version=0.0.4", ("\n".join(lines) + "\n").encode()


def _lb_table(res):
    lb = res["leaderboard"]
    if not lb:
        return None
    cols = list(lb[0].keys())
    return S.two_dim_table("Leaderboard", cols, ["string" if c in ("model_id", "algo") else "double" for c in cols],
                           [[r[c] for c in cols] for r in lb])


def _json_arg(v):
    """A JSON-valued REST argument (h2o-py sends maps as JSON or Python-literal text)."""
    if v is None or isinstance(v, (dict, list)):
        return v
    txt = v.decode() if isinstance(v, bytes) else str(v)
    if not txt.strip():
        return None
    try:
        return json.loads(txt)
    except ValueError:
        import ast

        return ast.literal_eval(txt)


def _jsonable(v):
    if isinstance(v, float) and not math.isfinite(v):
        return str(v)
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return float(v)
    if isinstance(v, Frame):
        return v.key
    return v


def _error_json(status, msg, exc_type, path):
    return {"__meta": S.meta("H2OErrorV3", "H2OError"), "timestamp": int(time.time() * 1000),
            "error_url": path, "msg": msg, "dev_msg": msg, "http_status": status, "values": {},
            "exception_type": exc_type, "exception_msg": msg, "stacktrace": []}


def _multipart_payload(body: bytes, headers) -> bytes:
    ctype = ""
    for k, v in (headers or {}).items():
        if k.lower() == "content-type":
            ctype = v
    m = re.search(r"boundary=\"?([^\";]+)\"?", ctype)
    if not m:
        return body
    boundary = ("--" + m.group(1)).encode()
    for part in body.split(boundary):
        if b"\r\n\r\n" not in part:
            continue
        head, data = part.split(b"\r\n\r\n", 1)
        if b"filename" in head or b"name=\"file\"" in head or b"Content-Type" in head:
            return data[:-2] if data.endswith(b"\r\n") else data
    return body


# ---------------------------------------------------------------------------
# HTTP transport
# ---------------------------------------------------------------------------
class _Handler(BaseHTTPRequestHandler):
    api: H2OApi = None
    context_path: str = ""
    protocol_version = "HTTP/1.1"

    def log_message(self, fmt, *args):  # route access logs into the node log
        log.debug("http: " + fmt, *args)

    def _do(self, method):
        u = urlparse(self.path)
        path = u.path
        cp = self.context_path
        if cp and path.startswith(cp):
            path = path[len(cp):] or "/"
        params = {k: v[-1] for k, v in parse_qs(u.query, keep_blank_values=True).items()}
        n = int(self.headers.get("Content-Length") or 0)
        body = self.rfile.read(n) if n else b""
        ctype = self.headers.get("Content-Type", "")
        if body and "application/x-www-form-urlencoded" in ctype:
            params.update({k: v[-1] for k, v in parse_qs(body.decode(), keep_blank_values=True).items()})
        elif body and "application/json" in ctype:
            try:
                js = json.loads(body.decode())
                if isinstance(js, dict):
                    params.update({k: (v if isinstance(v, str) else json.dumps(v)) for k, v in js.items()})
            except ValueError:
                pass
        status, ctype_out, payload = self.api.handle(method, path, params, body, dict(self.headers))
        data = payload if isinstance(payload, (bytes, bytearray)) else json.dumps(payload, default=_json_default).encode()
        self.send_response(status)
        self.send_header("Content-Type", ctype_out)
        self.send_header("Content-Length", str(len(data)))
        if ctype_out == "application/zip":
            self.send_header("Content-Disposition", "attachment; filename=model.zip")
        self.end_headers()
        if method != "HEAD":
            self.wfile.write(data)

    def do_GET(self):
        self._do("GET")

    def do_POST(self):
        self._do("POST")

    def do_DELETE(self):
        self._do("DELETE")

    def do_HEAD(self):
        self._do("HEAD")


def _json_default(o):
    if isinstance(o, (np.integer,)):
        return int(o)
    if isinstance(o, (np.floating,)):
        f = float(o)
        return f if math.isfinite(f) else str(f)
    if isinstance(o, np.ndarray):
        return o.tolist()
    if isinstance(o, Frame):
        return o.key
    return str(o)


def serve(api: H2OApi, host: str = "0.0.0.0", port: int = 54321, context_path: str = "") -> ThreadingHTTPServer:
    handler = type("H2OHandler", (_Handler,), {"api": api, "context_path": context_path.rstrip("/")})
    srv = ThreadingHTTPServer((host, port), handler)
    srv.daemon_threads = True
    t = threading.Thread(target=srv.serve_forever, name="h2o-rest", daemon=True)
    t.start()
    return srv


def mojo_zip_names(data: bytes) -> list[str]:
    return zipfile.ZipFile(io.BytesIO(data)).namelist()
