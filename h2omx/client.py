"""Minimal Python client for an h2omx (or H2O) cluster's REST API.

It issues the same requests as h2o-py for the common workflow
(``connect`` → ``import_file``/``upload_file`` → ``train`` → ``predict`` →
``download_mojo``), so the REST layer is exercised exactly as a real client
would use it; h2o-py itself is not installed in this environment.
"""
from __future__ import annotations

import json
import time
import urllib.error
import urllib.parse
import urllib.request


class H2OResponseError(RuntimeError):
    def __init__(self, status, payload):
        super().__init__(f"HTTP {status}: {payload.get('msg') if isinstance(payload, dict) else payload}")
        self.status = status
        self.payload = payload


def _fmt(v):
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(json.dumps(x) if isinstance(x, str) else _fmt(x) for x in v) + "]"
    return str(v)


class H2OConnection:
    def __init__(self, url: str = "http://127.0.0.1:54321", timeout: float = 600.0):
        self.url = url.rstrip("/")
        self.timeout = timeout
        self.session_key = None

    # -- transport --------------------------------------------------------------
    def request(self, endpoint: str, data=None, json_body=None, raw: bool = False, files=None):
        method, path = endpoint.split(" ", 1)
        url = self.url + path
        body, headers = None, {}
        if method == "GET" and data:
            url += ("&" if "?" in url else "?") + urllib.parse.urlencode({k: _fmt(v) for k, v in data.items()
                                                                           if v is not None})
        elif json_body is not None:
            body = json.dumps(json_body).encode()
            headers["Content-Type"] = "application/json"
        elif files is not None:
            boundary = "h2omxboundary7MA4YWxkTrZu0gW"
            name, content = files
            body = (f"--{boundary}\r\nContent-Disposition: form-data; name=\"file\"; filename=\"{name}\"\r\n"
                    f"Content-Type: application/octet-stream\r\n\r\n").encode() + content + \
                f"\r\n--{boundary}--\r\n".encode()
            headers["Content-Type"] = f"multipart/form-data; boundary={boundary}"
        elif data is not None:
            body = urllib.parse.urlencode({k: _fmt(v) for k, v in data.items() if v is not None}).encode()
            headers["Content-Type"] = "application/x-www-form-urlencoded"
        req = urllib.request.Request(url, data=body, method=method, headers=headers)
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as r:
                payload = r.read()
                if raw:
                    return payload
                return json.loads(payload.decode()) if payload else {}
        except urllib.error.HTTPError as e:
            p = e.read()
            try:
                p = json.loads(p.decode())
            except ValueError:
                p = p.decode(errors="replace")
            raise H2OResponseError(e.code, p) from None

    # -- h2o-py-like workflow --------------------------------------------------
    def connect(self):
        cloud = self.request("GET /3/Cloud")
        self.session_key = self.request("POST /4/sessions")["session_key"]
        return cloud

    def wait_job(self, job: dict, poll: float = 0.05) -> dict:
        key = job["key"]["name"]
        while True:
            j = self.request(f"GET /3/Jobs/{urllib.parse.quote(key, safe='')}")["jobs"][0]
            if j["status"] in ("DONE", "FAILED", "CANCELLED"):
                if j["status"] != "DONE":
                    raise RuntimeError(f"job {key} {j['status']}: {j.get('exception')}")
                return j
            time.sleep(poll)

    def import_file(self, path: str, destination_frame: str | None = None, col_types=None, header=0) -> str:
        imp = self.request("GET /3/ImportFiles", {"path": path})
        return self._parse(imp["destination_frames"], destination_frame, col_types, header)

    def upload_file(self, path: str, destination_frame: str | None = None, col_types=None, header=0) -> str:
        with open(path, "rb") as f:
            content = f.read()
        dest = destination_frame or ("upload_" + str(abs(hash(path)) % 10 ** 8))
        r = self.request(f"POST /3/PostFile?destination_frame={dest}", files=(path, content))
        return self._parse([r["destination_frame"]], destination_frame, col_types, header)

    def _parse(self, sources, dest, col_types, header):
        setup = self.request("POST /3/ParseSetup", {"source_frames": sources, "check_header": header})
        types = col_types or setup["column_types"]
        p = self.request("POST /3/Parse", {
            "destination_frame": dest or setup["destination_frame"], "source_frames": sources,
            "parse_type": setup["parse_type"], "separator": setup["separator"],
            "number_columns": setup["number_columns"], "column_names": setup["column_names"],
            "column_types": types, "check_header": setup["check_header"], "delete_on_done": True,
            "chunk_size": setup["chunk_size"]})
        self.wait_job(p["job"])
        return p["destination_frame"]["name"]

    def frame(self, key: str, rows: int = 10) -> dict:
        return self.request(f"GET /3/Frames/{urllib.parse.quote(key, safe='')}", {"row_count": rows})["frames"][0]

    def train(self, algo: str, training_frame: str, y: str | None = None, x=None, **params) -> dict:
        data = {"training_frame": training_frame}
        if y is not None:
            data["response_column"] = y
        if x is not None:
            fr = self.frame(training_frame, rows=0)
            cols = [c["label"] for c in fr["columns"]]
            data["ignored_columns"] = [c for c in cols if c not in set(x) and c != y]
        data.update(params)
        b = self.request(f"POST /3/ModelBuilders/{algo}", data)
        self.wait_job(b["job"])
        mid = b["job"]["dest"]["name"]
        return self.request(f"GET /3/Models/{mid}")["models"][0]

    def grid(self, algo: str, training_frame: str, hyper_params: dict, y: str | None = None,
             search_criteria: dict | None = None, grid_id: str | None = None, **params) -> dict:
        """Grid search (POST /99/Grid/{algo}); returns the grid (GET /99/Grids/{id})."""
        import json as _json

        data = {"training_frame": training_frame, "hyper_parameters": _json.dumps(hyper_params)}
        if y is not None:
            data["response_column"] = y
        if search_criteria:
            data["search_criteria"] = _json.dumps(search_criteria)
        if grid_id:
            data["grid_id"] = grid_id
        data.update(params)
        b = self.request(f"POST /99/Grid/{algo}", data)
        self.wait_job(b["job"])
        return self.get_grid(b["job"]["dest"]["name"])

    def get_grid(self, grid_id: str, sort_by: str | None = None, decreasing: bool | None = None) -> dict:
        q = {}
        if sort_by:
            q["sort_by"] = sort_by
        if decreasing is not None:
            q["decreasing"] = "true" if decreasing else "false"
        return self.request(f"GET /99/Grids/{grid_id}", q or None)

    def predict(self, model_id: str, frame: str) -> str:
        r = self.request(f"POST /4/Predictions/models/{model_id}/frames/{frame}")
        j = self.wait_job(r["job"])
        return j["dest"]["name"]

    def predict_contributions(self, model_id: str, frame: str) -> str:
        r = self.request(f"POST /3/Predictions/models/{model_id}/frames/{frame}", {"predict_contributions": True})
        return r["predictions_frame"]["name"]

    def partial_dependence(self, model_id: str, frame: str, cols=None, nbins: int = 20) -> list:
        data = {"model_id": model_id, "frame_id": frame, "nbins": nbins}
        if cols:
            data["cols"] = list(cols)
        r = self.request("POST /3/PartialDependence/", data)
        self.wait_job(r["job"])
        return self.request(f"GET /3/PartialDependence/{r['destination_key']['name']}")["partial_dependence_data"]

    def model_performance(self, model_id: str, frame: str) -> dict:
        return self.request(f"POST /3/ModelMetrics/models/{model_id}/frames/{frame}")["model_metrics"][0]

    def download_mojo(self, model_id: str) -> bytes:
        return self.request(f"GET /3/Models/{model_id}/mojo", raw=True)

    def rapids(self, ast: str) -> dict:
        return self.request("POST /99/Rapids", {"ast": ast, "session_id": self.session_key})

    def automl(self, training_frame: str, y: str, max_models: int = 4, seed: int = 1, nfolds: int = 3,
               project_name: str | None = None, **kw) -> dict:
        spec = {"build_control": {"project_name": project_name, "nfolds": nfolds,
                                  "stopping_criteria": {"max_models": max_models, "seed": seed}},
                "input_spec": {"training_frame": training_frame, "response_column": y},
                "build_models": kw.get("build_models", {})}
        r = self.request("POST /99/AutoMLBuilder", json_body=spec)
        self.wait_job(r["job"])
        return self.request(f"GET /99/AutoML/{r['build_control']['project_name']}")

    def remove_all(self):
        return self.request("DELETE /3/DKV")

    def shutdown(self):
        return self.request("POST /3/Shutdown")


def connect(url: str = "http://127.0.0.1:54321") -> H2OConnection:
    c = H2OConnection(url)
    c.connect()
    return c
