"""In-process fake Kubernetes API server for control-plane tests.

The reference tested `h2ok` only against a live K3s cluster
(.github/workflows/rust.yml:18-25 of isgasho/h2o-kubernetes).  There is no
cluster (or network) here, so this fixture implements the slice of the API
the control plane uses: create / get / list (label + field selectors) /
replace / merge-patch (incl. the status subresource) / delete and chunked
watch streams for services, statefulsets, pods, ingresses (v1, v1beta1) and
the h2o.ai/v1beta `H2O` custom resource.  Optional TLS and bearer-token auth,
fault injection, and a load balancer that assigns an ingress IP shortly after
creation (so `h2ok ingress` exercises its watch loop).

Authorisation (optional, ``rbac_rules``): every request is checked against a
list of ClusterRole rules (``{apiGroups, resources, verbs}``, the rules of
``deploy/operator.yaml`` via :func:`cluster_role_rules`) the way the real
apiserver's RBAC authoriser does - verb from the method (get / list / watch /
create / update / patch / delete), resource incl. the ``status``
subresource - and answered 403 Forbidden outside them.  Authorisation runs
before routing, as on a real apiserver, so a forbidden request to an API group
the cluster does not serve is 403, an allowed one 404.  ``served_groups``
(None = every group) lists the API groups the cluster serves: a K3s cluster
with its bundled Traefik serves ``traefik.io`` / ``traefik.containo.us``, a
plain kind cluster does not.

Deletion follows the real apiserver's propagation semantics: with
``propagationPolicy: Foreground`` the object stays (``deletionTimestamp`` +
``foregroundDeletion`` finalizer, MODIFIED event) until its dependents are
gone, for ``foreground_delay`` seconds here; a create of the same name in
that window answers 409 AlreadyExists.  Background / orphan deletes remove
the object at once.
"""
from __future__ import annotations

import copy
import json
import re
import ssl
import subprocess
import threading
import time
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlparse

_PATH = re.compile(
    r"^/(?:api/(?P<core>v1)|apis/(?P<group>[^/]+)/(?P<version>[^/]+))"
    r"(?:/namespaces/(?P<ns>[^/]+))?/(?P<plural>[^/]+)(?:/(?P<name>[^/]+))?(?:/(?P<sub>status))?$")


class FakeK8s:
    def __init__(self, token: str | None = None, tls: bool = False, tmpdir: str | None = None,
                 ingress_ip_delay: float = 0.3, foreground_delay: float = 0.5,
                 rbac_rules: list[dict] | None = None, served_groups: set[str] | None = None):
        self.objects: dict[tuple, dict] = {}
        self.rbac_rules = rbac_rules
        self.served_groups = served_groups
        self.forbidden: list[tuple[str, str, str]] = []   # (verb, group, resource) answered 403
        self.rv = 100
        self.lock = threading.Condition()
        self.events: list[tuple[int, tuple, str, dict]] = []
        self.token = token
        self.fail: dict[tuple[str, str], int] = {}   # (METHOD, plural) -> status
        self.requests: list[tuple[str, str]] = []
        self.ingress_ip_delay = ingress_ip_delay
        self.foreground_delay = foreground_delay
        self.tls = tls
        self.tmpdir = tmpdir
        # StatefulSet controller + kubelet stand-in (tests/fake_kubelet.py): runs the
        # rendered pod containers as local processes; None = canned pods only
        self.kubelet = None
        self.ca_pem = None
        self.httpd = ThreadingHTTPServer(("127.0.0.1", 0), self._handler())
        self.httpd.daemon_threads = True
        if tls:
            self._setup_tls()
        self.port = self.httpd.server_address[1]
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True)

    # -- lifecycle -------------------------------------------------------
    def start(self):
        self.thread.start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()

    @property
    def url(self) -> str:
        return f"{'https' if self.tls else 'http'}://127.0.0.1:{self.port}"

    def _setup_tls(self):
        import os

        d = self.tmpdir
        key, crt = os.path.join(d, "srv.key"), os.path.join(d, "srv.crt")
        subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", key, "-out", crt,
                        "-days", "2", "-subj", "/CN=127.0.0.1", "-addext", "subjectAltName=IP:127.0.0.1"],
                       check=True, capture_output=True)
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.load_cert_chain(crt, key)
        self.httpd.socket = ctx.wrap_socket(self.httpd.socket, server_side=True)
        self.ca_pem = open(crt).read()

    def kubeconfig(self, path: str, namespace: str = "default", token: str | None = None) -> str:
        import base64

        cluster = {"server": self.url}
        if self.tls:
            cluster["certificate-authority-data"] = base64.b64encode(self.ca_pem.encode()).decode()
        user = {"token": token or self.token} if (token or self.token) else {}
        lines = [
            "apiVersion: v1",
            "kind: Config",
            "# written by tests/fake_k8s.py",
            "clusters:",
            "- cluster:",
        ] + [f"    {k}: {v}" for k, v in cluster.items()] + [
            "  name: fake",
            "contexts:",
            "- context:",
            "    cluster: fake",
            "    user: tester",
            f"    namespace: {namespace}",
            "  name: fake-ctx",
            "current-context: fake-ctx",
            "preferences: {}",
            "users:",
            "- name: tester",
            "  user:" + ("" if user else " {}"),
        ] + [f"    {k}: {v}" for k, v in user.items()]
        with open(path, "w") as f:
            f.write("\n".join(lines) + "\n")
        return path

    # -- store helpers ---------------------------------------------------
    def list(self, plural: str, ns: str | None = None):
        with self.lock:
            return [copy.deepcopy(o) for (p, n, _), o in sorted(self.objects.items())
                    if p == plural and (ns is None or n == ns)]

    def get(self, plural: str, ns: str, name: str):
        with self.lock:
            o = self.objects.get((plural, ns, name))
            return copy.deepcopy(o) if o else None

    def put(self, plural: str, ns: str, obj: dict, event: str = "ADDED"):
        with self.lock:
            self.rv += 1
            md = obj.setdefault("metadata", {})
            md.setdefault("namespace", ns)
            md.setdefault("uid", str(uuid.uuid4()))
            md.setdefault("creationTimestamp", time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()))
            md["resourceVersion"] = str(self.rv)
            md.setdefault("generation", 1)
            self.objects[(plural, ns, md["name"])] = obj
            self.events.append((self.rv, (plural, ns), event, copy.deepcopy(obj)))
            self.lock.notify_all()
            return copy.deepcopy(obj)

    def delete(self, plural: str, ns: str, name: str):
        with self.lock:
            o = self.objects.pop((plural, ns, name), None)
            if o is None:
                return None
            self.rv += 1
            o["metadata"]["resourceVersion"] = str(self.rv)
            self.events.append((self.rv, (plural, ns), "DELETED", copy.deepcopy(o)))
            self.lock.notify_all()
            # garbage-collect dependents (ownerReferences), like the real GC
            uid = o["metadata"].get("uid")
            for key, dep in list(self.objects.items()):
                refs = dep.get("metadata", {}).get("ownerReferences", [])
                if any(r.get("uid") == uid for r in refs):
                    self.objects.pop(key, None)
            return o

    # -- HTTP --------------------------------------------------------------
    def _handler(self):
        fake = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def _send(self, status: int, body: dict | None):
                data = json.dumps(body or {}).encode()
                self.send_response(status)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(data)))
                self.send_header("Connection", "close")
                self.end_headers()
                self.wfile.write(data)
                self.close_connection = True

            def _status(self, code: int, reason: str, msg: str):
                self._send(code, {"kind": "Status", "apiVersion": "v1", "status": "Failure", "reason": reason,
                                  "message": msg, "code": code})

            def _body(self):
                n = int(self.headers.get("Content-Length") or 0)
                raw = self.rfile.read(n) if n else b""
                return json.loads(raw) if raw else {}

            def _route(self, method):
                u = urlparse(self.path)
                fake.requests.append((method, u.path))
                if fake.token and self.headers.get("Authorization") != f"Bearer {fake.token}":
                    return self._status(401, "Unauthorized", "bad token")
                m = _PATH.match(u.path)
                if not m:
                    return self._status(404, "NotFound", f"no route {u.path}")
                plural, ns, name, sub = m["plural"], m["ns"], m["name"], m["sub"]
                q = parse_qs(u.query)
                group = m["group"] or ""
                if fake.rbac_rules is not None:
                    verb = _verb(method, name, q)
                    resource = plural + ("/status" if sub else "")
                    if not _allowed(fake.rbac_rules, verb, group, resource):
                        fake.forbidden.append((verb, group, resource))
                        gr = f"{resource}.{group}" if group else resource
                        return self._status(403, "Forbidden",
                                            f'{gr} "{name or ""}" is forbidden: User "system:serviceaccount:'
                                            f'h2omx-system:h2omx-operator" cannot {verb} resource "{resource}" in '
                                            f'API group "{group}"')
                if fake.served_groups is not None and group and group not in fake.served_groups:
                    return self._status(404, "NotFound", f"the server could not find the requested resource "
                                                         f"({group})")
                inj = fake.fail.get((method, plural))
                if inj:
                    return self._status(inj, "InternalError", f"injected failure for {method} {plural}")
                if method == "GET" and name is None and q.get("watch", ["0"])[0] in ("1", "true"):
                    return self._watch(plural, ns, q)
                if method == "POST":
                    body = self._body()
                    nm = body.get("metadata", {}).get("name")
                    nsp = ns or body.get("metadata", {}).get("namespace") or "default"
                    if fake.get(plural, nsp, nm):
                        return self._status(409, "AlreadyExists", f'{plural} "{nm}" already exists')
                    obj = fake.put(plural, nsp, body)
                    if plural == "ingresses":
                        threading.Timer(fake.ingress_ip_delay, fake._assign_ip, args=(nsp, nm)).start()
                    if plural == "statefulsets":
                        fake._spawn_pods(obj)
                    return self._send(201, obj)
                if method == "GET":
                    if name:
                        o = fake.get(plural, ns, name)
                        return self._send(200, o) if o else self._status(404, "NotFound", f'"{name}" not found')
                    items = fake.list(plural, ns)
                    for sel in q.get("labelSelector", []):
                        for term in sel.split(","):
                            k, v = term.split("=", 1)
                            items = [o for o in items if o["metadata"].get("labels", {}).get(k) == v]
                    for sel in q.get("fieldSelector", []):
                        k, v = sel.split("=", 1)
                        if k == "metadata.name":
                            items = [o for o in items if o["metadata"]["name"] == v]
                    return self._send(200, {"kind": "List", "apiVersion": "v1", "items": items,
                                            "metadata": {"resourceVersion": str(fake.rv)}})
                if method == "DELETE":
                    policy = (self._body() or {}).get("propagationPolicy") or ""
                    cur = fake.get(plural, ns, name)
                    if cur is None:
                        return self._status(404, "NotFound", f'"{name}" not found')
                    if cur["metadata"].get("deletionTimestamp"):
                        return self._send(200, cur)       # already terminating
                    if policy == "Foreground":
                        cur["metadata"]["deletionTimestamp"] = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
                        cur["metadata"]["finalizers"] = ["foregroundDeletion"]
                        obj = fake.put(plural, ns, cur, "MODIFIED")
                        threading.Timer(fake.foreground_delay, fake._finish_delete, args=(plural, ns, name)).start()
                        return self._send(200, obj)
                    fake._finish_delete(plural, ns, name)
                    return self._send(200, {"kind": "Status", "status": "Success"})
                if method in ("PUT", "PATCH"):
                    cur = fake.get(plural, ns, name)
                    if cur is None:
                        return self._status(404, "NotFound", f'"{name}" not found')
                    body = self._body()
                    if method == "PUT":
                        new = body
                    else:
                        new = _merge(cur, body if not sub else {"status": body.get("status", {})})
                    if method == "PATCH" and "spec" in body:
                        new["metadata"]["generation"] = cur["metadata"].get("generation", 1) + 1
                    return self._send(200, fake.put(plural, ns, new, "MODIFIED"))
                return self._status(405, "MethodNotAllowed", method)

            def _watch(self, plural, ns, q):
                timeout = float(q.get("timeoutSeconds", ["30"])[0])
                since = int(q.get("resourceVersion", ["0"])[0] or 0)
                fsel = q.get("fieldSelector", [""])[0]
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Transfer-Encoding", "chunked")
                self.end_headers()
                deadline = time.time() + timeout
                sent = since
                try:
                    while time.time() < deadline:
                        with fake.lock:
                            evs = [e for e in fake.events if e[0] > sent and e[1][0] == plural
                                   and (ns is None or e[1][1] == ns)]
                            if not evs:
                                fake.lock.wait(timeout=max(0.0, min(0.2, deadline - time.time())))
                                continue
                        for rv, _, typ, obj in evs:
                            sent = rv
                            if fsel.startswith("metadata.name=") and obj["metadata"]["name"] != fsel.split("=", 1)[1]:
                                continue
                            line = (json.dumps({"type": typ, "object": obj}) + "\n").encode()
                            self.wfile.write(b"%x\r\n%s\r\n" % (len(line), line))
                            self.wfile.flush()
                    self.wfile.write(b"0\r\n\r\n")
                    self.wfile.flush()
                except (BrokenPipeError, ConnectionResetError, ssl.SSLError, OSError):
                    pass
                self.close_connection = True

            def do_GET(self):
                self._route("GET")

            def do_POST(self):
                self._route("POST")

            def do_DELETE(self):
                self._route("DELETE")

            def do_PUT(self):
                self._route("PUT")

            def do_PATCH(self):
                self._route("PATCH")

        return H

    def _finish_delete(self, plural, ns, name):
        o = self.delete(plural, ns, name)
        if o is not None and plural == "statefulsets":
            for p in self.list("pods", ns):
                if p["metadata"].get("labels", {}).get("app") == o["metadata"].get("labels", {}).get("app"):
                    self.delete("pods", ns, p["metadata"]["name"])
        return o

    def _assign_ip(self, ns, name):
        o = self.get("ingresses", ns, name)
        if o is None:
            return
        o.setdefault("status", {})["loadBalancer"] = {"ingress": [{"ip": "10.43.0.7"}]}
        self.put("ingresses", ns, o, "MODIFIED")

    def _spawn_pods(self, sts):
        """StatefulSet controller stand-in: pods <sts>-<ordinal>, pod 0 Ready (leader)."""
        if self.kubelet is not None:
            return self.kubelet.start(self, sts)
        ns = sts["metadata"]["namespace"]
        name = sts["metadata"]["name"]
        labels = sts["spec"]["template"]["metadata"].get("labels", {})
        for i in range(int(sts["spec"].get("replicas", 1))):
            pod = {"apiVersion": "v1", "kind": "Pod",
                   "metadata": {"name": f"{name}-{i}", "labels": dict(labels)},
                   "status": {"phase": "Running",
                              "conditions": [{"type": "Ready", "status": "True" if i == 0 else "False"}]}}
            self.put("pods", ns, pod)


def _verb(method: str, name: str | None, q: dict) -> str:
    if method == "GET":
        if name:
            return "get"
        return "watch" if q.get("watch", ["0"])[0] in ("1", "true") else "list"
    return {"POST": "create", "PUT": "update", "PATCH": "patch", "DELETE": "delete"}.get(method, method.lower())


def _allowed(rules: list[dict], verb: str, group: str, resource: str) -> bool:
    for r in rules:
        groups, res, verbs = r.get("apiGroups", []), r.get("resources", []), r.get("verbs", [])
        if ("*" in groups or group in groups) and ("*" in res or resource in res) and ("*" in verbs or verb in verbs):
            return True
    return False


def cluster_role_rules(manifest: str, name: str | None = None) -> list[dict]:
    """The rules of the ClusterRole in a multi-document manifest (deploy/operator.yaml)."""
    import yaml

    with open(manifest) as f:
        for doc in yaml.safe_load_all(f):
            if doc and doc.get("kind") == "ClusterRole" and (name is None or doc["metadata"]["name"] == name):
                return doc.get("rules", [])
    raise LookupError(f"no ClusterRole in {manifest}")


def _merge(a, b):
    if not isinstance(a, dict) or not isinstance(b, dict):
        return copy.deepcopy(b)
    out = copy.deepcopy(a)
    for k, v in b.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = _merge(out.get(k), v) if isinstance(v, dict) else copy.deepcopy(v)
    return out
