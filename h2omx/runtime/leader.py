"""Kubernetes readiness endpoint of a node (reference contract:
``GET :8081/kubernetes/isLeaderNode`` returns 2xx only on the leader once the
cloud has formed, ``src/k8s/templates.rs:34-40``), so the Service routes
client traffic to the leader pod only.  Also answers ``/kubernetes/isReady``
(any node that joined the cloud) for liveness-style checks."""
from __future__ import annotations

import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer


def serve_leader_probe(cluster, host: str = "0.0.0.0", port: int | None = None) -> ThreadingHTTPServer:
    port = cluster.cfg.api_port if port is None else port

    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def _reply(self, code, body):
            data = body.encode()
            self.send_response(code)
            self.send_header("Content-Type", "text/plain")
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

        def do_GET(self):
            path = self.path.split("?")[0].rstrip("/")
            if path == "/kubernetes/isLeaderNode":
                if cluster.formed and cluster.is_leader:
                    self._reply(200, "true")
                else:
                    self._reply(404, "false")
            elif path == "/kubernetes/isReady":
                self._reply(200 if cluster.formed else 503, "true" if cluster.formed else "false")
            else:
                self._reply(404, "not found")

    srv = ThreadingHTTPServer((host, port), H)
    srv.daemon_threads = True
    threading.Thread(target=srv.serve_forever, name="leader-probe", daemon=True).start()
    return srv
