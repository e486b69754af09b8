"""A kubelet stand-in for end-to-end tests: runs the pods of a StatefulSet
that the operator created in tests/fake_k8s.py as local processes, from the
RENDERED pod template.

For every replica ``<sts>-<ordinal>`` it starts the container's ``command`` +
``args`` with the container's ``env`` as rendered (``valueFrom.fieldRef``
``metadata.name`` / ``metadata.namespace`` resolved like the kubelet does),
and reports the pod Ready exactly when the container's ``readinessProbe``
(httpGet) answers 2xx.  A pod has its own network namespace and DNS in a real
cluster; here all pods share localhost, so the only departures from the
rendered spec are:

* every ``containerPort`` is remapped to a free local port and the env
  variables that carry those ports (``H2O_KUBERNETES_API_PORT``,
  ``H2OMX_REST_PORT``, ``MASTER_PORT``) point at the remapped ones;
* ``MASTER_ADDR=127.0.0.1`` (the rendezvous host would otherwise be pod 0's
  DNS name under the headless service);
* the image's filesystem is this checkout (``cwd`` / ``PYTHONPATH``) and the
  GPU is hidden (the kind / CPU configuration).

Reference: the reference's CI deploys to a live K3s cluster
(``/root/reference/.github/workflows/rust.yml:18-25``,
``/root/reference/src/k8s/mod.rs:218-239``); this is the process-level
version of that, with the data plane actually running.
"""
from __future__ import annotations

import os
import socket
import subprocess
import threading
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PORT_ENV = {8081: "H2O_KUBERNETES_API_PORT", 54321: "H2OMX_REST_PORT", 29500: "MASTER_PORT"}


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class FakeKubelet:
    def __init__(self, logdir: str, extra_env: dict | None = None):
        self.logdir = logdir
        self.extra_env = extra_env or {}
        self.pods: dict[str, dict] = {}          # pod name -> {proc, ports, ns, ready}
        self._stop = threading.Event()
        self._thread = None
        self.k8s = None

    # -- StatefulSet controller --------------------------------------------------
    def start(self, k8s, sts):
        self.k8s = k8s
        ns = sts["metadata"]["namespace"]
        name = sts["metadata"]["name"]
        tmpl = sts["spec"]["template"]
        labels = dict(tmpl["metadata"].get("labels", {}))
        for i in range(int(sts["spec"].get("replicas", 1))):
            pod = f"{name}-{i}"
            k8s.put("pods", ns, {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": pod, "labels": labels},
                                 "status": {"phase": "Pending",
                                            "conditions": [{"type": "Ready", "status": "False"}]}})
            self._run_pod(ns, pod, tmpl["spec"]["containers"][0])
        if self._thread is None:
            self._thread = threading.Thread(target=self._probe_loop, daemon=True)
            self._thread.start()

    def _run_pod(self, ns: str, pod: str, c: dict):
        ports = {p["containerPort"]: _free_port() for p in c.get("ports", [])}
        env = {"PATH": os.environ.get("PATH", "/usr/bin:/bin"), "HOME": os.environ.get("HOME", "/tmp"),
               "PYTHONPATH": ROOT, "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": "", "OMP_NUM_THREADS": "2"}
        for e in c.get("env", []):
            if "value" in e:
                env[e["name"]] = str(e["value"])
            elif "valueFrom" in e:
                path = e["valueFrom"].get("fieldRef", {}).get("fieldPath")
                env[e["name"]] = {"metadata.name": pod, "metadata.namespace": ns}.get(path, "")
        for cport, var in PORT_ENV.items():
            if cport in ports:
                env[var] = str(ports[cport])
        env["MASTER_ADDR"] = "127.0.0.1"
        env.update(self.extra_env)
        log = open(os.path.join(self.logdir, f"{pod}.log"), "w")
        proc = subprocess.Popen(list(c["command"]) + list(c.get("args", [])), cwd=ROOT, env=env, stdout=log,
                                stderr=subprocess.STDOUT)
        self.pods[pod] = {"proc": proc, "ports": ports, "ns": ns, "ready": False, "container": c, "log": log,
                          "env": env}

    # -- readiness probes ----------------------------------------------------------
    def _probe(self, info) -> bool:
        pr = info["container"].get("readinessProbe", {}).get("httpGet")
        if not pr:
            return info["proc"].poll() is None
        port = info["ports"].get(pr["port"], pr["port"])
        try:
            with urllib.request.urlopen(f"http://127.0.0.1:{port}{pr['path']}", timeout=1.0) as r:
                return 200 <= r.status < 400
        except Exception:  # noqa: BLE001 - not ready yet / not the leader
            return False

    def _probe_loop(self):
        while not self._stop.is_set():
            for pod, info in list(self.pods.items()):
                ok = self._probe(info)
                running = info["proc"].poll() is None
                if ok != info["ready"] or info.get("running") != running:
                    info["ready"], info["running"] = ok, running
                    o = self.k8s.get("pods", info["ns"], pod)
                    if o is not None:
                        o["status"] = {"phase": "Running" if running else "Failed",
                                       "conditions": [{"type": "Ready", "status": "True" if ok else "False"}]}
                        self.k8s.put("pods", info["ns"], o, "MODIFIED")
            self._stop.wait(0.3)

    def wait_ready(self, pod: str, timeout: float = 180.0) -> dict:
        t0 = time.monotonic()
        while time.monotonic() - t0 < timeout:
            info = self.pods.get(pod)
            if info is not None:
                if info["proc"].poll() is not None:
                    raise RuntimeError(f"pod {pod} exited with {info['proc'].returncode}: " + self.log_tail(pod))
                if info["ready"]:
                    return info
            time.sleep(0.2)
        raise TimeoutError(f"pod {pod} not Ready after {timeout:.0f}s: " + self.log_tail(pod))

    def log_tail(self, pod: str, n: int = 3000) -> str:
        try:
            with open(os.path.join(self.logdir, f"{pod}.log")) as f:
                return f.read()[-n:]
        except OSError:
            return ""

    def stop(self):
        self._stop.set()
        for info in self.pods.values():
            p = info["proc"]
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(timeout=15)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            info["log"].close()
