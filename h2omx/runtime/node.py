"""Node entry point: ``python -m h2omx.runtime.node`` is the container
command of every pod of the StatefulSet (the reference ran
``java -jar h2o.jar``, ``src/k8s/templates.rs:30``).

1. read the environment contract and form the cloud (cluster.form_cluster)
2. serve the leader probe on ``H2O_KUBERNETES_API_PORT`` (all ranks)
3. rank 0: serve the H2O REST API on 54321 and lead the command bus;
   other ranks: follow the bus until shutdown

Options mirror H2O's launcher where they make sense (``-port``,
``-context_path``, ``-name``); ``--device cpu`` forces the gloo/CPU path.
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import sys
import threading

log = logging.getLogger("h2omx.node")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="h2omx-node", description="h2omx cluster node (H2O-compatible)")
    ap.add_argument("-port", "--port", type=int, default=None, help="REST port (default 54321)")
    ap.add_argument("-context_path", "--context-path", default=os.environ.get("H2OMX_CONTEXT_PATH", ""))
    ap.add_argument("-name", "--name", default=None, help="cloud name")
    ap.add_argument("--device", choices=["cuda", "cpu"], default=None)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--no-probe", action="store_true", help="do not serve the leader probe")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")

    # a pod with several GPUs runs one rank per GPU: the pod's main process only
    # starts them (before any GPU call) and fails the pod as soon as one dies
    gpn = int(os.environ.get("H2OMX_GPUS_PER_NODE", "1") or "1")
    if gpn > 1 and "H2OMX_LOCAL_RANK" not in os.environ:
        from .launch import spawn_ranks

        cmd = [sys.executable, "-m", "h2omx.runtime.node", *(sys.argv[1:] if argv is None else argv)]
        env = dict(os.environ)
        log.info("starting %d local ranks (one per GPU)", gpn)
        # rendezvous address / ranks come from the StatefulSet contract in each child
        return spawn_ranks(cmd, gpn, env=env, master_addr=None)

    from ..api.server import H2OApi, serve
    from .cluster import config_from_env, form_cluster
    from .leader import serve_leader_probe

    cfg = config_from_env()
    if a.port:
        cfg.rest_port = a.port
    if a.name:
        cfg.cloud_name = a.name
    log.info("node rank %d/%d, master %s:%d", cfg.rank, cfg.world_size, cfg.master_addr, cfg.master_port)
    cl = form_cluster(cfg, device=a.device)
    # one probe server per pod (the ranks of a pod share its network namespace)
    probe = None if (a.no_probe or cfg.local_rank != 0) else serve_leader_probe(cl, a.host)
    stop = threading.Event()

    def _term(*_):
        stop.set()

    signal.signal(signal.SIGTERM, _term)
    if cl.is_leader:
        def shutdown():
            cl.shutdown_workers()
            stop.set()

        api = H2OApi(cl, shutdown_cb=shutdown)
        srv = serve(api, a.host, cfg.rest_port, a.context_path)
        log.info("H2O REST API on %s:%d%s (cloud %s, %d nodes)", a.host, cfg.rest_port, a.context_path,
                 cfg.cloud_name, cfg.world_size)
        print(f"h2omx node ready: http://{a.host}:{cfg.rest_port}{a.context_path}", flush=True)
        try:
            while not stop.wait(1.0):
                pass
        finally:
            srv.shutdown()
    else:
        cl.worker_loop()
    if probe is not None:
        probe.shutdown()
    cl.comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
