"""Cluster formation and distributed execution on CPU (gloo, world 2).

* the StatefulSet environment contract -> rank / world / rendezvous address
* peer discovery timeout, the leader readiness probe
* a real 2-node cloud (two ``python -m h2omx.runtime.node`` processes): the
  leader serves REST, both ranks parse their shard of the CSV, train with
  all-reduced statistics; results match single-process training on the
  whole file; an injected fault on rank 1 fails the job instead of hanging;
  ``/3/Shutdown`` stops both nodes.
"""
import os
import socket
import subprocess
import sys
import time
import urllib.request

import numpy as np
import pandas as pd
import pytest

from h2omx.client import H2OConnection, H2OResponseError
from h2omx.runtime.cluster import Cluster, ClusterConfig, config_from_env, wait_for_peers
from h2omx.runtime.leader import serve_leader_probe

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_env_contract_statefulset():
    env = {"H2O_KUBERNETES_SERVICE_DNS": "demo-service.ns.svc.cluster.local", "H2O_NODE_EXPECTED_COUNT": "4",
           "H2O_NODE_LOOKUP_TIMEOUT": "30", "H2O_KUBERNETES_API_PORT": "8081", "HOSTNAME": "demo-stateful-set-2"}
    cfg = config_from_env(env)
    assert (cfg.rank, cfg.world_size, cfg.api_port) == (2, 4, 8081)
    assert cfg.master_addr == "demo-stateful-set-0.demo-service.ns.svc.cluster.local"
    assert cfg.lookup_timeout_s == 30
    with pytest.raises(ValueError):
        config_from_env(dict(env, HOSTNAME="no-ordinal"))
    with pytest.raises(ValueError):
        config_from_env(dict(env, HOSTNAME="demo-stateful-set-7"))


def test_env_contract_torchrun():
    cfg = config_from_env({"RANK": "1", "WORLD_SIZE": "2", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "1234"})
    assert (cfg.rank, cfg.world_size, cfg.master_addr, cfg.master_port) == (1, 2, "127.0.0.1", 1234)


def test_peer_discovery():
    cfg = ClusterConfig(rank=0, world_size=3, service_dns="svc", lookup_timeout_s=5)
    calls = {"n": 0}

    def resolver(*a):
        calls["n"] += 1
        k = min(calls["n"], 3)
        return [(0, 0, 0, "", (f"10.0.0.{i}", 0)) for i in range(k)]

    assert wait_for_peers(cfg, resolver=resolver, sleep=lambda s: None) == ["10.0.0.0", "10.0.0.1", "10.0.0.2"]
    t = [0.0]

    def clock():
        t[0] += 1.0
        return t[0]

    with pytest.raises(TimeoutError, match="1/3 nodes"):
        wait_for_peers(cfg, resolver=lambda *a: [(0, 0, 0, "", ("10.0.0.1", 0))], sleep=lambda s: None, clock=clock)


def test_leader_probe():
    from h2omx.parallel.comm import Comm

    out = {}
    for rank in (0, 1):
        port = _free_port()
        cl = Cluster(ClusterConfig(rank=rank, world_size=2, api_port=port), Comm(rank, 2))
        srv = serve_leader_probe(cl, "127.0.0.1")
        try:
            urllib.request.urlopen(f"http://127.0.0.1:{port}/kubernetes/isLeaderNode", timeout=5)
            out[rank] = 200
        except urllib.error.HTTPError as e:
            out[rank] = e.code
        srv.shutdown()
    assert out == {0: 200, 1: 404}


@pytest.fixture(scope="module")
def two_node_cloud(tmp_path_factory):
    d = tmp_path_factory.mktemp("cloud")
    rng = np.random.default_rng(5)
    n = 4000
    df = pd.DataFrame({"a": rng.normal(size=n), "b": rng.normal(size=n), "c": rng.choice(list("pqrs"), n),
                       "d": rng.normal(size=n)})
    s = df.a - 0.8 * df.b + (df.c == "p") * 1.2
    df["y"] = np.where(rng.random(n) < 1 / (1 + np.exp(-s)), "1", "0")
    csv = d / "train.csv"
    df.to_csv(csv, index=False)
    from h2omx.runtime.launch import free_ports

    mport, rest = free_ports(2)   # mport + 1 (the command bus) is free as well
    procs = []
    for rank in (0, 1):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(mport),
                   PYTHONPATH=REPO, H2OMX_ENABLE_FAULT_INJECTION="1", OMP_NUM_THREADS="2")
        log = open(d / f"node{rank}.log", "w")
        procs.append(subprocess.Popen([sys.executable, "-m", "h2omx.runtime.node", "--device", "cpu", "--port",
                                       str(rest), "--host", "127.0.0.1", "--no-probe"], env=env, stdout=log,
                                      stderr=subprocess.STDOUT, cwd=REPO))
    conn = H2OConnection(f"http://127.0.0.1:{rest}", timeout=300)
    deadline = time.time() + 120
    while True:
        try:
            conn.connect()
            break
        except Exception:  # noqa: BLE001
            if time.time() > deadline or any(p.poll() is not None for p in procs):
                for p in procs:
                    p.kill()
                logs = "".join(open(d / f"node{r}.log").read()[-3000:] for r in (0, 1))
                pytest.fail(f"cloud did not come up:\n{logs}")
            time.sleep(0.5)
    yield conn, str(csv), df, procs, d
    for p in procs:
        if p.poll() is None:
            p.kill()
            p.wait(timeout=30)


def test_two_node_cloud_end_to_end(two_node_cloud):
    from h2omx.frame import Frame
    from h2omx.models import H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator

    conn, csv, df, procs, d = two_node_cloud
    cloud = conn.request("GET /3/Cloud")
    assert cloud["cloud_size"] == 2
    topo = cloud["h2omx_topology"]
    assert topo["world"] == 2 and "collectives" in topo and isinstance(topo["problems"], list)
    key = conn.import_file(csv, destination_frame="train.hex")
    fr = conn.frame(key, rows=3)
    assert fr["rows"] == len(df)                          # both shards counted
    assert fr["columns"][2]["domain"] == ["p", "q", "r", "s"]   # unified domains
    assert abs(fr["columns"][0]["mean"] - df.a.mean()) < 1e-5
    local = Frame.from_pandas(df.assign(y=df.y.astype("category")))
    g = conn.train("glm", key, y="y", family="binomial", **{"lambda": 0})
    gl = H2OGeneralizedLinearEstimator(family="binomial", lambda_=0.0).train(y="y", training_frame=local)
    names = g["output"]["coefficients_table"]["names"]
    coefs = dict(zip(names, g["output"]["coefficients_table"]["coefficients"]))
    for k, v in gl.coef().items():
        assert abs(coefs[k] - v) < 1e-4, k
    m = conn.train("gbm", key, y="y", ntrees=10, max_depth=3, seed=1, distribution="bernoulli")
    ml = H2OGradientBoostingEstimator(ntrees=10, max_depth=3, seed=1).train(y="y", training_frame=local)
    assert abs(m["output"]["training_metrics"]["AUC"] - ml.training_metrics["AUC"]) < 0.01
    km = conn.train("kmeans", key, x=["a", "b", "d"], k=3, seed=1)
    assert sum(km["output"]["training_metrics"]["centroid_stats"]["data"][1]) == len(df)
    dl = conn.train("deeplearning", key, y="y", hidden=[8], epochs=3, seed=1, distribution="bernoulli")
    assert dl["output"]["training_metrics"]["AUC"] > 0.7
    pred = conn.predict(m["model_id"]["name"], key)
    assert conn.frame(pred)["rows"] == len(df)
    mm = conn.model_performance(m["model_id"]["name"], key)
    assert abs(mm["AUC"] - m["output"]["training_metrics"]["AUC"]) < 1e-9
    # rank 1 fails a command: the leader reports it, the cloud stays usable
    with pytest.raises(H2OResponseError) as e:
        conn.request("POST /99/h2omx/fault", {"rank": 1})
    assert "rank 1" in e.value.payload["msg"]
    assert conn.frame(key)["rows"] == len(df)
    conn.shutdown()
    for p in procs:
        assert p.wait(timeout=60) == 0
