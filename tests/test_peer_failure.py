"""Rank-failure handling with bounded detection time (runtime/watchdog.py).

* unit: a peer whose heartbeat counter stops moving is declared lost after
  dead_s; the communicator fails fast, callbacks run, the process exit is
  scheduled with code 75; a worker that loses the store host does the same.
* integration (CPU, gloo, two ``python -m h2omx.runtime.node`` processes):
  rank 1 is frozen (SIGSTOP: its sockets stay open, so gloo alone would block
  until the process-group timeout) in the middle of a GBM training job; the
  leader reports the job FAILED with PeerLost within 30 s and then exits
  with code 75.
"""
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.parse

import numpy as np
import pandas as pd
import pytest

from h2omx.parallel.comm import Comm
from h2omx.runtime.watchdog import EXIT_PEER_LOST, PeerLost, PeerWatchdog

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _FakeStore:
    def __init__(self):
        self.kv = {}
        self.down = False

    def set(self, k, v):
        if self.down:
            raise RuntimeError("connection reset")
        self.kv[k] = v.encode() if isinstance(v, str) else v

    def check(self, keys):
        if self.down:
            raise RuntimeError("connection reset")
        return all(k in self.kv for k in keys)

    def get(self, k):
        return self.kv[k]


def _wait(pred, timeout):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return time.time() - t0
        time.sleep(0.02)
    raise AssertionError("timed out")


def test_watchdog_declares_silent_peer_lost():
    st = _FakeStore()
    comm = Comm(0, 2)
    exits, reasons = [], []
    wd = PeerWatchdog("x", 0, 0, 2, comm, hb_s=0.05, dead_s=0.5, grace_s=0.1, exit_fn=exits.append, store=st)
    wd.on_lost(reasons.append)
    wd.start()
    # rank 1 heartbeats for a while, then goes silent
    for i in range(10):
        st.set("hb/1", str(i))
        time.sleep(0.05)
    assert wd.failed is None
    dt = _wait(lambda: wd.failed is not None, 5.0)
    assert dt < 2.0
    assert "rank 1" in wd.failed and reasons == [wd.failed]
    assert comm.failed == wd.failed
    with pytest.raises(PeerLost):
        comm.all_reduce_(np.zeros(1))
    _wait(lambda: exits == [EXIT_PEER_LOST], 2.0)
    assert int(st.get("hb/0")) > 10          # our own heartbeat kept moving


def test_worker_loses_store_host():
    st = _FakeStore()
    exits = []
    wd = PeerWatchdog("x", 0, 1, 2, Comm(1, 2), hb_s=0.05, dead_s=5.0, grace_s=0.0, exit_fn=exits.append, store=st)
    wd.start()
    time.sleep(0.2)
    st.down = True
    _wait(lambda: wd.failed is not None, 3.0)
    assert "rank 0" in wd.failed
    _wait(lambda: exits == [EXIT_PEER_LOST], 2.0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_frozen_rank_fails_leader_job_within_bound(tmp_path):
    from h2omx.client import H2OConnection

    rng = np.random.default_rng(3)
    n = 6000
    df = pd.DataFrame({f"x{i}": rng.normal(size=n) for i in range(6)})
    df["y"] = np.where(rng.random(n) < 1 / (1 + np.exp(-(df.x0 - df.x1))), "1", "0")
    csv = tmp_path / "train.csv"
    df.to_csv(csv, index=False)
    from h2omx.runtime.launch import free_ports

    mport, rest = free_ports(2)
    procs = []
    for rank in (0, 1):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(mport),
                   PYTHONPATH=REPO, OMP_NUM_THREADS="2", H2OMX_PEER_DEAD_S="6", H2OMX_HEARTBEAT_S="0.5",
                   H2OMX_PEER_GRACE_S="4", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        log = open(tmp_path / f"node{rank}.log", "w")
        procs.append(subprocess.Popen([sys.executable, "-m", "h2omx.runtime.node", "--device", "cpu", "--port",
                                       str(rest), "--host", "127.0.0.1", "--no-probe"], env=env, stdout=log,
                                      stderr=subprocess.STDOUT, cwd=REPO))
    try:
        conn = H2OConnection(f"http://127.0.0.1:{rest}", timeout=60)
        deadline = time.time() + 120
        while True:
            try:
                conn.connect()
                break
            except Exception:  # noqa: BLE001
                if time.time() > deadline or any(p.poll() is not None for p in procs):
                    pytest.fail("cloud did not come up:\n" +
                                "".join(open(tmp_path / f"node{r}.log").read()[-3000:] for r in (0, 1)))
                time.sleep(0.5)
        key = conn.import_file(str(csv), destination_frame="train.hex")
        b = conn.request("POST /3/ModelBuilders/gbm", {"training_frame": key, "response_column": "y",
                                                       "ntrees": 100000, "max_depth": 3, "seed": 1})
        jkey = urllib.parse.quote(b["job"]["key"]["name"], safe="")
        time.sleep(2.0)                       # training is under way (collectives every level)
        assert conn.request(f"GET /3/Jobs/{jkey}")["jobs"][0]["status"] == "RUNNING"
        os.kill(procs[1].pid, signal.SIGSTOP)
        t0 = time.time()
        status = None
        while time.time() - t0 < 30:
            try:
                j = conn.request(f"GET /3/Jobs/{jkey}")["jobs"][0]
            except Exception:  # noqa: BLE001 - leader already exiting
                break
            status = j["status"]
            if status == "FAILED":
                break
            time.sleep(0.2)
        detect = time.time() - t0
        assert status == "FAILED", status
        assert "PeerLost" in j["exception"] and "rank 1" in j["exception"]
        assert detect < 30
        assert procs[0].wait(timeout=30) == EXIT_PEER_LOST
    finally:
        for p in procs:
            if p.poll() is None:
                os.kill(p.pid, signal.SIGKILL)
                p.wait(timeout=30)
