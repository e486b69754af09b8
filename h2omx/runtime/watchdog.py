"""Peer-failure detection with a bounded detection time.

H2O-3 notices a dead node through its heartbeat (the cloud turns unhealthy
and running jobs fail).  A ``torch.distributed`` collective, by contrast,
blocks until the process-group timeout (600-1800 s here) when a peer is
gone or hung.  Every rank of a multi-node h2omx cloud therefore runs:

* a **heartbeat**: a counter in the command-bus ``TCPStore`` (``hb/<rank>``),
  bumped every ``hb_s`` seconds over a dedicated short-timeout client
  connection (no cross-host clock comparison: a peer is judged by whether
  its counter moves);
* a **watchdog**: if any peer's counter has not moved for ``dead_s``
  seconds, or the store (hosted by rank 0) stops answering, the rank
  declares the peer lost:

  1. ``Comm.failed`` is set, so every later collective raises
     :class:`PeerLost` before it is issued;
  2. the registered callbacks run (the leader fails its RUNNING jobs with
     the reason and reports the cloud unhealthy);
  3. the process group is aborted (``ncclCommAbort`` for RCCL, which
     unblocks a collective stuck on the lost peer);
  4. after ``grace_s`` the process exits with :data:`EXIT_PEER_LOST`
     (75, EX_TEMPFAIL), so Kubernetes restarts the pod and the StatefulSet
     re-forms the cloud.  The process never re-execs itself.

Defaults (``H2OMX_HEARTBEAT_S`` 1, ``H2OMX_PEER_DEAD_S`` 10,
``H2OMX_PEER_GRACE_S`` 5): a lost peer fails the job within ~11 s and the
pod exits within ~16 s.
"""
from __future__ import annotations

import datetime
import logging
import os
import threading
import time

log = logging.getLogger("h2omx.watchdog")

EXIT_PEER_LOST = 75


class PeerLost(RuntimeError):
    """A peer rank stopped answering; the cloud can no longer run collectives."""


class PeerWatchdog:
    def __init__(self, host: str, port: int, rank: int, world_size: int, comm=None, *, hb_s: float | None = None,
                 dead_s: float | None = None, grace_s: float | None = None, exit_fn=None, store=None):
        env = os.environ
        self.rank, self.world = rank, world_size
        self.comm = comm
        self.hb_s = float(hb_s if hb_s is not None else env.get("H2OMX_HEARTBEAT_S", "1"))
        self.dead_s = float(dead_s if dead_s is not None else env.get("H2OMX_PEER_DEAD_S", "10"))
        self.grace_s = float(grace_s if grace_s is not None else env.get("H2OMX_PEER_GRACE_S", "5"))
        self.exit_fn = exit_fn or (lambda code: os._exit(code))
        self.callbacks: list = []
        self.failed: str | None = None
        self._stop = threading.Event()
        self._host, self._port = host, port
        self._store = store
        self._thread: threading.Thread | None = None

    def _client(self):
        if self._store is None:
            import torch.distributed as dist

            # own connection with a short timeout: a hung store host must not
            # block the watchdog for the process-group timeout
            self._store = dist.TCPStore(self._host, self._port, self.world, False,
                                        timeout=datetime.timedelta(seconds=max(2.0, 2 * self.hb_s)))
        return self._store

    def on_lost(self, fn) -> None:
        self.callbacks.append(fn)

    def start(self) -> "PeerWatchdog":
        self._thread = threading.Thread(target=self._run, name="h2omx-watchdog", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()

    def _run(self) -> None:
        n = 0
        peers = [r for r in range(self.world) if r != self.rank]
        seen = {r: (None, time.monotonic()) for r in peers}
        while not self._stop.is_set():
            now = time.monotonic()
            try:
                st = self._client()
                n += 1
                st.set(f"hb/{self.rank}", str(n))
                for r in peers:
                    key = f"hb/{r}"
                    v = st.get(key) if st.check([key]) else None
                    if v != seen[r][0]:
                        seen[r] = (v, now)
            except Exception as e:  # noqa: BLE001 - store host gone / hung
                if self.rank != 0:
                    self.lost(f"rank 0 (command-bus store) unreachable: {type(e).__name__}: {e}")
                    return
            stale = [r for r in peers if now - seen[r][1] > self.dead_s]
            if stale:
                self.lost(", ".join(f"rank {r}: no heartbeat for {now - seen[r][1]:.0f} s" for r in stale))
                return
            self._stop.wait(self.hb_s)

    def lost(self, reason: str) -> None:
        if self.failed is not None:
            return
        self.failed = reason
        log.error("peer lost: %s", reason)
        if self.comm is not None:
            self.comm.failed = reason
        for fn in self.callbacks:
            try:
                fn(reason)
            except Exception:  # noqa: BLE001
                log.exception("peer-lost callback failed")
        try:
            import torch.distributed as dist

            if dist.is_initialized():
                dist.distributed_c10d._abort_process_group()
        except Exception:  # noqa: BLE001
            log.exception("process-group abort failed")
        if self.grace_s >= 0:
            t = threading.Timer(self.grace_s, self.exit_fn, args=(EXIT_PEER_LOST,))
            t.daemon = True
            t.start()
