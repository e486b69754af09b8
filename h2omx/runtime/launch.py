"""One process per GPU: the local rank launcher.

An MI355X node runs one rank per GPU.  Inside a pod that owns several GPUs
(``h2ok deploy --gpus_per_node 8 --cluster_size 1``) and for ``bench.py
--gpus N`` outside torchrun, this module starts the ranks as fresh child
processes, the way torchrun would:

* the parent never touches the GPU (no HIP call, no ``torch.cuda`` init):
  it only forks, forwards signals and waits;
* child ``i`` gets ``LOCAL_RANK=i``, ``RANK=rank_base+i``, ``WORLD_SIZE``,
  ``LOCAL_WORLD_SIZE`` and the rendezvous address, and selects
  ``cuda:LOCAL_RANK`` itself (all GPUs stay visible, so RCCL sees the xGMI
  peers and picks its P2P transport);
* if any child exits non-zero the others are terminated (SIGTERM, then
  SIGKILL after a grace period) and the launcher exits with that child's
  code: a dead rank fails the node in bounded time instead of leaving its
  peers blocked inside a collective.

The reference scales by StatefulSet replicas plus an environment contract
(``/root/reference/src/k8s/templates.rs:17-18,48-56``); this is the
intra-pod half of that contract (``H2OMX_GPUS_PER_NODE`` ranks per pod).

CLI (torchrun-like, used by tests and scripts)::

    python -m h2omx.runtime.launch --nproc 2 [--master-port P] -- python worker.py args...
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time

GRACE_S = 10.0


def free_port(host: str = "127.0.0.1") -> int:
    s = socket.socket()
    s.bind((host, 0))
    p = s.getsockname()[1]
    s.close()
    return p


def free_ports(k: int = 2, host: str = "127.0.0.1") -> list[int]:
    """``k`` distinct ports, all bound at once while choosing (so none repeats);
    the first is a rendezvous port whose successor (the command bus,
    ClusterConfig.bus_port) is free too."""
    held, out = [], []
    try:
        while len(out) < k:
            s = socket.socket()
            s.bind((host, 0))
            held.append(s)
            p = s.getsockname()[1]
            if not out:
                t = socket.socket()
                try:
                    t.bind((host, p + 1))
                except OSError:
                    t.close()
                    continue
                held.append(t)
            out.append(p)
    finally:
        for s in held:
            s.close()
    return out


def rank_env(base: dict, local_rank: int, nproc: int, rank_base: int, world: int, master_addr: str | None,
             master_port: int | None) -> dict:
    """Child environment.  ``master_addr=None``: the global rank / world /
    rendezvous come from elsewhere (the StatefulSet contract, see
    cluster.config_from_env); only the local rank is set."""
    env = dict(base)
    env.update({
        "LOCAL_RANK": str(local_rank),
        "H2OMX_LOCAL_RANK": str(local_rank),
        "LOCAL_WORLD_SIZE": str(nproc),
    })
    if master_addr is not None:
        env.update({
            "RANK": str(rank_base + local_rank),
            "WORLD_SIZE": str(world),
            "MASTER_ADDR": master_addr,
            "MASTER_PORT": str(master_port),
        })
    # the host driver only supports dmabuf IPC (RCCL / CUDA-tensor sharing)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def spawn_ranks(cmd: list[str], nproc: int, *, rank_base: int = 0, world: int | None = None,
                master_addr: str | None = "127.0.0.1", master_port: int | None = None, env: dict | None = None,
                poll_s: float = 0.2, grace_s: float = GRACE_S) -> int:
    """Run ``cmd`` as ``nproc`` local ranks; return the first non-zero exit
    code (0 if every rank succeeded)."""
    if nproc < 1:
        raise ValueError("nproc must be >= 1")
    world = nproc if world is None else world
    port = None
    if master_addr is not None:
        port = master_port or free_ports(1, master_addr if master_addr != "0.0.0.0" else "127.0.0.1")[0]
    base = dict(os.environ if env is None else env)
    procs = [subprocess.Popen(cmd, env=rank_env(base, i, nproc, rank_base, world, master_addr, port))
             for i in range(nproc)]

    def _forward(sig, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)

    old = {}
    for sig in (signal.SIGTERM, signal.SIGINT):
        try:
            old[sig] = signal.signal(sig, _forward)
        except ValueError:        # not the main thread (tests): no forwarding
            pass
    try:
        rc = 0
        while True:
            alive = 0
            for i, p in enumerate(procs):
                code = p.poll()
                if code is None:
                    alive += 1
                elif code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    sys.stderr.write(f"[h2omx.launch] local rank {i} exited with {code}; stopping the other ranks\n")
            if rc != 0 or alive == 0:
                break
            time.sleep(poll_s)
        if rc != 0:
            _terminate(procs, grace_s)
        return rc
    finally:
        for sig, h in old.items():
            signal.signal(sig, h)


def _terminate(procs, grace_s: float) -> None:
    for p in procs:
        if p.poll() is None:
            p.terminate()
    deadline = time.monotonic() + grace_s
    for p in procs:
        left = deadline - time.monotonic()
        try:
            p.wait(timeout=max(left, 0.01))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="h2omx-launch", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nproc", type=int, required=True, help="local ranks (one per GPU)")
    ap.add_argument("--rank-base", type=int, default=0)
    ap.add_argument("--world", type=int, default=0, help="world size (default: nproc)")
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=0)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        ap.error("missing command")
    return spawn_ranks(cmd, a.nproc, rank_base=a.rank_base, world=a.world or None,
                       master_addr=a.master_addr, master_port=a.master_port or None)


if __name__ == "__main__":
    sys.exit(main())
