"""Peer visibility / transport check at cloud formation.

One rank per MI355X only pays off if RCCL's collectives run over xGMI
peer-to-peer links.  RCCL picks that transport when the peer GPU is visible
and peer-accessible from the rank's process; a pod that sees only its own GPU
(the stock device-plugin allocation for "one pod per GPU", see
``control/src/deployment.cpp`` and SURVEY.md §7.5.1) silently falls back to a
shared-memory or socket transport at a fraction of the bandwidth.  This
module makes that visible at cloud formation:

* every rank reports its host, local device, visible device count, PCI bus id
  and the ``hipDeviceCanAccessPeer`` row of its device against the other
  visible devices;
* rank 0 assembles the cloud's report: per host, whether every pair of the
  ranks' GPUs is peer-accessible from inside the ranks' processes;
* a node whose ranks cannot reach each other's GPUs is an error when
  ``H2OMX_REQUIRE_P2P=1`` (formation fails loudly) and a loud warning
  otherwise;
* ``H2OMX_COMM_PROBE_MB=<MB>`` adds a timed all-reduce of that size and
  reports its bus bandwidth (2 (N-1)/N x bytes / time).

The reference's scale-out contract is the StatefulSet replica count plus the
clustering env (``/root/reference/src/k8s/templates.rs:17-18,48-56``); this
is the GPU-interconnect half of forming that cloud.
"""
from __future__ import annotations

import os
import socket
import sys
import time


def rank_info(device) -> dict:
    """This process's view: host, device index, visible devices, PCI bus, peer row."""
    info = {"host": socket.gethostname(), "device": None, "visible": 0, "pci_bus": None, "peer_row": []}
    try:
        import torch

        n = torch.cuda.device_count()
        info["visible"] = n
        if device is not None and getattr(device, "type", "cpu") == "cuda" and n:
            i = device.index or 0
            info["device"] = i
            props = torch.cuda.get_device_properties(i)
            info["pci_bus"] = getattr(props, "pci_bus_id", None)
            uid = getattr(props, "uuid", None)
            # physical identity of the GPU (several ranks on one GPU = test mode)
            info["gpu_id"] = str(uid) if uid is not None else (
                None if info["pci_bus"] is None else f"pci:{getattr(props, 'pci_domain_id', 0)}:{info['pci_bus']}")
            info["name"] = props.name
            info["peer_row"] = [bool(j == i or torch.cuda.can_device_access_peer(i, j)) for j in range(n)]
    except Exception as e:  # noqa: BLE001 - report, never fail formation on a probe error
        info["error"] = f"{type(e).__name__}: {e}"
    return info


def assess(infos: list[dict]) -> dict:
    """Cloud-level verdict from every rank's :func:`rank_info` (pure function)."""
    by_host: dict[str, list[tuple[int, dict]]] = {}
    for r, inf in enumerate(infos):
        by_host.setdefault(inf.get("host", "?"), []).append((r, inf))
    hosts, problems = {}, []
    for host, members in by_host.items():
        gpu = [(r, i) for r, i in members if i.get("device") is not None]
        entry = {"ranks": [r for r, _ in members], "gpu_ranks": len(gpu)}
        ids = [i.get("gpu_id") for _, i in gpu]
        if len(gpu) <= 1:
            entry["p2p"] = "n/a (one GPU rank on this host)"
        elif all(x is not None for x in ids) and len(set(ids)) < len(ids):
            entry["p2p"] = "shared device"
            problems.append(f"{host}: several ranks drive the same GPU ({len(set(ids))} distinct GPUs for "
                            f"{len(ids)} ranks; test mode only)")
        elif all(i.get("visible", 0) <= 1 for _, i in gpu):
            entry["p2p"] = "not visible"
            problems.append(f"{host}: {len(gpu)} GPU ranks each see only their own GPU (pod-per-GPU without peer "
                            "visibility): RCCL cannot use xGMI peer-to-peer and falls back to SHM / sockets; expose "
                            "the node's GPUs to every rank pod (hostIPC + all render nodes, HIP_VISIBLE_DEVICES "
                            "pinning) or run one pod with H2OMX_GPUS_PER_NODE ranks")
        else:
            devs = [i["device"] for _, i in gpu]
            bad = [(ra, devs[kb]) for (ra, ia) in gpu for kb in range(len(gpu))
                   if devs[kb] != ia["device"] and (devs[kb] >= len(ia.get("peer_row", []))
                                                    or not ia["peer_row"][devs[kb]])]
            if len(set(devs)) < len(devs):
                entry["p2p"] = "shared device"
                problems.append(f"{host}: several ranks drive the same GPU {sorted(devs)} (test mode only)")
            elif bad:
                entry["p2p"] = "partial"
                problems.append(f"{host}: no peer access for (rank, device) pairs {bad[:8]}")
            else:
                entry["p2p"] = "all pairs peer-accessible"
        hosts[host] = entry
    return {"world": len(infos), "hosts": hosts, "problems": problems, "ok": not problems}


def probe_allreduce(comm, mb: float) -> dict:
    """Timed all-reduce of ``mb`` MB (fp32) on the comm's device: bus bandwidth."""
    import torch

    n = max(1, int(mb * (1 << 20) // 4))
    t = torch.ones((n,), dtype=torch.float32, device=comm.device)
    comm.all_reduce_(t)          # warm-up (connection setup)
    if comm.device.type == "cuda":
        torch.cuda.synchronize(comm.device)
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        comm.all_reduce_(t)
    if comm.device.type == "cuda":
        torch.cuda.synchronize(comm.device)
    dt = comm.max_scalar((time.perf_counter() - t0) / reps)
    w = comm.world_size
    nbytes = 4 * n
    return {"bytes": nbytes, "s": dt, "algbw_GBs": nbytes / dt / 1e9, "busbw_GBs": 2 * (w - 1) / w * nbytes / dt / 1e9}


def check_cloud(comm, require: bool | None = None, probe_mb: float | None = None, log=None) -> dict:
    """Gather every rank's view, assess it on every rank (same verdict
    everywhere), log it on rank 0 and fail loudly if peers are required."""
    if comm.world_size <= 1:
        return {"world": 1, "hosts": {}, "problems": [], "ok": True}
    infos = comm.all_gather_object(rank_info(comm.device))
    rep = assess(infos)
    if probe_mb is None:
        probe_mb = float(os.environ.get("H2OMX_COMM_PROBE_MB", "0") or 0)
    if probe_mb > 0:
        rep["probe"] = probe_allreduce(comm, probe_mb)
    if require is None:
        require = os.environ.get("H2OMX_REQUIRE_P2P", "0") == "1"
    log = log or (lambda m: sys.stderr.write(m + "\n"))
    if comm.rank == 0:
        for host, e in rep["hosts"].items():
            log(f"[h2omx.topology] {host}: ranks {e['ranks']} -> {e['p2p']}")
        if "probe" in rep:
            log(f"[h2omx.topology] all-reduce {rep['probe']['bytes'] / 2**20:.0f} MB: "
                f"bus {rep['probe']['busbw_GBs']:.1f} GB/s")
        for p in rep["problems"]:
            log(f"[h2omx.topology] WARNING: {p}")
    if rep["problems"] and require:
        raise RuntimeError("GPU peer access required (H2OMX_REQUIRE_P2P=1) but: " + "; ".join(rep["problems"]))
    return rep


def cloud_summary(report: dict | None, comm=None) -> dict:
    """Compact topology verdict for /3/Cloud and the operator's CR status:
    per-host peer access, problems, and the transport the small collectives
    use (one-shot P2P kernels over IPC-mapped HBM, or RCCL / gloo)."""
    out = {"world": 1, "p2p": {}, "problems": [], "ok": True, "collectives": "none (1 rank)"}
    if report:
        out.update(world=report.get("world", 1), p2p={h: e.get("p2p") for h, e in report.get("hosts", {}).items()},
                   problems=list(report.get("problems", [])), ok=bool(report.get("ok", True)))
        if "probe" in report:
            out["allreduce_busbw_GBs"] = report["probe"].get("busbw_GBs")
    if comm is not None and comm.world_size > 1:
        if getattr(comm, "p2p", None) is not None:
            out["collectives"] = "p2p one-shot (IPC-mapped HBM) + rccl for large messages"
        else:
            try:
                import torch.distributed as dist

                be = dist.get_backend(comm.group) if dist.is_initialized() else "?"
            except Exception:        # noqa: BLE001
                be = "?"
            out["collectives"] = ("rccl" if be == "nccl" else be) + (
                f" (p2p off: {comm.p2p_error})" if getattr(comm, "p2p_error", None) else "")
    return out
