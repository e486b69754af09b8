"""Collective communication for the data plane.

Replaces H2O-3's MRTask map/reduce fabric: every
algorithm keeps its row shard resident on its GPU and combines per-shard
statistics with one fused collective per tree level / IRLS iteration /
optimizer step.  On MI355X the process group uses backend ``"nccl"`` which
is RCCL over xGMI on ROCm; on CPU-only hosts (tests, the kind/CPU config) it
uses ``gloo``.  Collectives are enqueued on the current stream, ordered
after the producing kernel, with no host synchronisation.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch
import torch.distributed as dist


class Comm:
    def __init__(self, rank: int = 0, world_size: int = 1, device: torch.device | None = None,
                 group=None):
        self.rank = rank
        self.world_size = world_size
        self.device = device or torch.device("cpu")
        self.group = group
        # every collective: calls / bytes / host seconds inside the call (for RCCL the
        # enqueue cost; gloo blocks, so there it is the whole collective).  With
        # timing enabled (enable_timing / H2OMX_COMM_TIMING=1) HIP events also
        # bracket each collective on the current stream: device time including
        # the wait for the slowest peer, resolved lazily by collective_stats()
        self.stats = {"all_reduce_calls": 0, "all_reduce_bytes": 0, "all_reduce_s": 0.0,
                      "all_gather_calls": 0, "all_gather_bytes": 0, "all_gather_s": 0.0,
                      "broadcast_calls": 0, "broadcast_bytes": 0, "broadcast_s": 0.0}
        self.timing = os.environ.get("H2OMX_COMM_TIMING") == "1"
        self._events: list = []
        self._device_ms: dict[str, float] = {}
        # set by the peer watchdog (runtime/watchdog.py) once a rank is lost:
        # collectives then fail fast instead of blocking on the missing peer
        self.failed: str | None = None
        # one-shot P2P all-reduce over IPC-mapped HBM for small messages
        # (parallel/p2p.py): graph-capturable, so tree steps replay as one graph
        self.p2p = None
        self._p2p_dead = None     # a P2P instance disabled after a timeout (closed at shutdown)
        self.p2p_error: str | None = None
        self.stats.update({"p2p_calls": 0, "p2p_bytes": 0, "p2p_s": 0.0})
        self._side = None         # stream of the bucketed P2P all-reduces (all_reduce_bucket_)

    def _check(self) -> None:
        """Raise ``PeerLost`` once a peer is known lost: by the watchdog
        (``failed``) or by a P2P exchange whose poll timed out on the device
        (pinned host word, read without a device sync).  A timed-out exchange
        also disables P2P on this Comm for good: the ranks' epochs no longer
        line up, so every later result of it would be wrong."""
        if self.failed is None and self.p2p is not None and self.p2p.failed():
            self._p2p_dead = self.p2p
            self.p2p = None
            self.failed = (f"{self._p2p_dead.failure_reason()} (H2OMX_P2P_TIMEOUT_S; rank {self.rank} of "
                           f"{self.world_size}); results computed since are invalid")
        if self.failed is not None:
            from ..runtime.watchdog import PeerLost

            raise PeerLost(self.failed)

    def check_health(self) -> None:
        """Public form of :meth:`_check` (tree steps, graph flushes, fit ends)."""
        self._check()

    # ------------------------------------------------------------------
    @classmethod
    def from_env(cls, device: str | None = None, timeout_s: float = 600.0) -> "Comm":
        """Initialise from torchrun / StatefulSet env (RANK, WORLD_SIZE, MASTER_ADDR)."""
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", str(rank)))
        if device is None:
            device = "cuda" if torch.cuda.device_count() > 0 else "cpu"
        if device == "cuda":
            dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
            torch.cuda.set_device(dev)
        else:
            dev = torch.device("cpu")
        if world > 1 and not dist.is_initialized():
            import datetime

            # H2OMX_DIST_BACKEND=gloo: several ranks sharing one GPU (tests of the
            # multi-rank GPU path on a one-GPU box); production uses RCCL
            backend = os.environ.get("H2OMX_DIST_BACKEND") or ("nccl" if dev.type == "cuda" else "gloo")
            kw = {}
            if dev.type == "cuda" and backend == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
        c = cls(rank, world, dev)
        # H2OMX_P2P: auto (default: on when IPC works and the self-test passes), 0 off, 1 required
        mode = os.environ.get("H2OMX_P2P", "auto")
        if world > 1 and dev.type == "cuda" and mode != "0":
            c.enable_p2p(required=mode == "1")
        return c

    def enable_p2p(self, required: bool = False) -> bool:
        """Set up the one-shot P2P all-reduce (collective over the group)."""
        from .p2p import setup

        if self.p2p is None and self.world_size > 1:
            self.p2p = setup(self, required=required)
        return self.p2p is not None

    @property
    def graph_collectives(self) -> bool:
        """True when the small collectives are device-side kernels (P2P), so a
        step graph can be captured whole instead of segmented at collectives."""
        return self.p2p is not None

    @property
    def is_leader(self) -> bool:
        return self.rank == 0

    # ------------------------------------------------------------------
    def enable_timing(self, on: bool = True) -> None:
        self.timing = on

    def _begin(self, kind: str, nbytes: int):
        self.stats[f"{kind}_calls"] += 1
        self.stats[f"{kind}_bytes"] += nbytes
        ev = None
        if self.timing and self.device.type == "cuda":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
        return kind, ev, time.perf_counter()

    def _end(self, tok) -> None:
        kind, ev, t0 = tok
        self.stats[f"{kind}_s"] += time.perf_counter() - t0
        if ev is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self._events.append((kind, ev, e1))
            if len(self._events) > 4096:
                self._drain()

    def _drain(self) -> None:
        for kind, a, b in self._events:
            b.synchronize()
            self._device_ms[kind] = self._device_ms.get(kind, 0.0) + a.elapsed_time(b)
        self._events.clear()

    def collective_stats(self, reset: bool = False) -> dict:
        """Counters of every collective so far (+ device ms per kind when timed)."""
        self._drain()
        out = dict(self.stats)
        out.update({f"{k}_device_ms": v for k, v in self._device_ms.items()})
        if reset:
            for k in self.stats:
                self.stats[k] = 0.0 if k.endswith("_s") else 0
            if self.p2p is not None:
                self.p2p.check()
            self._device_ms.clear()
        return out

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.world_size == 1:
            return t
        self._check()
        if self._p2p_chunks(t, op):
            # device-side one-shot collectives (kernels: no host-issued RCCL call);
            # a tensor above the symmetric buffer goes as consecutive cap-sized chunks
            tok = self._begin("p2p", t.numel() * t.element_size())
            step = self.p2p.cap // t.element_size() // 4 * 4
            flat = t.view(-1)
            for s in range(0, flat.numel(), step):
                self.p2p.all_reduce_(flat[s:s + step], op)
            self._end(tok)
            return t
        tok = self._begin("all_reduce", t.numel() * t.element_size())
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        dist.all_reduce(t, op=rop, group=self.group)
        self._end(tok)
        return t

    def _p2p_chunks(self, t: torch.Tensor, op: str) -> bool:
        """True when the P2P exchange carries ``t`` (whole, or in cap-sized chunks)."""
        p2p = self.p2p
        if p2p is None or not t.is_contiguous():
            return False
        if p2p.supports(t, op):
            return True
        step = p2p.cap // t.element_size() // 4 * 4
        return step > 0 and p2p.supports(t.view(-1)[:step], op)

    def all_reduce_bucket_(self, t: torch.Tensor, op: str = "sum"):
        """In-place all-reduce of one gradient bucket, overlapped with the
        producer's remaining work; returns a handle whose ``wait()`` joins it
        back into the current stream.  With P2P the collective is a kernel on
        this Comm's side stream (forked from / joined to the current stream by
        events: graph-capturable, no host-issued collective, and every bucket
        summed in rank order, so the replicas stay bit-identical); otherwise an
        asynchronous RCCL call."""
        if self.world_size == 1:
            return _Done()
        self._check()
        if self._p2p_chunks(t, op) and t.is_cuda:
            main = torch.cuda.current_stream(t.device)
            if self._side is None:
                self._side = torch.cuda.Stream(t.device)
            side = self._side
            side.wait_stream(main)
            with torch.cuda.stream(side):
                self.all_reduce_(t, op)
            return _StreamJoin(main, side)
        return self.all_reduce_async(t, op)

    def all_reduce_async(self, t: torch.Tensor, op: str = "sum"):
        """Non-blocking all-reduce; returns a handle with ``wait()`` (gradient
        buckets overlapped with the rest of back-propagation)."""
        if self.world_size == 1:
            return _Done()
        self._check()
        self.stats["all_reduce_calls"] += 1
        self.stats["all_reduce_bytes"] += t.numel() * t.element_size()
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        t0 = time.perf_counter()
        work = dist.all_reduce(t, op=rop, group=self.group, async_op=True)
        self.stats["all_reduce_s"] += time.perf_counter() - t0
        return work

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        return self.broadcast_(t, src)

    def all_reduce_numpy(self, a: np.ndarray, op: str = "sum") -> np.ndarray:
        if self.world_size == 1:
            return a
        t = torch.from_numpy(np.ascontiguousarray(a))
        if self.device.type == "cuda":
            t = t.to(self.device)
        self.all_reduce_(t, op)
        return t.cpu().numpy()

    def all_gather_cat(self, t: torch.Tensor, dim: int = 0) -> torch.Tensor:
        if self.world_size == 1:
            return t
        self._check()
        # shapes may differ in `dim`: gather sizes first
        n = torch.tensor([t.shape[dim]], dtype=torch.int64, device=t.device)
        sizes = [torch.zeros_like(n) for _ in range(self.world_size)]
        dist.all_gather(sizes, n, group=self.group)
        sizes = [int(s.item()) for s in sizes]
        mx = max(sizes)
        pad_shape = list(t.shape)
        pad_shape[dim] = mx
        buf = torch.zeros(pad_shape, dtype=t.dtype, device=t.device)
        buf.narrow(dim, 0, t.shape[dim]).copy_(t)
        outs = [torch.empty_like(buf) for _ in range(self.world_size)]
        tok = self._begin("all_gather", buf.numel() * buf.element_size() * self.world_size)
        dist.all_gather(outs, buf, group=self.group)
        self._end(tok)
        return torch.cat([o.narrow(dim, 0, s) for o, s in zip(outs, sizes)], dim=dim)

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.world_size > 1:
            self._check()
            tok = self._begin("broadcast", t.numel() * t.element_size())
            dist.broadcast(t, src=src, group=self.group)
            self._end(tok)
        return t

    def broadcast_object(self, obj, src: int = 0):
        if self.world_size == 1:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=src, group=self.group)
        return lst[0]

    def all_gather_object(self, obj) -> list:
        """Every rank's picklable ``obj``, in rank order (small control data)."""
        if self.world_size == 1:
            return [obj]
        self._check()
        out = [None] * self.world_size
        tok = self._begin("all_gather", 0)
        dist.all_gather_object(out, obj, group=self.group)
        self._end(tok)
        return out

    def barrier(self) -> None:
        if self.world_size > 1:
            self._check()
            if self.device.type == "cuda" and dist.get_backend(self.group) == "nccl":
                dist.barrier(group=self.group, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.group)

    def max_scalar(self, v: float) -> float:
        if self.world_size == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=self.device)
        self.all_reduce_(t, "max")
        return float(t.item())

    def shutdown(self) -> None:
        """Barrier, release the P2P buffers, tear the group down - and only then
        report a P2P timeout nobody checked (raising first would leave the
        other ranks waiting in the barrier)."""
        err = None
        p2p = self.p2p or self._p2p_dead
        if p2p is not None:
            lost = p2p.failed()
            if not lost and self.failed is None:
                self.barrier()
            p2p.close()
            self.p2p = self._p2p_dead = None
            if lost and self.failed is None:
                err = RuntimeError(f"P2P all-reduce: a poll timed out waiting for a peer (rank {self.rank} of "
                                   f"{self.world_size}); results computed since then are invalid")
        if self.world_size > 1 and dist.is_initialized():
            dist.destroy_process_group()
        if err is not None:
            raise err


class LoopbackComm(Comm):
    """One process standing in for ``world`` identical ranks on one GPU (the
    strong-scaling proxy, ``bench.py --loopback-ranks N``): the one-shot P2P
    path runs with every "peer" buffer mapped to this process's own, so the
    N-rank launch sequence - fused level exchanges, N-way sums, the same
    grids - is what gets timed.  Host-side collectives behave as N copies of
    this rank (sums x N, max / min / gathers of identical values).  Results
    are those of N identical shards, not of one: this is a timing harness."""

    def __init__(self, device: torch.device, world: int):
        if world < 2:
            raise ValueError("loopback needs a stand-in world of >= 2 ranks")
        super().__init__(0, world, device)
        from .p2p import P2PAllReduce

        self.p2p = P2PAllReduce.loopback_for(self)

    def barrier(self) -> None:
        self._check()

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        self._check()
        if self.p2p is not None and self.p2p.supports(t, op):
            tok = self._begin("p2p", t.numel() * t.element_size())
            self.p2p.all_reduce_(t, op)
            self._end(tok)
        elif op == "sum":
            t.mul_(self.world_size)
        return t

    def _p2p_chunks(self, t: torch.Tensor, op: str) -> bool:
        """True when the P2P exchange carries ``t`` (whole, or in cap-sized chunks)."""
        p2p = self.p2p
        if p2p is None or not t.is_contiguous():
            return False
        if p2p.supports(t, op):
            return True
        step = p2p.cap // t.element_size() // 4 * 4
        return step > 0 and p2p.supports(t.view(-1)[:step], op)

    def all_reduce_bucket_(self, t: torch.Tensor, op: str = "sum"):
        """In-place all-reduce of one gradient bucket, overlapped with the
        producer's remaining work; returns a handle whose ``wait()`` joins it
        back into the current stream.  With P2P the collective is a kernel on
        this Comm's side stream (forked from / joined to the current stream by
        events: graph-capturable, no host-issued collective, and every bucket
        summed in rank order, so the replicas stay bit-identical); otherwise an
        asynchronous RCCL call."""
        if self.world_size == 1:
            return _Done()
        self._check()
        if self._p2p_chunks(t, op) and t.is_cuda:
            main = torch.cuda.current_stream(t.device)
            if self._side is None:
                self._side = torch.cuda.Stream(t.device)
            side = self._side
            side.wait_stream(main)
            with torch.cuda.stream(side):
                self.all_reduce_(t, op)
            return _StreamJoin(main, side)
        return self.all_reduce_async(t, op)

    def all_reduce_async(self, t: torch.Tensor, op: str = "sum"):
        self.all_reduce_(t, op)
        return _Done()

    def all_reduce_bucket_(self, t: torch.Tensor, op: str = "sum"):
        self.all_reduce_(t, op)
        return _Done()

    def all_gather_cat(self, t: torch.Tensor, dim: int = 0) -> torch.Tensor:
        return torch.cat([t] * self.world_size, dim=dim)

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        return t

    def broadcast_object(self, obj, src: int = 0):
        return obj

    def all_gather_object(self, obj) -> list:
        return [obj] * self.world_size

    def max_scalar(self, v: float) -> float:
        return v

    def shutdown(self) -> None:
        p2p = self.p2p or self._p2p_dead
        if p2p is not None:
            p2p.close()
        self.p2p = self._p2p_dead = None


class _Done:
    def wait(self):
        return True


class _StreamJoin:
    """Handle of a side-stream collective: wait() makes the main stream wait."""

    def __init__(self, main, side):
        self.main, self.side = main, side

    def wait(self):
        self.main.wait_stream(self.side)
        return True


class Timer:
    def __init__(self):
        self.t = {}

    def __call__(self, name):
        timer = self

        class _Ctx:
            def __enter__(self_):
                self_.t0 = time.perf_counter()

            def __exit__(self_, *a):
                timer.t[name] = timer.t.get(name, 0.0) + time.perf_counter() - self_.t0

        return _Ctx()
