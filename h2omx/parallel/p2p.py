"""One-shot P2P all-reduce over IPC-mapped HBM (``csrc/p2p_kernels.hip``).

The latency-bound messages of the data plane (tree level histograms and leaf
sums, GLM Gram, metrics) do not need a ring: every rank maps
every peer's symmetric buffer once (``hipIpcGetMemHandle`` handles exchanged
over the process group), and one kernel launch per collective copies the
local shard in, posts an epoch flag to each peer, waits for the peers' flags
and sums the N buffers in rank order.  The launch has no per-call host state
(the epoch is a device counter), so it is captured in the tree step's HIP
graph: an N-rank tree is one graph replay with zero host-issued collectives.
RCCL stays in charge of large messages (DL gradients > ``cap``) and is the
fallback whenever IPC mapping or the start-up self-test fails.

On one 8-GPU node the peers are reached over xGMI; two ranks sharing one GPU
(the development box) map the same HBM through IPC, which exercises the same
code path (the multi-rank GPU tests use that).

The tree engine runs its level-histogram and leaf-sum exchanges inside its
own kernels over the same buffers and epoch (``csrc/p2p_device.h``): an N-rank
level is one ``reduce_split_p2p`` launch - a reduce-scatter of the level's
histogram rows by feature (rank r owns the features f = r mod N and scans only
those) with an all-gather of the split records - plus the level finalisation,
exactly the launches of the single-rank level.  Every exchange PUSHES: a rank
writes its bytes into the consumer's buffer (write-through, system scope) and
reads only its own buffer, so no kernel waits on a remote read over xGMI.

Contract: every rank calls :meth:`all_reduce_` (and the fused tree kernels)
with the same sequence of (numel, dtype, op), as with any collective.  A peer
that never arrives makes each poll give up after ``timeout_s``; the kernel
then sets the device error word AND a pinned host word, every later
collective stops waiting, and :meth:`failed` (a plain host read, no device
sync) reports it - ``Comm._check`` turns it into ``PeerLost`` at the next
step, graph flush or collective, and P2P is disabled for good on that Comm
(the epochs of the ranks can no longer be trusted).

Memory kinds (``P2PAllReduce.SYM_KIND``): the symmetric data buffers are fine-grained
device memory by default, so a peer's read over xGMI is coherent at system
scope by allocation type, not by relying on the writer's L2 write-back
reaching the remote reader; ``coarse`` (plain hipMalloc) and ``uncached`` are
the A/B alternatives.  Flags are always uncached.

Loopback (:meth:`P2PAllReduce.loopback`): one process stands in for N ranks
(every "peer" buffer is its own), so the N-rank launch sequence of a tree
step - same kernels, same grids, N-way sums read from HBM - runs and is timed
on one GPU (``bench.py --loopback-ranks N``); only the xGMI link is missing.
"""
from __future__ import annotations

import ctypes
import os

import torch

from .. import ops

DTYPES = {torch.int64: 0, torch.float32: 1, torch.float64: 2, torch.int32: 3}
OPS = {"sum": 0, "max": 1}
SYM_KINDS = {"coarse": 0, "uncached": 1, "fine": 2}


class P2PUnavailable(RuntimeError):
    pass


class P2PAllReduce:
    """Symmetric buffers + flags of one process group; see module docstring."""

    DEFAULT_CAP = 8 << 20      # bytes per parity: Airlines depth-6 last level = 32 x 127 KB = 4 MB
    # symmetric-buffer memory kind: fine-grained by default; coarse / uncached
    # measured within noise on one GPU (profiles/r5/p2p/README.md)
    SYM_KIND = "fine"

    def __init__(self, comm, cap_bytes: int | None = None, timeout_s: float | None = None,
                 loopback: bool = False):
        if comm.world_size < 2 or comm.device.type != "cuda":
            raise P2PUnavailable("P2P all-reduce needs >= 2 ranks on GPUs")
        lib = ops.p2p_lib()
        if comm.world_size > lib.h2omx_p2p_max_ranks():
            raise P2PUnavailable(f"world {comm.world_size} > {lib.h2omx_p2p_max_ranks()} ranks")
        self.lib, self.comm = lib, comm
        self.world, self.rank = comm.world_size, comm.rank
        self.loopback = loopback
        self.cap = int(cap_bytes or int(os.environ.get("H2OMX_P2P_CAP_MB", "0")) << 20 or self.DEFAULT_CAP)
        self.timeout_s = float(timeout_s if timeout_s is not None else os.environ.get("H2OMX_P2P_TIMEOUT_S", "20"))
        kind = self.SYM_KIND
        if kind not in SYM_KINDS:
            raise ValueError(f"P2PAllReduce.SYM_KIND={kind!r}: expected one of {sorted(SYM_KINDS)}")
        self.sym_kind = kind
        self.calls = 0
        self._own: list[int] = []       # pointers this rank allocated
        self._opened: list[int] = []    # peer pointers this rank mapped
        self._host: int | None = None   # pinned error word (host address)
        self._err_word = None
        with torch.cuda.device(comm.device):
            # two exchange parities + the tree level's split-record table (2 x cap / 2)
            sym = self._alloc(3 * self.cap, SYM_KINDS[kind])
            flags = self._alloc(int(lib.h2omx_p2p_flags_bytes()), SYM_KINDS["uncached"])
            # control words live in torch memory: [epoch, ticket, error, timeouts]
            self.ctrl = torch.zeros((4,), dtype=torch.int32, device=comm.device)
            h, dv = ctypes.c_void_p(), ctypes.c_void_p()
            if lib.h2omx_p2p_host_alloc(64, ctypes.addressof(h), ctypes.addressof(dv)) != 0 or not h.value:
                raise P2PUnavailable("pinned host error word allocation failed")
            self._host, host_dev = h.value, dv.value
            self._err_word = ctypes.c_uint32.from_address(self._host)
            if loopback:
                syms, flgs = [sym] * self.world, [flags] * self.world
            else:
                lib.h2omx_p2p_enable_peers()
                hb = lib.h2omx_p2p_handle_bytes()
                mine = [self._handle(sym, hb), self._handle(flags, hb)]
                # every rank's handles (small control data over the process group)
                allh = comm.all_gather_object(mine)
                syms, flgs = [], []
                for r, (hs, hf) in enumerate(allh):
                    if r == self.rank:
                        syms.append(sym)
                        flgs.append(flags)
                    else:
                        syms.append(self._open(hs))
                        flgs.append(self._open(hf))
        khz = lib.h2omx_p2p_clock_khz()
        if khz <= 0:
            khz = 100_000
        R = lib.h2omx_p2p_max_ranks()

        class Desc(ctypes.Structure):
            _fields_ = [("sym", ctypes.c_void_p * R), ("flags", ctypes.c_void_p * R), ("ctrl", ctypes.c_void_p),
                        ("host_err", ctypes.c_void_p), ("cap", ctypes.c_int64), ("timeout_ticks", ctypes.c_int64),
                        ("world", ctypes.c_int32), ("rank", ctypes.c_int32), ("loopback", ctypes.c_int32),
                        ("pad", ctypes.c_int32)]

        if ctypes.sizeof(Desc) != lib.h2omx_p2p_desc_bytes():
            raise P2PUnavailable("P2PDesc layout mismatch")
        d = Desc()
        for r in range(self.world):
            d.sym[r], d.flags[r] = syms[r], flgs[r]
        d.ctrl = self.ctrl.data_ptr()
        d.host_err = host_dev
        d.cap = self.cap
        d.timeout_ticks = int(self.timeout_s * khz * 1000)
        d.world, d.rank = self.world, self.rank
        d.loopback = 1 if loopback else 0
        self.desc = d

    @classmethod
    def loopback_for(cls, comm, cap_bytes: int | None = None) -> "P2PAllReduce":
        """One process standing in for ``comm.world_size`` ranks (see module docstring)."""
        return cls(comm, cap_bytes=cap_bytes, loopback=True)

    @property
    def desc_ptr(self) -> int:
        """Host address of the P2PDesc image (the fused tree kernels take it by value)."""
        return ctypes.addressof(self.desc)

    def failed(self) -> bool:
        """True once any poll of this process timed out (pinned host word: no device sync)."""
        return self._err_word is not None and self._err_word.value != 0

    # -- setup helpers -------------------------------------------------------
    def _alloc(self, nbytes: int, kind: int) -> int:
        p = ctypes.c_void_p()
        rc = self.lib.h2omx_p2p_alloc(nbytes, kind, ctypes.addressof(p))
        if rc != 0 or not p.value:
            raise P2PUnavailable(f"symmetric buffer allocation failed ({rc})")
        self._own.append(p.value)
        return p.value

    def _handle(self, ptr: int, hb: int) -> bytes:
        buf = ctypes.create_string_buffer(hb)
        rc = self.lib.h2omx_p2p_get_handle(ptr, ctypes.addressof(buf))
        if rc != 0:
            raise P2PUnavailable("hipIpcGetMemHandle failed")
        return buf.raw

    def _open(self, h: bytes) -> int:
        buf = ctypes.create_string_buffer(h, len(h))
        p = ctypes.c_void_p()
        rc = self.lib.h2omx_p2p_open_handle(ctypes.addressof(buf), ctypes.addressof(p))
        if rc != 0 or not p.value:
            raise P2PUnavailable("hipIpcOpenMemHandle failed (peer memory not mappable from this process)")
        self._opened.append(p.value)
        return p.value

    # -- collective ------------------------------------------------------------
    def supports(self, t: torch.Tensor, op: str = "sum") -> bool:
        return (t.is_cuda and t.device == self.comm.device and t.dtype in DTYPES and op in OPS
                and t.is_contiguous() and t.numel() * t.element_size() <= self.cap
                and t.data_ptr() % 16 == 0)

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """In-place all-reduce on the current stream (graph-capturable)."""
        if not self.supports(t, op):
            raise ValueError("tensor not supported by the P2P all-reduce")
        self.calls += 1
        rc = self.lib.h2omx_p2p_allreduce(ctypes.addressof(self.desc), t.data_ptr(), t.numel(), DTYPES[t.dtype],
                                          OPS[op], ops.stream(t.device))
        ops.check(rc, "p2p_allreduce")
        return t

    def failure_reason(self) -> str:
        v = self._err_word.value if self._err_word is not None else 0
        if v == 1:
            return f"a P2P exchange timed out after {self.timeout_s:g} s waiting for a peer"
        if v == 2:
            return "a peer rank aborted its P2P exchanges (it timed out waiting for this or another rank)"
        return ""

    def check(self) -> None:
        """Raise if any poll timed out (a peer never arrived) or a peer aborted."""
        if self.failed():
            raise RuntimeError(f"P2P all-reduce: {self.failure_reason()} (rank {self.rank} of {self.world})")
        c = self.ctrl.cpu().tolist()
        if c[2] != 0:
            raise RuntimeError(f"P2P all-reduce: {c[3]} block poll(s) timed out waiting for a peer "
                               f"(rank {self.rank} of {self.world}, epoch {c[0]})")

    def self_test(self) -> bool:
        """Collective sanity check (every rank calls it): int64 / float64 sums of
        rank-dependent patterns, odd sizes included, plus a max."""
        dev = self.comm.device
        ok = True
        # loopback: every stand-in rank holds rank 0's data
        mult = self.world if self.loopback else self.world * (self.world + 1) // 2
        for n, dt in ((3, torch.int64), (4099, torch.int64), (1 << 17, torch.int64), (1001, torch.float64),
                      (16, torch.float32)):
            base = torch.arange(n, device=dev, dtype=torch.float64)
            x = ((base * 7 + 1) * (self.rank + 1)).to(dt)
            self.all_reduce_(x)
            want = ((base * 7 + 1) * mult).to(dt)
            ok &= bool(torch.equal(x, want))
        m = torch.full((5,), float(self.rank), device=dev, dtype=torch.float32)
        self.all_reduce_(m, "max")
        ok &= bool((m == float(0 if self.loopback else self.world - 1)).all())
        torch.cuda.synchronize(dev)
        ok &= int(self.ctrl[2]) == 0
        return ok

    def close(self) -> None:
        try:
            torch.cuda.synchronize(self.comm.device)
        except Exception:
            pass
        for p in self._opened:
            self.lib.h2omx_p2p_close_handle(p)
        for p in self._own:
            self.lib.h2omx_p2p_free(p)
        self._opened, self._own = [], []
        if self._host is not None:
            self._err_word = None
            self.lib.h2omx_p2p_host_free(self._host)
            self._host = None


def setup(comm, required: bool = False) -> P2PAllReduce | None:
    """Create and verify the P2P all-reduce of ``comm`` (collective: every rank
    calls it).  Returns None -- RCCL then carries everything -- when IPC
    mapping is unavailable on any rank or the self-test fails on any rank;
    ``required`` raises instead."""
    err = None
    p2p = None
    try:
        p2p = P2PAllReduce(comm)
    except Exception as e:      # noqa: BLE001 - any rank's failure disables P2P on all
        err = f"{type(e).__name__}: {e}"
    # agree on availability before any P2P kernel runs (a kernel waiting for a
    # rank that gave up would only drain by its timeout)
    errs = comm.all_gather_object(err)
    bad = [f"rank {r}: {e}" for r, e in enumerate(errs) if e]
    if not bad:
        ok = p2p.self_test()
        oks = comm.all_gather_object(bool(ok))
        if not all(oks):
            bad = [f"rank {r}: self-test mismatch" for r, o in enumerate(oks) if not o]
    if bad:
        if p2p is not None:
            p2p.close()
        if required:
            raise P2PUnavailable("; ".join(bad))
        comm.p2p_error = "; ".join(bad)
        return None
    return p2p

