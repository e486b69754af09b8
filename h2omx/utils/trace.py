"""Tracing and per-phase GPU timers.

* ``trace.range(name)`` — a roctx range (``librocprofiler-sdk-roctx``) so
  ``rocprofv3 --marker-trace`` shows algorithm phases around the kernels;
  enabled with ``H2OMX_ROCTX=1`` (no cost otherwise).
* :class:`PhaseTimer` — HIP-event timers per named phase, recorded on the
  current stream without host synchronisation and resolved once at the end
  of a job (``H2OMX_PHASE_TIMERS=1`` or ``PhaseTimer(enabled=True)``); the
  totals land in the model's ``timings`` output.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_roctx = None
_ENABLED = os.environ.get("H2OMX_ROCTX") == "1"


def _lib():
    global _roctx
    if _roctx is None:
        for name in ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
                     "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so.4"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePop.argtypes = []
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _roctx = lib
                break
            except OSError:
                continue
        else:
            _roctx = False
    return _roctx or None


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    lib = _lib() if _ENABLED else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _lib() if _ENABLED else None
    if lib is not None:
        lib.roctxMarkA(name.encode())


class PhaseTimer:
    """Accumulates GPU time per phase with HIP events (no host sync until
    :meth:`totals`)."""

    def __init__(self, enabled: bool | None = None, device=None):
        self.enabled = (os.environ.get("H2OMX_PHASE_TIMERS") == "1") if enabled is None else enabled
        self.device = device
        self.pending: list[tuple[str, object, object]] = []
        self.acc: dict[str, float] = {}

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            with range(name):
                yield
            return
        import torch

        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        with range(name):
            yield
        b.record()
        self.pending.append((name, a, b))
        if len(self.pending) > 4096:
            self._drain()

    def _drain(self):
        for name, a, b in self.pending:
            b.synchronize()
            self.acc[name] = self.acc.get(name, 0.0) + a.elapsed_time(b)
        self.pending.clear()

    def totals(self) -> dict:
        """Milliseconds per phase."""
        self._drain()
        return {k: round(v, 4) for k, v in sorted(self.acc.items())}
