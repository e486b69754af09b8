"""Host-side stateless hashes shared by the GPU engine's host code (per-tree
column masks) and the CPU reference builder; identical to common.h mix32 /
hash4 / u01 on the device, so both draw the same samples."""
from __future__ import annotations

import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def _mix32(x):
    x = np.asarray(x, dtype=np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x


def hash4(a, b, c, d):
    a, b, c, d = (np.asarray(v, dtype=np.uint64) & M32 for v in (a, b, c, d))
    return _mix32(a ^ _mix32(b ^ _mix32(c ^ _mix32((d + np.uint64(0x9E3779B9)) & M32))))


def u01(hv):
    return (np.asarray(hv, dtype=np.uint64) >> np.uint64(8)).astype(np.float64) * (1.0 / 16777216.0)
