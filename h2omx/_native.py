"""Loader for the in-tree native libraries (HIP kernels for gfx950 + host C++).

The kernels are built by ``python -m h2omx.build`` (also run by
``__graft_entry__.build()``) into ``h2omx/lib/*.so`` and are called through a
flat C ABI with raw device pointers and the caller's HIP stream (the PyTorch
current stream), so kernel launches interleave correctly with PyTorch ops and
RCCL collectives issued by ``torch.distributed``.

On a GPU device the HIP path is mandatory: :func:`require` raises if a
library is missing instead of silently falling back.
"""
from __future__ import annotations

import ctypes
import os
import threading

_LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
_lock = threading.Lock()
_libs: dict[str, ctypes.CDLL] = {}

# library name -> source files (relative to h2omx/csrc)
KERNEL_LIBS = {
    "tree": ["tree_kernels.hip", "sketch_kernels.hip"],
    "dense": ["dense_kernels.hip", "kmeans_wave.hip"],
    "metrics": ["metrics_kernels.hip"],
    "explain": ["explain_kernels.hip"],
    "p2p": ["p2p_kernels.hip"],
    "mlp": ["mlp_kernels.hip"],
}
HOST_LIBS = {
    "host": ["host/parser.cpp", "host/solvers.cpp"],
}


class NativeLibraryMissing(RuntimeError):
    pass


def lib_path(name: str) -> str:
    # H2OMX_LIB_DIR: load kernel-tuning variants built elsewhere (sweeps)
    return os.path.join(os.environ.get("H2OMX_LIB_DIR") or _LIB_DIR, f"libh2omx_{name}.so")


def available(name: str) -> bool:
    return os.path.exists(lib_path(name))


def require(name: str) -> ctypes.CDLL:
    """Load ``libh2omx_<name>.so`` (raise loudly if it has not been built)."""
    with _lock:
        lib = _libs.get(name)
        if lib is not None:
            return lib
        path = lib_path(name)
        if not os.path.exists(path) and name in HOST_LIBS:
            # host C++ (no GPU code): cheap to build on first use
            from .build import build_host_lib

            os.makedirs(_LIB_DIR, exist_ok=True)
            build_host_lib(name)
        if not os.path.exists(path):
            raise NativeLibraryMissing(
                f"{path} is missing: build the native kernels with `python -m h2omx.build` "
                "(hipcc --offload-arch=gfx950)")
        if name in KERNEL_LIBS:
            # make sure the HIP runtime PyTorch uses is the one our code objects
            # bind to (soname libamdhip64.so.7 is shared)
            import torch  # noqa: F401
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        _libs[name] = lib
        return lib


def loaded_libraries() -> list[str]:
    return sorted(lib_path(n) for n in _libs)


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"h2omx native call {what} failed with status {rc}")


def ptr(t) -> ctypes.c_void_p:
    """Raw data pointer of a tensor/array (None -> NULL)."""
    if t is None:
        return ctypes.c_void_p(0)
    if hasattr(t, "data_ptr"):
        return ctypes.c_void_p(t.data_ptr())
    return ctypes.c_void_p(t.ctypes.data)


def stream_of(device) -> ctypes.c_void_p:
    import torch

    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
