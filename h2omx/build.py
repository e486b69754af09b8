"""Build the in-tree native libraries.

    python -m h2omx.build            # incremental
    python -m h2omx.build --force    # rebuild everything

HIP kernels are compiled for gfx950 (MI355X / CDNA4) only; host C++ with g++.
Outputs land in ``h2omx/lib`` so they travel with the source tree.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

from ._native import HOST_LIBS, KERNEL_LIBS, _LIB_DIR, lib_path

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ARCH = os.environ.get("H2OMX_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm install expected at /opt/rocm)")


def _stale(out: str, srcs: list[str]) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    deps = list(srcs)
    for d in (CSRC, os.path.join(CSRC, "host")):
        if os.path.isdir(d):
            deps += [os.path.join(d, f) for f in os.listdir(d) if f.endswith((".h", ".hpp"))]
    return any(os.path.getmtime(s) > t for s in deps if os.path.exists(s))


def build_kernel_lib(name: str, force: bool = False, verbose: bool = False) -> str | None:
    srcs = [os.path.join(CSRC, s) for s in KERNEL_LIBS[name]]
    if not all(os.path.exists(s) for s in srcs):
        return None
    out = lib_path(name)
    if not force and not _stale(out, srcs):
        return out
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC",
           "-munsafe-fp-atomics", "-I", CSRC, "-o", out + ".tmp", *srcs]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build_host_lib(name: str, force: bool = False, verbose: bool = False) -> str | None:
    srcs = [os.path.join(CSRC, s) for s in HOST_LIBS[name]]
    if not all(os.path.exists(s) for s in srcs):
        return None
    out = lib_path(name)
    if not force and not _stale(out, srcs):
        return out
    cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-pthread", "-I", CSRC, "-o", out + ".tmp", *srcs]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build_all(force: bool = False, verbose: bool = False) -> list[str]:
    os.makedirs(_LIB_DIR, exist_ok=True)
    jobs = [(build_kernel_lib, n) for n in KERNEL_LIBS] + [(build_host_lib, n) for n in HOST_LIBS]
    with ThreadPoolExecutor(max_workers=min(4, len(jobs))) as ex:
        outs = list(ex.map(lambda j: j[0](j[1], force, verbose), jobs))
    return [o for o in outs if o]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    for o in build_all(a.force, a.verbose):
        print(o)
    return 0


if __name__ == "__main__":
    sys.exit(main())
