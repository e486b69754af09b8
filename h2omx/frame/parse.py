"""CSV import through the native parser (csrc/host/parser.cpp).

``parse_setup`` mirrors H2O's /3/ParseSetup (separator, header, column names
and types guessed from the data); ``import_file`` mirrors /3/ImportFiles +
/3/Parse and produces a :class:`Frame`.  With ``shard=(rank, world)`` every
rank parses only its byte range of the file (split at line boundaries), the
way H2O distributes parsed chunks over the cloud.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from .. import _native
from .frame import ENUM, INT, REAL, Frame, Vec

_TYPES = {0: REAL, 1: ENUM, 2: "string"}
_TYPE_CODES = {"numeric": 0, "real": 0, "int": 0, "enum": 1, "categorical": 1, "factor": 1, "string": 2}


def _lib():
    lib = _native.require("host")
    if not getattr(lib, "_h2omx_bound", False):
        lib.h2omx_csv_parse.argtypes = [ctypes.c_char_p, ctypes.c_char, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                        ctypes.c_int64, ctypes.c_void_p, ctypes.c_int]
        lib.h2omx_csv_parse.restype = ctypes.c_void_p
        lib.h2omx_csv_parse_text.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_char, ctypes.c_int,
                                             ctypes.c_int]
        lib.h2omx_csv_parse_text.restype = ctypes.c_void_p
        for fn, res in (("h2omx_csv_error", ctypes.c_char_p), ("h2omx_csv_ncols", ctypes.c_int),
                        ("h2omx_csv_nrows", ctypes.c_int64), ("h2omx_csv_header", ctypes.c_int),
                        ("h2omx_csv_sep", ctypes.c_char)):
            getattr(lib, fn).argtypes = [ctypes.c_void_p]
            getattr(lib, fn).restype = res
        lib.h2omx_csv_colname.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib.h2omx_csv_colname.restype = ctypes.c_char_p
        lib.h2omx_csv_coltype.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib.h2omx_csv_numeric.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        lib.h2omx_csv_codes.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        lib.h2omx_csv_domain_size.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib.h2omx_csv_domain.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        lib.h2omx_csv_domain.restype = ctypes.c_char_p
        lib.h2omx_csv_free.argtypes = [ctypes.c_void_p]
        lib._h2omx_bound = True
    return lib


class _Parsed:
    def __init__(self, h):
        self.h = h
        self.lib = _lib()
        err = self.lib.h2omx_csv_error(h)
        if err:
            self.lib.h2omx_csv_free(h)
            self.h = None
            raise IOError(err.decode())

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.h2omx_csv_free(self.h)

    def setup(self) -> dict:
        lib, h = self.lib, self.h
        n = lib.h2omx_csv_ncols(h)
        return {
            "number_columns": n,
            "column_names": [lib.h2omx_csv_colname(h, j).decode() for j in range(n)],
            "column_types": ["Enum" if lib.h2omx_csv_coltype(h, j) == 1 else "Numeric" for j in range(n)],
            "separator": ord(lib.h2omx_csv_sep(h)),
            "check_header": 1 if lib.h2omx_csv_header(h) else -1,
            "nrows": lib.h2omx_csv_nrows(h),
        }

    def frame(self, device="cpu", key=None) -> Frame:
        lib, h = self.lib, self.h
        n = lib.h2omx_csv_nrows(h)
        vecs = []
        for j in range(lib.h2omx_csv_ncols(h)):
            name = lib.h2omx_csv_colname(h, j).decode()
            t = lib.h2omx_csv_coltype(h, j)
            if t == 0:
                buf = np.empty(n, np.float64)
                lib.h2omx_csv_numeric(h, j, buf.ctypes.data)
                finite = buf[~np.isnan(buf)]
                vt = INT if finite.size and np.all(np.floor(finite) == finite) else REAL
                vecs.append(Vec(name, torch.from_numpy(buf.astype(np.float32)).to(device), vt))
            else:
                codes = np.empty(n, np.int32)
                lib.h2omx_csv_codes(h, j, codes.ctypes.data)
                dom = [lib.h2omx_csv_domain(h, j, k).decode() for k in range(lib.h2omx_csv_domain_size(h, j))]
                vecs.append(Vec(name, torch.from_numpy(codes).to(device), ENUM, dom))
        return Frame(vecs, key=key)


def _parse(path, sep=None, header=None, col_types=None, shard=None, nthreads=8):
    sep_b = (sep or "\0").encode()[:1]
    hdr = -1 if header is None else (1 if header else 0)
    start, end = 0, -1
    if shard is not None:
        rank, world = shard
        size = os.path.getsize(path)
        start, end = size * rank // world, size * (rank + 1) // world
        if rank > 0 and header is None:
            hdr = 0  # only the first shard can hold the header
    forced = None
    nf = 0
    if col_types:
        arr = (ctypes.c_int * len(col_types))(*[_TYPE_CODES.get(str(t).lower(), -1) if t else -1 for t in col_types])
        forced, nf = ctypes.cast(arr, ctypes.c_void_p), len(col_types)
    h = _lib().h2omx_csv_parse(os.fsencode(path), sep_b, hdr, nthreads, start, end, forced, nf)
    return _Parsed(h)


def parse_setup(path: str, sep: str | None = None, header: bool | None = None) -> dict:
    return _parse(path, sep, header).setup()


def import_file(path: str, sep: str | None = None, header: bool | None = None, col_types=None, device="cpu",
                key=None, shard=None, col_names=None) -> Frame:
    fr = _parse(path, sep, header, col_types, shard).frame(device, key)
    if col_names:
        for v, nm in zip(fr.vecs, col_names):
            v.name = nm
    return fr


def sample_setup(path: str, sep: str | None = None, header: bool | None = None, nbytes: int = 1 << 22) -> dict:
    """ParseSetup guessed from the first ``nbytes`` of the file (cheap on big files)."""
    size = os.path.getsize(path)
    if size <= nbytes:
        return parse_setup(path, sep, header)
    with open(path, "rb") as f:
        head = f.read(nbytes)
    head = head[: head.rfind(b"\n") + 1] or head
    h = _lib().h2omx_csv_parse_text(head, len(head), (sep or "\0").encode()[:1],
                                    -1 if header is None else int(bool(header)), 8)
    return _Parsed(h).setup()


def import_shard(path: str, rank: int, world: int, setup: dict, device="cpu", key=None) -> Frame:
    """Parse rank's byte range of ``path`` with the column names / types / separator
    agreed on by the leader (``setup`` from :func:`sample_setup`)."""
    types = ["enum" if t == "Enum" else ("string" if t == "String" else "numeric") for t in setup["column_types"]]
    sep = chr(setup["separator"]) if setup.get("separator") else None
    header = setup.get("check_header") == 1
    try:
        fr = import_file(path, sep=sep, header=header if rank == 0 else False, col_types=types, device=device,
                         key=key, shard=(rank, world) if world > 1 else None, col_names=setup["column_names"])
    except IOError as e:
        if "empty" not in str(e):
            raise
        vecs = []
        for name, t in zip(setup["column_names"], types):
            if t == "enum":
                vecs.append(Vec(name, torch.zeros(0, dtype=torch.int32, device=device), ENUM, []))
            else:
                vecs.append(Vec(name, torch.zeros(0, dtype=torch.float32, device=device), REAL))
        fr = Frame(vecs, key=key)
    return fr


def parse_text(text: str, sep: str | None = None, header: bool | None = None, device="cpu", key=None) -> Frame:
    raw = text.encode()
    h = _lib().h2omx_csv_parse_text(raw, len(raw), (sep or "\0").encode()[:1],
                                    -1 if header is None else int(bool(header)), 8)
    return _Parsed(h).frame(device, key)
