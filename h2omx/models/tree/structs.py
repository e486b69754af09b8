"""Binary layouts shared with ``csrc/tree_kernels.hip`` (checked at load time)."""
from __future__ import annotations

import ctypes

import numpy as np

TREE_NODE_DTYPE = np.dtype([
    ("feat", "<i4"), ("bin", "<i4"), ("left", "<i4"), ("na_left", "<i4"),
    ("thr", "<f4"), ("value", "<f4"), ("gain", "<f4"), ("weight", "<f4"),
])
NODE_LINK_BYTES = 16
PART_INFO_BYTES = 32
FEAT_BEST_BYTES = 64


class SplitParams(ctypes.Structure):
    _fields_ = [
        ("mode", ctypes.c_int), ("leaf_mode", ctypes.c_int), ("F", ctypes.c_int), ("is_last_level", ctypes.c_int),
        ("min_rows", ctypes.c_double), ("min_child_weight", ctypes.c_double), ("lambda_", ctypes.c_double),
        ("alpha", ctypes.c_double), ("gamma", ctypes.c_double), ("min_split_improvement", ctypes.c_double),
        ("learn_rate", ctypes.c_double), ("max_abs_leaf", ctypes.c_double),
        ("seed", ctypes.c_uint32), ("tree_index", ctypes.c_int), ("depth", ctypes.c_int),
        ("col_rate", ctypes.c_float), ("mtries", ctypes.c_int), ("children_leaves", ctypes.c_int),
        ("pad2", ctypes.c_int), ("mono", ctypes.c_void_p), ("gbound", ctypes.c_void_p),
        ("ifsets", ctypes.c_void_p), ("istate", ctypes.c_void_p),
    ]


class GradParams(ctypes.Structure):
    _fields_ = [
        ("dist", ctypes.c_int), ("apply_tree", ctypes.c_int), ("sample_rate", ctypes.c_float),
        ("seed", ctypes.c_uint32), ("tree_index", ctypes.c_int), ("tweedie_power", ctypes.c_float),
        ("quantile_alpha", ctypes.c_float), ("huber_delta", ctypes.c_float), ("row_base", ctypes.c_int64),
        ("skip_nid", ctypes.c_int), ("pad", ctypes.c_int),
    ]


def interaction_masks(sets, F: int) -> np.ndarray:
    """Per-feature bit masks of the interaction sets holding it (uint64; 0 =
    unlisted: such a feature only interacts with itself).  ``sets`` holds
    feature indices; at most 64 sets."""
    if len(sets) > 64:
        raise ValueError(f"interaction_constraints: at most 64 sets, got {len(sets)}")
    m = np.zeros(F, np.uint64)
    for si, st in enumerate(sets):
        for f in st:
            if not 0 <= int(f) < F:
                raise ValueError(f"interaction_constraints: feature index {f} out of range")
            m[int(f)] |= np.uint64(1) << np.uint64(si)
    return m


def interaction_allowed(state, fsets: np.ndarray, f: int) -> bool:
    """Mirror of inter_ok (csrc/tree_kernels.hip): state = (set mask, solo)."""
    mask, solo = state
    if solo == -2:
        return True
    if solo >= 0:
        return f == solo
    return bool(int(fsets[f]) & mask)


def interaction_child(state, fsets: np.ndarray, f: int):
    """Mirror of inter_children: the state both children of a split on f get."""
    mask, solo = state
    fs = int(fsets[f])
    if fs == 0:
        return (0, f)
    comp = (1 << 64) - 1 if solo == -2 else mask
    return (comp & fs, -1)


# distribution codes of boost_update_kernel
DIST_CODES = {
    "gaussian": 0, "bernoulli": 1, "poisson": 2, "gamma": 3, "tweedie": 4,
    "laplace": 5, "quantile": 6, "huber": 7, "drf": 8,
}


def check_layout(lib) -> None:
    sizes = (ctypes.c_int * 8)()
    lib.h2omx_tree_sizes(sizes)
    want = [ctypes.sizeof(SplitParams), FEAT_BEST_BYTES, NODE_LINK_BYTES, PART_INFO_BYTES,
            TREE_NODE_DTYPE.itemsize, ctypes.sizeof(GradParams)]
    got = list(sizes)[:6]
    if got != want:
        raise RuntimeError(f"tree kernel ABI mismatch: kernel sizes {got} != python {want}")
