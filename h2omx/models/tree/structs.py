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
        ("catf", ctypes.c_void_p), ("fbcat", ctypes.c_void_p), ("treecat", ctypes.c_void_p),
        ("edges", ctypes.c_void_p), ("frange", ctypes.c_void_p), ("hist_mode", ctypes.c_int),
        ("hist_top", ctypes.c_int), ("hist_nbins", ctypes.c_int), ("pad3", ctypes.c_int),
    ]


# TreeNode.na_left bit 1: categorical group split (the tree's bitset table holds
# the LEFT set of level codes, 8 x uint32 per node)
NA_LEFT_BIT, CAT_SPLIT_BIT = 1, 2
CAT_WORDS = 8


def bitset_words(levels) -> np.ndarray:
    """8 uint32 words with the bits of ``levels`` (codes 0..255) set."""
    w = np.zeros(CAT_WORDS, np.uint32)
    for b in np.asarray(levels, np.int64).ravel():
        w[b >> 5] |= np.uint32(1) << np.uint32(b & 31)
    return w


def bitset_has(words: np.ndarray, codes: np.ndarray) -> np.ndarray:
    """Membership of integer ``codes`` (out of 0..255: False) in bitsets
    ``words`` [..., 8] (broadcast against codes)."""
    c = np.asarray(codes, np.int64)
    ok = (c >= 0) & (c <= 255)
    cc = np.where(ok, c, 0)
    word = np.take_along_axis(np.asarray(words, np.uint32), (cc >> 5)[..., None], axis=-1)[..., 0] \
        if np.ndim(words) > 1 else np.asarray(words, np.uint32)[cc >> 5]
    return ok & (((word >> (cc & 31).astype(np.uint32)) & np.uint32(1)) != 0)


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


class TreeWalker:
    """Device-side routing of raw feature values through one tree's records
    (Python scoring helpers: leaf assignment, RuleFit rules, ...), numeric
    thresholds and categorical group splits alike."""

    def __init__(self, tree: np.ndarray, catbits: np.ndarray | None, dev):
        import torch

        self.feat = torch.from_numpy(tree["feat"].astype(np.int64)).to(dev)
        self.thr = torch.from_numpy(tree["thr"].astype(np.float32)).to(dev)
        self.left = torch.from_numpy(tree["left"].astype(np.int64)).to(dev)
        nl = tree["na_left"].astype(np.int64)
        self.nal = torch.from_numpy((nl & NA_LEFT_BIT) != 0).to(dev)
        self.iscat = torch.from_numpy((nl & CAT_SPLIT_BIT) != 0).to(dev)
        self.cb = None
        if catbits is not None and bool(self.iscat.any()):
            self.cb = torch.from_numpy(np.asarray(catbits, np.uint32).astype(np.int64)).to(dev)

    def go_left(self, idx, v):
        import torch

        nan = torch.isnan(v)
        res = torch.where(nan, self.nal[idx], v <= self.thr[idx])
        if self.cb is not None:
            cat = self.iscat[idx] & ~nan
            c = torch.nan_to_num(v, nan=-1.0).long()
            oor = (c < 0) | (c > 255)
            cc = c.clamp(0, 255)
            word = self.cb[idx.clamp(max=self.cb.shape[0] - 1), cc >> 5]
            inset = ((word >> (cc & 31)) & 1) != 0
            res = torch.where(cat, torch.where(oor, self.nal[idx], inset), res)
        return res
