"""Typed bindings of the native kernel libraries.

Each binding is declared with a compact signature string so every ctypes
argument has an explicit C type (``P`` pointer, ``I`` int32, ``L`` int64,
``F`` float, ``D`` double, ``S`` hipStream_t).  ``ops.tree`` / ``ops.dense`` /
``ops.metrics`` return the bound libraries; on a GPU tensor the HIP path is
the only path (missing libraries raise :class:`NativeLibraryMissing`).
"""
from __future__ import annotations

import ctypes

from .. import _native

_CT = {"P": ctypes.c_void_p, "I": ctypes.c_int, "L": ctypes.c_int64, "F": ctypes.c_float,
       "D": ctypes.c_double, "S": ctypes.c_void_p, "U": ctypes.c_uint32}

TREE_SIGS = {
    "h2omx_tree_sizes": "P",
    "h2omx_bin_features": "PLLIPPIPLS",
    "h2omx_hist_build": "PLPPPPPPPIIIIIIIIIIPPIPS",
    "h2omx_hist_reduce": "PIIIIIIIPPS",
    "h2omx_hist_build_route": "PLPPPPIPPPIIIIIIIIIPIPS",
    "h2omx_hist_build_grad": "PLPPPIIIIIIIIIPPPPPPIPPIIIPS",
    "h2omx_split_find": "PPPPPPPPPIIPS",
    "h2omx_reduce_split": "PIIIIPPPPPPPPIPS",
    "h2omx_reduce_split_p2p": "PPIIIPPPPPPPPIIPPIPPPIPPS",
    "h2omx_reduce_split_fin": "PIIIPPPPPPPPIPPPIPPPIPPS",
    "h2omx_node_best_finalize_p2p": "PPPPPPIIPPPIPS",
    "h2omx_leaf_finalize_p2p": "PPPPPPIIPIIPPLPS",
    "h2omx_level_finalize": "PPPPPPIIPPPIPIPS",
    "h2omx_partition": "PLPPIPPPPIPPPIIIPS",
    "h2omx_partition_blocks": "",
    "h2omx_partition_final": "PLPPPIPPPPIPPPIPPPIPS",
    "h2omx_partition_route": "PLPPPIPPIPIS",
    "h2omx_leaf_reduce": "PIIPS",
    "h2omx_boost_update": "PPPLLPPPPPPPLPIPIPPIIPPS",
    "h2omx_apply_tree": "PLPPS",
    "h2omx_tree_archive": "PLPIPS",
    "h2omx_sketch_bins": "",
    "h2omx_sketch": "PLIIIPIPPPPPPPPPPPPS",
    "h2omx_softmax_grad": "PILPPLLIPPPPPPS",
    "h2omx_oob_accumulate": "PPLPPPUIFLIS",
    "h2omx_stat_blocks": "",
    "h2omx_stat_reduce": "PPS",
    "h2omx_tree_begin": "PIIPPPPILIPS",
    "h2omx_leaf_stats": "PPPPLPIPS",
    "h2omx_leaf_finalize": "PPPPPIS",
    "h2omx_leaf_finalize_begin": "PPPPPIPIIPPLPS",
    "h2omx_leaf_finalize_mono": "PPPPPIPS",
    "h2omx_predict_raw": "PLLPPIIPLPS",
    "h2omx_predict_binned": "PLLPPIIIPLPS",
    "h2omx_pc_rows": "",
    "h2omx_tree_begin_seg": "PIIPPPPIPIIIPPPPPLIPS",
    "h2omx_bag_compact": "PLPPPPPPPPPIS",
    "h2omx_bag_route_out": "PLPIPIPS",
    "h2omx_hist_build_seg": "PIPPPPPPPPPIIIIIIIIPIPPS",
    "h2omx_hist_reduce_seg": "PPPPIIIIIIPS",
    "h2omx_part_count": "PLPPPPPPIIPIPPIPPIPS",
    "h2omx_level_close": "PPPPPPPPPPPPPPIPIS",
    "h2omx_level_close_mb": "PPPPPPPPPPPPPPIPIIIPPPPPS",
    "h2omx_part_scatter": "PLPPPIPPPPPPPIPPPPIPIIPPPPPPIPPPPIPPS",
    "h2omx_seg_direct": "PIPPPPPPPPPIPIIIPIPPPPIPIPPPLS",
    "h2omx_seg_colmajor": "PIIPILPLS",
    "h2omx_codes_rowmajor": "PLILPIS",
    "h2omx_level_finalize_ns": "PPPPPPIIPPPIIPS",
    "h2omx_direct_dp_stride": "PI",
    "h2omx_direct_dp": "IPIPPPPPPPPPPIIIPPIPS",
}

DENSE_SIGS = {
    "h2omx_dense_sizes": "P",
    "h2omx_glm_irls": "PLLPPPPPPIIPPS",
    "h2omx_slab_reduce_upper": "PIIPS",
    "h2omx_glm_irls_wave": "PLLPPPPPPILPPS",
    "h2omx_glm_irls_split": "PLLPPPPPPILPPS",
    "h2omx_slab_reduce16_dev": "PIIPPS",
    "h2omx_adadelta_fix": "PPPPLFFFPS",
    "h2omx_out_wgrad_partial": "PPPIIIIS",
    "h2omx_gemm_skinny_softmax": "PPPPIIIPPS",
    "h2omx_out_backward": "PPPPPPIIIIIS",
    "h2omx_slab_reduce16": "PIIPS",
    "h2omx_slab_sum": "PIIPS",
    "h2omx_slab_sum_f32": "PIIPS",
    "h2omx_kmeans": "PLLIPPIIPPS",
    "h2omx_kmeans_wave": "PLLIPPPIIIIPPS",
    "h2omx_kmeans_mfma": "PLLIPPIIIIIPPS",
    "h2omx_glm_wz": "PLPPPPPPPPIS",
    "h2omx_glm_grad": "PLLPPPPPPPIPIS",
    "h2omx_glm_grad_max_k": "",
    "h2omx_glm_aug": "PILPPPPS",
    "h2omx_kmeans_stage": "PLILLPS",
    "h2omx_kmeans_argmin": "PILPPIPPIS",
    "h2omx_kmeans_onehot": "PILPS",
    "h2omx_gemm": "PPPPIIIIIIFIPS",
    "h2omx_act_backward": "PPLIS",
    "h2omx_gemm_skinny_nt": "PPPPIIIIS",
    "h2omx_gemm_set_tile": "I",
    "h2omx_gemm_set_full": "I",
    "h2omx_gemm_thin_k": "PPPLIIPIS",
    "h2omx_act_backward_bias": "PPPIIIIS",
    "h2omx_gemm_dact": "PPPPPIIIIIPS",
    "h2omx_out_wgrad": "PPPPIIIIS",
    "h2omx_thin_dact": "PPPPPIIIIIS",
    "h2omx_gemm_wgrad_bias": "PPPIIIIPPIIPS",
    "h2omx_bias_grad": "PPIIPIS",
    "h2omx_softmax_xent": "PPPPIIS",
    "h2omx_adadelta": "PPPPLFFFS",
    "h2omx_sgd_momentum": "PPPLFFFS",
    "h2omx_gemm_bf16": "PIPIIIIPIPIIPPIPIFIPPS",
    "h2omx_cvt_bf16_multi": "PIIIS",
    "h2omx_gemm_bf16_variant": "I",
    "h2omx_softmax_xent_bf16": "PPPIPIPIIS",
    "h2omx_cvt_bf16": "PIIIPIPIS",
    "h2omx_rowsum_bf16": "PIIIPS",
}

METRICS_SIGS = {
    "h2omx_auc_hist": "PPPLIDDPS",
}

EXPLAIN_SIGS = {
    "h2omx_tree_shap": "PLLIPIPPIPPS",
}

P2P_SIGS = {
    "h2omx_p2p_allreduce": "PPLIIS",
    "h2omx_p2p_desc_bytes": "",
    "h2omx_p2p_clock_khz": "",
    "h2omx_p2p_max_ranks": "",
    "h2omx_p2p_flags_bytes": "",
    "h2omx_p2p_alloc": "LIP",
    "h2omx_p2p_free": "P",
    "h2omx_p2p_host_alloc": "LPP",
    "h2omx_p2p_host_free": "P",
    "h2omx_p2p_handle_bytes": "",
    "h2omx_p2p_get_handle": "PP",
    "h2omx_p2p_open_handle": "PP",
    "h2omx_p2p_close_handle": "P",
    "h2omx_p2p_enable_peers": "",
}

_bound: dict[str, ctypes.CDLL] = {}


def _bind(name: str, sigs: dict[str, str]) -> ctypes.CDLL:
    lib = _bound.get(name)
    if lib is not None:
        return lib
    lib = _native.require(name)
    for fn, sig in sigs.items():
        f = getattr(lib, fn, None)
        if f is None:
            continue
        f.argtypes = [_CT[c] for c in sig]
        f.restype = ctypes.c_int
    _bound[name] = lib
    return lib


def tree_lib() -> ctypes.CDLL:
    lib = _bind("tree", TREE_SIGS)
    lib.h2omx_direct_dp_stride.restype = ctypes.c_int64
    return lib


def dense_lib() -> ctypes.CDLL:
    return _bind("dense", DENSE_SIGS)


def metrics_lib() -> ctypes.CDLL:
    return _bind("metrics", METRICS_SIGS)


def explain_lib() -> ctypes.CDLL:
    return _bind("explain", EXPLAIN_SIGS)


def p2p_lib() -> ctypes.CDLL:
    lib = _bind("p2p", P2P_SIGS)
    lib.h2omx_p2p_flags_bytes.restype = ctypes.c_int64
    return lib


P = _native.ptr
check = _native.check
stream = _native.stream_of
