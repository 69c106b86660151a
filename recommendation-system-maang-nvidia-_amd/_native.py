"""ctypes binding of librecsys_hip.so (the C-ABI declared in include/recsys_hip.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (``make -C csrc``) and ships
next to this file. There is deliberately NO fallback: if the library is missing or fails to
load, every hot-path op raises — a silent eager/CPU substitute would void the parity claims.
"""
from __future__ import annotations

import ctypes
import os
import threading
from ctypes import POINTER, c_double, c_float, c_int, c_int32, c_int64, c_size_t, c_void_p
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RECSYS_HIP_LIB", os.path.join(_HERE, "librecsys_hip.so"))
ABI_VERSION = 2

_lock = threading.Lock()
_lib: Optional[ctypes.CDLL] = None


class NativeError(RuntimeError):
    """A C-ABI entry point returned a non-zero status."""


# name -> (restype, argtypes); mirrors include/recsys_hip.h one-to-one.
_P = c_void_p
_SIGNATURES = {
    "rs_abi_version": (c_int, []),
    "rs_last_error": (ctypes.c_char_p, []),
    "rs_embedding_gather_f32": (c_int, [_P, c_int64, c_int64, _P, c_int64, _P, _P, _P]),
    "rs_embedding_gather_tables_f32": (c_int, [c_int, _P, _P, _P, _P, _P, c_int64, _P, _P]),
    "rs_embedding_gather_tables_rows_f32": (c_int, [c_int, _P, _P, _P, _P, _P, _P, _P, c_int64, _P, _P]),
    "rs_sparse_adagrad_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int64]),
    "rs_sparse_adagrad_f32": (c_int, [_P, _P, c_int64, c_int64, _P, _P, c_int64, _P, c_float, c_float,
                                      c_int64, c_float, c_float, _P, c_size_t, _P]),
    "rs_sparse_adagrad_ld_f32": (c_int, [_P, _P, c_int64, c_int64, _P, _P, c_int64, c_int64, _P, c_float,
                                         c_float, c_int64, c_float, c_float, _P, c_size_t, _P]),
    "rs_sparse_adagrad_multi_workspace_bytes": (c_size_t, [c_int, _P, c_int64]),
    "rs_sparse_adagrad_multi_f32": (c_int, [c_int, _P, _P, _P, c_int64, _P, _P, _P, _P, _P, _P, c_float, c_float,
                                            c_int64, c_float, c_float, _P, c_size_t, _P]),
    "rs_sparse_adagrad_multi_step_f32": (c_int, [c_int, _P, _P, _P, c_int64, _P, _P, _P, _P, _P, _P, c_float,
                                                 c_float, c_int64, c_float, c_float, _P, c_size_t, _P]),
    "rs_sparse_adagrad_multi_step_ordered_f32": (c_int, [c_int, _P, _P, _P, c_int64, _P, _P, _P, _P, _P, _P,
                                                         c_float, c_float, c_int64, c_float, c_float, _P, _P,
                                                         c_size_t, _P]),
    "rs_sparse_adagrad_sumsq_f32": (c_int, [_P, _P, c_int64, c_int64, _P, _P, c_int64, c_int64, _P, _P, c_float,
                                            c_float, c_int64, c_float, c_float, _P, c_size_t, _P]),
    "rs_sparse_dedupe_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int64]),
    "rs_sparse_dedupe_f32": (c_int, [_P, _P, c_int64, c_int64, c_int64, c_int64, _P, _P, _P, _P, _P, c_size_t, _P]),
    "rs_multi_embedding_gather_f32": (c_int, [_P, _P, c_int, c_int64, _P, c_int64, _P, c_int64, _P, c_int64,
                                              _P, _P]),
    "rs_gemm_f32": (c_int, [c_int, c_int, c_int64, c_int64, c_int64, _P, c_int64, _P, c_int64, _P,
                            c_int64, _P, c_int, _P, c_int64, c_float, _P]),
    "rs_gemm_prec_f32": (c_int, [c_int, c_int, c_int64, c_int64, c_int64, _P, c_int64, _P, c_int64, _P,
                                 c_int64, _P, c_int, _P, c_int64, c_float, c_int, _P]),
    "rs_gemm_splitk_prec_f32": (c_int, [c_int, c_int, c_int64, c_int64, c_int64, _P, c_int64, _P, c_int64,
                                        _P, c_int64, _P, c_float, c_int, _P, c_size_t, _P]),
    "rs_gemm_splitk_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int64]),
    "rs_gemm_splitk_f32": (c_int, [c_int, c_int, c_int64, c_int64, c_int64, _P, c_int64, _P, c_int64,
                                   _P, c_int64, _P, c_float, _P, c_size_t, _P]),
    "rs_plane_image_bytes": (c_size_t, [c_int64, c_int64]),
    "rs_plane_image_f32": (c_int, [_P, c_int64, c_int64, c_int64, c_int, _P, _P]),
    "rs_gemm_planes_prec_f32": (c_int, [c_int, c_int, c_int64, c_int64, c_int64, _P, _P, _P, c_int64, _P, c_int,
                                        c_float, c_int, _P]),
    "rs_gemm_planes_splitk_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int64]),
    "rs_gemm_planes_splitk_prec_f32": (c_int, [c_int, c_int, c_int64, c_int64, c_int64, _P, _P, _P, _P, c_float,
                                               c_int, _P, c_size_t, _P]),
    "rs_xgemm_image_dual_workspace_bytes": (c_size_t, [c_int64, c_int64]),
    "rs_xgemm_image_dual_f32": (c_int, [_P, _P, c_int64, c_int64, _P, _P, _P, _P, c_size_t, _P]),
    "rs_gemm_group_prec_f32": (c_int, [c_int, c_int, c_int, c_int64, c_int64, c_int64, _P, c_int64, _P, c_int64,
                                       _P, c_int64, _P, c_int, _P, c_int64, c_float, c_int, _P]),
    "rs_mlp_weight_image_bytes": (c_size_t, [c_int, _P]),
    "rs_mlp_weight_image_f32": (c_int, [c_int, c_int, _P, _P, _P, _P]),
    "rs_mlp_weight_images_f32": (c_int, [c_int, _P, _P, _P, _P, _P]),
    "rs_mlp_fwd_prec_f32": (c_int, [c_int, c_int, _P, c_int64, _P, _P, _P, _P, _P, c_int, _P]),
    "rs_mlp_bwd_chain_prec_f32": (c_int, [c_int, c_int, _P, c_int64, _P, _P, _P, _P, _P, c_int, _P]),
    "rs_mlp_wgrad_workspace_bytes": (c_size_t, [c_int, c_int, _P, c_int64]),
    "rs_mlp_wgrad_prec_f32": (c_int, [c_int, c_int, _P, c_int64, _P, _P, _P, _P, c_float, _P, c_int, _P, c_size_t,
                                      _P, _P]),
    "rs_gemm_group_img_prec_f32": (c_int, [c_int, c_int, c_int, c_int64, c_int64, c_int64, _P, c_int64, _P,
                                           c_int64, _P, c_int64, _P, c_int, _P, c_int64, c_float, c_int, _P, _P]),
    "rs_gemm_group_rows_prec_f32": (c_int, [c_int, c_int, c_int64, c_int64, c_int64, _P, c_int64, _P, _P,
                                            c_int64, _P, c_int64, _P, c_int, _P, c_int64, _P, _P, c_int, _P]),
    "rs_gemm_wgrad_bias_group_rows_prec_f32": (c_int, [c_int, c_int64, c_int64, c_int64, _P, c_int64, _P, _P,
                                                       c_int64, _P, c_int, _P, c_size_t, _P, _P]),
    "rs_gemm_wgrad_bias_group_workspace_bytes": (c_size_t, [c_int, c_int64, c_int64, c_int64]),
    "rs_gemm_wgrad_bias_group_prec_f32": (c_int, [c_int, c_int64, c_int64, c_int64, _P, c_int64, _P, c_int64, _P,
                                                  c_int, _P, c_size_t, _P, _P]),
    "rs_gemm_wgrad_bias_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int64]),
    "rs_gemm_wgrad_bias_prec_f32": (c_int, [c_int64, c_int64, c_int64, _P, c_int64, _P, c_int64, _P, _P, c_float, _P,
                                            c_int, _P, c_size_t, _P, _P]),
    "rs_sum_squares_multi_workspace_bytes": (c_size_t, [c_int, _P]),
    "rs_sum_squares_multi_f32": (c_int, [c_int, _P, _P, c_float, _P, _P, c_size_t, _P]),
    "rs_loss_combine_f32": (c_int, [_P, _P, _P, c_float, c_float, c_float, _P, _P]),
    "rs_loss_combine_bwd_f32": (c_int, [_P, c_float, c_float, c_float, _P, _P]),
    "rs_xgemm_image_bytes": (c_size_t, [c_int64, c_int64]),
    "rs_xgemm_image_f32": (c_int, [_P, c_int64, c_int64, c_int64, c_int, _P, _P]),
    "rs_xgemm_prec_f32": (c_int, [c_int64, c_int64, c_int64, _P, _P, _P, c_int64, _P, c_int, c_float, c_int, _P]),
    "rs_xgemm_splitk_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int64]),
    "rs_xgemm_splitk_prec_f32": (c_int, [c_int64, c_int64, c_int64, _P, _P, _P, _P, c_float, c_int, _P, c_size_t,
                                         _P]),
    "rs_colsum_workspace_bytes": (c_size_t, [c_int64, c_int64]),
    "rs_relu_bwd_colsum_f32": (c_int, [_P, _P, c_int64, c_int64, _P, _P, _P, c_size_t, _P, _P]),
    "rs_sum_squares_workspace_bytes": (c_size_t, [c_int64]),
    "rs_sum_squares_f32": (c_int, [_P, c_int64, c_float, _P, _P, c_size_t, _P]),
    "rs_dcn_cross_vec_fwd_f32": (c_int, [_P, _P, c_int64, c_int64, c_int, _P, _P, _P, _P, _P, _P]),
    "rs_dcn_cross_vec_bwd_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int]),
    "rs_dcn_cross_vec_bwd_f32": (c_int, [_P, _P, _P, _P, c_int64, c_int64, c_int, _P, _P, _P, _P, _P, _P,
                                         _P, c_size_t, _P, _P]),
    "rs_dcn_cross_vec_bwd_add_f32": (c_int, [_P, _P, _P, _P, c_int64, c_int64, c_int, _P, _P, _P, _P, _P, _P,
                                             _P, _P, _P, c_size_t, _P, _P]),
    "rs_dcn_cross_mat_fwd_f32": (c_int, [_P, c_int64, c_int64, c_int, _P, _P, _P, _P, _P]),
    "rs_dcn_cross_mat_fwd_prec_f32": (c_int, [_P, c_int64, c_int64, c_int, _P, _P, _P, _P, c_int, _P]),
    "rs_dcn_cross_mat_bwd_prec_f32": (c_int, [_P, _P, _P, _P, c_int64, c_int64, c_int, _P, _P, _P, _P, _P, c_int,
                                              _P, c_size_t, _P]),
    "rs_dcn_cross_mat_planes_bytes": (c_size_t, [c_int64, c_int64, c_int]),
    "rs_dcn_cross_mat_fwd_planes_workspace_bytes": (c_size_t, [c_int64, c_int64]),
    "rs_dcn_cross_mat_fwd_planes_x0img_f32": (c_int, [_P, c_int64, c_int64, c_int, _P, _P, _P, _P, _P, _P, c_int,
                                                      _P, c_size_t, _P]),
    "rs_dcn_cross_mat_fwd_planes_f32": (c_int, [_P, c_int64, c_int64, c_int, _P, _P, _P, _P, _P, c_int, _P, c_size_t,
                                                _P]),
    "rs_dcn_cross_mat_bwd_planes_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int]),
    "rs_dcn_cross_mat_bwd_planes_f32": (c_int, [_P, _P, _P, _P, _P, c_int64, c_int64, c_int, _P, _P, _P, _P, _P,
                                                c_int, _P, c_size_t, _P]),
    "rs_dcn_cross_mat_bwd_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int]),
    "rs_dcn_cross_mat_bwd_f32": (c_int, [_P, _P, _P, _P, c_int64, c_int64, c_int, _P, _P, _P, _P, _P, _P,
                                         c_size_t, _P]),
    "rs_heads_fwd_f32": (c_int, [_P, c_int64, _P, c_int64, c_int64, _P, _P, _P, _P, _P, _P, _P]),
    "rs_heads_bwd_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int64]),
    "rs_heads_bwd_f32": (c_int, [_P, c_int64, _P, c_int64, c_int64, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                 _P, _P, _P, _P, _P, _P, _P, c_size_t, _P, _P]),
    "rs_heads_bwd_combine_f32": (c_int, [_P, c_int64, _P, c_int64, c_int64, _P, _P, _P, _P, _P, _P, c_float,
                                         c_float, c_float, c_int, _P, _P, _P, _P, _P, _P, _P, _P, c_size_t, _P, _P]),
    "rs_ranking_losses_combine_f32": (c_int, [_P, _P, _P, _P, c_int64, c_int, c_float, c_float, c_int, _P, _P,
                                              c_float, c_float, c_float, c_int, _P, _P, _P, _P, _P, _P, c_size_t, _P]),
    "rs_ranking_losses_workspace_bytes": (c_size_t, [c_int64]),
    "rs_ranking_losses_f32": (c_int, [_P, _P, _P, _P, c_int64, c_int, c_float, c_float, c_int, _P, _P,
                                      _P, _P, c_size_t, _P]),
    "rs_inbatch_softmax_workspace_bytes": (c_size_t, [c_int64, c_int64]),
    "rs_inbatch_softmax_xent_fwd_f32": (c_int, [_P, _P, c_int64, c_int64, c_float, _P, _P, _P, _P, _P,
                                                _P, c_size_t, _P]),
    "rs_inbatch_softmax_xent_bwd_f32": (c_int, [_P, _P, c_int64, c_int64, c_float, _P, _P, _P, _P, _P,
                                                _P, c_size_t, _P]),
    "rs_adagrad_dense_workspace_bytes": (c_size_t, [c_int, c_int64]),
    "rs_adagrad_dense_f32": (c_int, [_P, c_int, c_int64, _P, c_float, c_float, c_int64, c_float, c_float,
                                     _P, c_size_t, _P]),
    "rs_iteration_increment": (c_int, [_P, _P]),
    "rs_topk_ip_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int64, c_int]),
    "rs_topk_ip_f32": (c_int, [_P, c_int64, _P, c_int64, c_int64, c_int, c_int64, _P, _P, _P, c_size_t,
                               _P]),
    "rs_topk_ip_prec_f32": (c_int, [_P, c_int64, _P, c_int64, c_int64, c_int, c_int64, _P, _P, c_int, _P, c_size_t,
                                    _P]),
    "rs_topk_merge_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int]),
    "rs_topk_merge_f32": (c_int, [_P, _P, c_int64, c_int64, c_int, _P, _P, _P, c_size_t, _P]),
    "rs_inbatch_scores_bytes": (c_size_t, [c_int64]),
    "rs_inbatch_softmax_xent_fwd_store_f32": (c_int, [_P, _P, c_int64, c_int64, c_float, _P, _P, _P, _P, _P, _P, _P,
                                                      c_size_t, _P]),
    "rs_inbatch_softmax_xent_bwd_stored_f32": (c_int, [_P, _P, c_int64, c_int64, c_float, _P, _P, _P, _P, _P, _P,
                                                       _P, c_size_t, _P]),
    "rs_inbatch_softmax_xent_fwd_store_prec_f32": (c_int, [_P, _P, c_int64, c_int64, c_float, _P, _P, _P, _P, _P,
                                                           _P, c_int, _P, c_size_t, _P]),
    "rs_inbatch_softmax_xent_bwd_stored_prec_f32": (c_int, [_P, _P, c_int64, c_int64, c_float, _P, _P, _P, _P, _P,
                                                            _P, c_int, _P, c_size_t, _P]),
    "rs_inbatch_unique_rows_workspace_bytes": (c_size_t, [c_int64]),
    "rs_inbatch_unique_rows_f32": (c_int, [_P, c_int64, c_int64, _P, _P, _P, _P, _P, c_size_t, _P]),
    "rs_inbatch_unique_pair_workspace_bytes": (c_size_t, [c_int64]),
    "rs_inbatch_unique_pair_f32": (c_int, [_P, _P, c_int64, c_int64, _P, _P, _P, _P, _P, _P, _P, _P, c_size_t, _P]),
    "rs_reduction_queue_bytes": (c_size_t, []),
    "rs_reduction_queue_init": (c_int, [_P, c_size_t]),
    "rs_reduction_queue_flush": (c_int, [_P, _P]),
    "rs_reduction_queue_pending": (c_int, [_P]),
    "rs_inbatch_unique_ids_pair_i64": (c_int, [_P, _P, c_int64, c_int64, c_int64, _P, _P, _P, _P, _P, _P, _P, _P,
                                               c_size_t, _P]),
    "rs_inbatch_unique_ids_pair_order_i64": (c_int, [_P, _P, c_int64, c_int64, c_int64, _P, _P, _P, _P, _P, _P,
                                                     _P, _P, _P, _P, c_size_t, _P]),
    "rs_embedding_gather_tables_ordered_f32": (c_int, [c_int, _P, _P, _P, _P, _P, _P, c_int64, _P, _P]),
    "rs_inbatch_unique_ids_plan_i64": (c_int, [_P, _P, c_int64, c_int64, c_int64, _P, _P, _P, _P, _P, _P, _P, _P,
                                               _P, _P, _P, _P, _P, _P, c_size_t, _P]),
    "rs_sparse_adagrad_multi_step_planned_f32": (c_int, [c_int, _P, _P, _P, c_int64, _P, _P, _P, _P, _P, _P,
                                                         c_float, c_float, c_int64, c_float, c_float, _P, _P, _P, _P,
                                                         _P, c_size_t, _P]),
    "rs_embedding_gather_tables_ids_f32": (c_int, [c_int, _P, _P, _P, _P, _P, c_int64, _P, _P]),
    "rs_sparse_dedupe_planned_f32": (c_int, [_P, _P, c_int64, c_int64, c_int64, c_int64, _P, _P, _P, _P, _P, _P, _P,
                                             _P, _P, c_size_t, _P]),
    "rs_merge_runs_order_i64": (c_int, [_P, _P, c_int, _P, _P]),
    "rs_inbatch_dedup_workspace_bytes": (c_size_t, [c_int64, c_int64]),
    "rs_inbatch_softmax_xent_fwd_dedup_f32": (c_int, [_P, _P, c_int64, c_int64, c_float, _P, _P, c_int64, _P, _P,
                                                      c_int64, _P, _P, _P, _P, _P, _P, c_int, _P, c_size_t, _P]),
    "rs_inbatch_softmax_xent_bwd_dedup_f32": (c_int, [_P, c_int64, c_int64, c_float, _P, _P, _P, _P, _P, _P, _P, _P,
                                                      c_int64, _P, c_int64, c_int, _P, c_size_t, _P]),
    "rs_inbatch_softmax_xent_fwd_dedup_dev_f32": (c_int, [_P, _P, c_int64, c_int64, c_float, _P, _P, _P, _P, _P,
                                                          _P, _P, _P, _P, _P, _P, c_int, _P, c_size_t, _P]),
    "rs_inbatch_softmax_xent_bwd_dedup_dev_f32": (c_int, [_P, c_int64, c_int64, c_float, _P, _P, _P, _P, _P, _P,
                                                          _P, _P, _P, _P, c_int, _P, c_size_t, _P]),
    "rs_rank_metrics_workspace_bytes": (c_size_t, [c_int64, c_int, c_int64]),
    "rs_rank_metrics_i64": (c_int, [_P, c_int64, c_int, _P, _P, _P, c_int, c_int64, _P, _P, c_size_t, _P]),
    "rs_l2_normalize_rows_f32": (c_int, [_P, c_int64, c_int64, _P, _P]),
    "rs_shuffle_buffer_order_i64": (c_int, [c_int64, c_int64, ctypes.c_uint64, ctypes.c_uint64, _P]),
}


def exported_symbols():
    return sorted(_SIGNATURES)


def load(path: Optional[str] = None) -> ctypes.CDLL:
    """Load (once) and type the library. Raises NativeError if it is absent or mismatched."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise NativeError(
                f"librecsys_hip.so not found at {p}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (make -C csrc)")
        try:
            lib = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL)
        except OSError as e:  # pragma: no cover - environment specific
            raise NativeError(f"failed to load {p}: {e}") from e
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(lib, name)  # AttributeError if the ABI lacks a symbol
            fn.restype = res
            fn.argtypes = args
        if lib.rs_abi_version() != ABI_VERSION:
            raise NativeError(f"ABI mismatch: library {lib.rs_abi_version()} != {ABI_VERSION}")
        if path is None:
            _lib = lib
        return lib


def _typed(lib, name):
    """The entry point, only if its argument types are in _SIGNATURES (an untyped ctypes call
    would pass every integer as a 32-bit int)."""
    if name not in _SIGNATURES:
        raise NativeError(f"{name}: no signature in _native._SIGNATURES (add it beside include/recsys_hip.h)")
    return getattr(lib, name)


def call(name: str, *args) -> None:
    """Invoke an int-returning entry point and raise on a non-zero status."""
    lib = load()
    rc = _typed(lib, name)(*args)
    if rc != 0:
        msg = lib.rs_last_error().decode(errors="replace")
        raise NativeError(f"{name} failed (status {rc}): {msg}")


def query(name: str, *args) -> int:
    return int(_typed(load(), name)(*args))
