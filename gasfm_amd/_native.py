"""ctypes binding of the gasfm C ABI (include/gasfm.h).

The HIP library is REQUIRED: if ``libgasfm.so`` is missing or fails to load,
importing the compute entry points raises — there is no CPU or PyTorch
fallback for the attention path.  Host-only entry points (graph
preprocessing) work without a GPU, so DataLoader workers can use them.
"""
import ctypes
import threading
import os

import numpy as np
import torch

from .build import LIB

GASFM_OK, GASFM_ERR_INVALID, GASFM_ERR_OOM, GASFM_ERR_HIP, GASFM_ERR_UNSUPPORTED = range(5)

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f32 = ctypes.c_float

# name -> (restype, argtypes); mirrors include/gasfm.h
_SIGS = {
    "gasfm_last_error": (ctypes.c_char_p, []),
    "gasfm_version": (_i32, []),
    "gasfm_dispatch_counts": (_i32, [_vp, _i32]),
    "gasfm_dispatch_reset": (None, []),
    "gasfm_tuning_set": (_i32, [_i32, ctypes.c_double]),
    "gasfm_tuning_get": (ctypes.c_double, [_i32]),
    "gasfm_build_csr": (_i32, [_vp, _i64, _i32, _vp, _vp]),
    "gasfm_plan_work": (_i32, [_vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_gat_attn_fwd": (_i32, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _f32, _i32,
                                  _vp, _i64, _vp, _vp, _i64, _vp, _vp]),
    "gasfm_gat_attn_combine": (_i32, [_vp, _i32, _i32, _i32, _vp, _vp, _i32, _vp, _i64, _vp, _vp, _i64, _vp]),
    "gasfm_gat_attn_bwd_waves": (_i32, [_i32, _i32, _i32]),
    "gasfm_gat_attn_bwd": (_i32, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _f32, _vp,
                                  _i64, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _i32, _vp]),
    "gasfm_gat_attn_bwd_lanes": (_i32, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _f32, _vp,
                                  _i64, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _i32, _vp]),
    "gasfm_gat_attn_fwd_lanes": (_i32, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _f32, _i32,
                                  _vp, _i64, _vp, _vp, _i64, _vp, _vp]),
    "gasfm_gat_attn_bwd_combine": (_i32, [_vp, _i32, _i32, _vp, _vp, _i64, _vp]),
    "gasfm_gat_attn_bwd_combine2": (_i32, [_vp, _i32, _i32, _vp, _vp, _i64, _vp, _vp, _i64, _vp]),
    "gasfm_colsum_ws_floats": (_i64, [_i64, _i32]),
    "gasfm_edge_part_floats": (_i32, [_i32, _i64, _i32]),
    "gasfm_edge_prologue_fwd": (_i32, [_vp, _i64, _vp, _vp, _f32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp]),
    "gasfm_edge_epilogue_fwd": (_i32, [_vp, _vp, _vp, _vp, _i64, _vp, _vp, _f32, _vp, _i32, _vp, _vp, _vp, _i64,
                                       _vp, _f32, _vp, _vp]),
    "gasfm_edge_epilogue_bwd": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _f32, _vp, _i32, _f32, _vp, _vp, _vp,
                                       _vp, _vp]),
    "gasfm_edge_cam_bwd_part_rows": (_i32, [_i32]),
    "gasfm_edge_cam_bwd_part_cols": (_i32, []),
    "gasfm_edge_seam_fwd": (_i32, [_vp, _vp, _vp, _vp, _vp, _f32, _vp, _i32, _vp, _vp, _vp, _i64, _vp, _f32, _vp, _vp,
                                   _vp, _f32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _f32, _vp, _i32,
                                   _i32, _vp, _i64, _vp, _vp, _i64, _vp, _vp]),
    "gasfm_edge_cam_pbwd_part_rows": (_i32, [_i32]),
    "gasfm_edge_cam_pbwd_part_cols": (_i32, []),
    "gasfm_edge_cam_pbwd": (_i32, [_vp, _vp, _vp, _f32, _vp, _vp, _vp, _vp, _i32, _f32, _vp, _i64, _vp, _vp, _f32, _vp,
                                   _i64, _vp, _vp, _i64, _vp, _i64, _vp, _i32, _vp, _i64, _vp, _vp, _vp, _i64, _vp,
                                   _vp, _vp]),
    "gasfm_edge0_seam_fwd": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _f32,
                                    _vp, _vp, _vp, _f32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _f32,
                                    _vp, _i32, _i32, _vp, _i64, _vp, _vp, _i64, _vp, _vp]),
    "gasfm_edge_cam_pbwd_ex": (_i32, [_vp, _vp, _vp, _f32, _vp, _vp, _vp, _vp, _i32, _f32, _vp, _i64, _vp, _vp, _f32,
                                      _vp, _i64, _vp, _vp, _i64, _vp, _i64, _vp, _i32, _vp, _i64, _vp, _vp, _vp, _i64,
                                      _vp, _vp, _i64, _vp, _i32, _f32, _vp, _vp, _vp, _vp, _i32, _vp]),
    "gasfm_edge_cam_fwd": (_i32, [_vp, _vp, _vp, _f32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _f32,
                                  _vp, _i32, _i32, _vp, _i64, _vp, _vp, _i64, _vp, _vp]),
    "gasfm_edge_cam_bwd": (_i32, [_vp, _vp, _vp, _f32, _vp, _vp, _vp, _i64, _vp, _vp, _f32, _vp, _i64, _vp, _vp, _i64,
                                  _vp, _i64, _vp, _i32, _vp, _i64, _vp, _i64, _vp, _vp, _vp]),
    "gasfm_edge_prologue_bwd": (_i32, [_vp, _i64, _vp, _vp, _i64, _vp, _vp, _f32, _vp, _vp, _vp, _i32, _f32, _vp,
                                       _vp, _vp, _i64, _vp]),
    "gasfm_segment_rowsum": (_i32, [_vp, _i32, _vp, _vp, _i64, _f32, _vp, _vp, _vp]),
    "gasfm_colsum_counters": (_i32, [_i32]),
    "gasfm_colsum_multi": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_colsum_multi_counters": (_i32, [_i32, _vp]),
    "gasfm_colsum": (_i32, [_vp, _i64, _i32, _i64, _vp, _vp, _vp, _vp]),
    "gasfm_colsum_tall_ok": (_i32, [_i32]),
    "gasfm_colsum_tall_ws_floats": (_i64, [_i64, _i32]),
    "gasfm_colsum_tall": (_i32, [_vp, _i64, _i32, _vp, _vp, _vp, _vp]),
    "gasfm_edge0_part_rows": (_i32, [_i32, _i64, _i32]),
    "gasfm_edge0_prologue_fwd": (_i32, [_vp, _i64, _vp, _vp, _f32, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_edge0_prologue_fwd_rows": (_i32, [_vp, _i64, _vp, _vp, _f32, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_edge0_epilogue_fwd": (_i32, [_vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _vp, _vp, _vp,
                                        _vp, _i64, _vp, _f32, _vp, _vp]),
    "gasfm_edge0_epilogue_bwd": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _f32, _vp, _vp,
                                        _vp, _vp, _vp]),
    "gasfm_edge0_prologue_bwd": (_i32, [_vp, _vp, _vp, _i64, _vp, _vp, _f32, _vp, _vp, _vp, _vp]),
    "gasfm_node_part_rows": (_i32, [_i64, _i32, _i32]),
    "gasfm_gvec_fwd": (_i32, [_vp, _i32, _vp, _vp, _f32, _vp, _vp, _i32, _vp, _vp, _vp]),
    "gasfm_gvec_bwd_chunks": (_i32, [_i32]),
    "gasfm_gvec_bwd": (_i32, [_vp, _vp, _i32, _vp, _vp, _f32, _vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_node_ln_linear_fwd": (_i32, [_vp, _i64, _i32, _vp, _vp, _f32, _vp, _vp, _i32, _i32, _vp, _i64, _vp]),
    "gasfm_node_ln_linear_bwd": (_i32, [_vp, _vp, _i64, _i32, _vp, _vp, _f32, _vp, _i32, _i32, _vp, _vp, _vp]),
    "gasfm_view_tail_part_cols": (_i32, [_i32]),
    "gasfm_view_hub_part_cols": (_i32, [_i32]),
    "gasfm_view_scratch_floats": (_i64, [_i64, _i32]),
    "gasfm_view_tail_fwd": (_i32, [_vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _vp]),
    "gasfm_view_tail_bwd": (_i32, [_vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_view_hub_fwd": (_i32, [_vp, _i64, _i32, _f32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                  _vp, _i32, _vp, _vp, _vp]),
    "gasfm_view_hub_bwd": (_i32, [_vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                  _vp, _vp, _vp, _vp, _vp]),
    "gasfm_gvec_multi_fwd": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f32, _vp]),
    "gasfm_gvec_multi_bwd": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp,
                                    _vp, _vp, _f32, _vp]),
    "gasfm_view_chain_ok": (_i32, [_i64, _i32]),
    "gasfm_view_chain_scratch_floats": (_i64, [_i64, _i32]),
    "gasfm_view_chain_counters": (_i32, [_i64]),
    "gasfm_view_chain_tail_fwd": (_i32, [_vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _vp, _vp, _vp, _vp,
                                         _vp]),
    "gasfm_view_chain_hub_fwd": (_i32, [_vp, _i64, _i32, _f32] + [_vp] * 15 + [_i32, _vp, _vp]),
    "gasfm_view_chain_hub_bwd": (_i32, [_vp, _vp, _i64, _i32] + [_vp] * 18),
    "gasfm_view_chain_tail_bwd": (_i32, [_vp] * 5 + [_i64, _i32] + [_vp] * 12),
    "gasfm_gchain_fwd": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_gchain_scratch_floats": (_i64, [_vp]),
    "gasfm_gchain_counters": (_i32, [_vp]),
    "gasfm_gchain_bwd": (_i32, [_vp] * 16),
    "gasfm_gatt_scratch_floats": (_i64, [_i32, _vp]),
    "gasfm_gatt_counters": (_i32, [_i32, _vp]),
    "gasfm_gatt_fwd": (_i32, [_i32, _vp, _f32, _vp, _vp, _vp]),
    "gasfm_gatt_bwd": (_i32, [_i32, _vp, _f32, _vp, _vp, _vp]),
    "gasfm_gatt_merge": (_i32, [_i32, _vp, _i32, _i64, _vp]),
    "gasfm_exchange_unpack": (_i32, [_vp, _i32, _i64, _i64, _i32, _i32, _i32, _vp, _i64, _i64, _i32, _vp, _vp]),
    "gasfm_gatt_merge_unpack": (_i32, [_i32, _vp, _i32, _i64, _vp, _i32, _i64, _i64, _i32, _i32, _i32, _vp, _i64,
                                       _vp]),
    "gasfm_pose_fwd": (_i32, [_vp, _i64, _i64, _vp, _vp]),
    "gasfm_pose_bwd": (_i32, [_vp, _i64, _i64, _vp, _vp, _i64, _vp]),
    "gasfm_esfm_part_rows": (_i32, [_i64]),
    "gasfm_reproj_error": (_i32, [_vp, _vp, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp]),
    "gasfm_scene_mask_words": (_i64, [_i32]),
    "gasfm_scene_tiles": (_i64, [_i32, _i32]),
    "gasfm_scan_i32": (_i32, [_vp, _i64, _vp, _vp]),
    "gasfm_scene_mask": (_i32, [_vp, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_scene_emit": (_i32, [_vp, _i64, _vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_scene_point_csr": (_i32, [_vp, _vp, _vp, _vp, _i32, _i32, _vp, _vp, _vp]),
    "gasfm_scene_homography": (_i32, [_vp, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "gasfm_outlier_counts": (_i32, [_vp, _vp, _vp, _vp, _i32, _i32, _vp, _vp, _vp, _vp]),
    "gasfm_outlier_mark": (_i32, [_vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _vp]),
    "gasfm_outlier_moments": (_i32, [_vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_outlier_apply": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp]),
    "gasfm_ba_partials": (_i64, [_i64]),
    "gasfm_ba_eval": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _i32, _vp, _vp, _vp, _vp,
                             _vp]),
    "gasfm_ba_sum": (_i32, [_vp, _i64, _vp, _vp]),
    "gasfm_ba_normals": (_i32, [_i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_ba_damp": (_i32, [_i32, _i32, _i32, _vp, _vp, ctypes.c_double, _vp, _vp, _vp, _vp]),
    "gasfm_ba_schur": (_i32, [_i32, _i32, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp,
                              _vp, _vp, _vp, _vp]),
    "gasfm_ba_backsub": (_i32, [_i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_ba_model": (_i32, [_i32, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_ba_dlt": (_i32, [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_sum_n": (_i32, [_i32, _vp, _i64, _vp, _vp]),
    "gasfm_esfm_fwd": (_i32, [_vp, _vp, _vp, _i64, _vp, _vp, _i64, _f32, _f32, _i32, _vp, _vp]),
    "gasfm_esfm_bwd": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp, _vp, _i64, _f32, _f32, _i32, _i32,
                              _i32, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_esfm_seg_part_rows": (_i32, [_i32]),
    "gasfm_esfm_seg_fwd": (_i32, [_vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _i64, _f32, _f32, _i32, _vp, _vp, _vp,
                                  _vp]),
    "gasfm_esfm_seg_bwd": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _f32,
                                  _f32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_reproj_error_seg": (_i32, [_vp, _vp, _vp, _vp, _i32, _vp, _vp, _i64, _vp, _vp, _vp]),
    "gasfm_union_fill_scene": (_i32, [_vp, _vp, _vp]),
    "gasfm_fold_scene_rows_fwd": (_i32, [_vp, _i64, _vp, _i64, _vp, _i64, _i32, _vp, _i64, _vp]),
    "gasfm_fold_scene_rows_bwd": (_i32, [_vp, _i64, _vp, _i64, _i32, _i32, _vp, _i64, _vp]),
    "gasfm_adam_step": (_i32, [_vp, _vp, _i32, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                               ctypes.c_double, _i64, _vp]),
    "gasfm_union_fill_pad": (_i32, [_vp, _vp, _vp]),
    "gasfm_point_tail_part_shape": (_i32, [_i64, _i32, _vp]),
    "gasfm_point_hub_part_shape": (_i32, [_i64, _i32, _i32, _vp]),
    "gasfm_point_tail_fwd": (_i32, [_vp, _vp, _i64, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _vp, _vp]),
    "gasfm_point_tail_bwd": (_i32, [_vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_point_hub_fwd": (_i32, [_vp, _i64, _f32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _vp, _vp, _vp]),
    "gasfm_point_tail_hub_fwd": (_i32, [_vp, _vp, _i64, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _vp, _f32] + [_vp] * 15),
    "gasfm_point_hub_bwd_c": (_i32, [_vp, _i64, _f32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_point_hub_bwd_ab": (_i32, [_vp, _i64, _f32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_point_hub_bwd": (_i32, [_vp, _i64, _f32] + [_vp] * 17),
    "gasfm_point_head_part_shape": (_i32, [_i64, _i32, _vp]),
    "gasfm_point_head_fwd": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_point_head_bwd": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gasfm_embed2_part_rows": (_i32, [_i64]),
    "gasfm_embed2_fwd": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp]),
    "gasfm_embed2_bwd": (_i32, [_vp, _vp, _i64, _vp, _vp]),
    "gasfm_gemm_bf16": (_i32, [_i32, _i32, _i32, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _vp, _vp, _i64, _vp]),
    "gasfm_gemm_f32": (_i32, [_i32, _i32, _i32, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _vp, _vp, _i64, _vp]),
    "gasfm_gemm_f32_smallm_ok": (_i32, [_i32, _i32, _i32, _i32]),
    "gasfm_gemm_f32_smallm": (_i32, [_i32, _i32, _i32, _i32, _vp, _i64, _vp, _i64, _vp, _vp, _i64, _vp, _i64, _vp]),
}

_lib = None


def lib():
    """Load libgasfm.so (raising loudly if absent)."""
    global _lib
    if _lib is None:
        path = os.environ.get("GASFM_LIB") or LIB  # GASFM_LIB: an A/B build variant (build.build(out=...))
        if not os.path.exists(path):
            raise ImportError(
                f"gasfm native library not built: {path} missing. Run `python -m gasfm_amd.build` "
                "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
        L = ctypes.CDLL(path)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def exported_symbols():
    return list(_SIGS)


def check(status, what):
    if status == GASFM_OK:
        return
    msg = lib().gasfm_last_error().decode(errors="replace")
    if status == GASFM_ERR_OOM:
        raise torch.OutOfMemoryError(f"{what}: {msg}")
    raise RuntimeError(f"{what} failed (status {status}): {msg}")


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(t):
    if _RAW_STREAM is not None and t.device.index is not None:
        # the current stream's handle without building a torch.cuda.Stream object (~2 us per
        # launch on the host: ~4,700 launches per eager training step)
        return ctypes.c_void_p(_RAW_STREAM(t.device.index))
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


# ---------------------------------------------------------------- kernel-choice record, tuning
# mirrors the GASFM_K_* / GASFM_TUNE_* enums of include/gasfm.h
KERNELS = {
    "attn_fwd_grp": 0, "attn_fwd_glds": 1, "attn_fwd_vec": 2, "attn_fwd_generic": 3, "attn_fwd_lanes": 4,
    "attn_bwd_glds": 5, "attn_bwd_vec": 6, "attn_bwd_generic": 7, "attn_bwd_lanes": 8,
    "attn_combine_vec": 9, "attn_combine_generic": 10, "seam_reg": 13, "attn_fwd_grp_s2": 14, "attn_fwd_grp_s4": 15,
}
TUNING = {"attn_grp_rows": 0, "attn_grp_min_fill": 1, "attn_glds": 2, "attn_wave_cap": 3, "attn_grp_split": 4}


def dispatch_counts():
    """{kernel name: launches since the last reset} of the size-dependent dispatches."""
    n = len(KERNELS) + 8
    buf = (_i64 * n)()
    lib().gasfm_dispatch_counts(buf, n)
    return {k: int(buf[i]) for k, i in KERNELS.items()}


def dispatch_reset():
    lib().gasfm_dispatch_reset()


def tuning_get(key):
    return float(lib().gasfm_tuning_get(TUNING[key]))


def tuning_set(key, value):
    check(lib().gasfm_tuning_set(TUNING[key], float(value)), "gasfm_tuning_set")


class tuned:
    """Context manager: set dispatch thresholds, restore them on exit."""

    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.prev = {k: tuning_get(k) for k in self.kv}
        for k, v in self.kv.items():
            tuning_set(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.prev.items():
            tuning_set(k, v)
        return False


class dispatch_record:
    """Context manager: ``rec.counts`` = launches per kernel inside the block."""

    def __enter__(self):
        self.start = dispatch_counts()
        return self

    def __exit__(self, *exc):
        end = dispatch_counts()
        self.counts = {k: end[k] - self.start[k] for k in end}
        return False


# ---------------------------------------------------------------- host graph preprocessing
def build_csr(key, n):
    """Stable counting sort of int32 keys in [0, n): returns (ptr[n+1], perm[E]) numpy int32."""
    key = np.ascontiguousarray(key, dtype=np.int32)
    E = key.shape[0]
    ptr = np.empty(n + 1, dtype=np.int32)
    perm = np.empty(max(E, 1), dtype=np.int32)
    st = lib().gasfm_build_csr(key.ctypes.data_as(_vp), E, n, ptr.ctypes.data_as(_vp),
                               perm.ctypes.data_as(_vp))
    check(st, "gasfm_build_csr")
    return ptr, perm[:E]


def plan_work(seg_ptr, max_piece, all_partial=False):
    """Split segments into work items; returns (items[n,4], combine[k,4], n_slots) numpy int32."""
    seg_ptr = np.ascontiguousarray(seg_ptr, dtype=np.int32)
    N = seg_ptr.shape[0] - 1
    ni, nc, ns = _i32(0), _i32(0), _i32(0)
    L = lib()
    L.gasfm_plan_work(seg_ptr.ctypes.data_as(_vp), N, max_piece, int(all_partial), None,
                      ctypes.byref(ni), None, ctypes.byref(nc), ctypes.byref(ns))
    items = np.empty((max(ni.value, 1), 4), dtype=np.int32)
    comb = np.empty((max(nc.value, 1), 4), dtype=np.int32)
    ni2, nc2 = _i32(ni.value), _i32(nc.value)
    st = L.gasfm_plan_work(seg_ptr.ctypes.data_as(_vp), N, max_piece, int(all_partial),
                           items.ctypes.data_as(_vp), ctypes.byref(ni2), comb.ctypes.data_as(_vp),
                           ctypes.byref(nc2), ctypes.byref(ns))
    check(st, "gasfm_plan_work")
    return items[:ni2.value], comb[:nc2.value], ns.value


# ---------------------------------------------------------------- device kernels
def attn_fwd(XL, XR, att, bias, perm, items, n_items, H, C, slope, finalize, out, seg_max, seg_sum, part=None,
             ldStat=None, lanes=False):
    """part: packed partial rows [slots, H*C + 2H] (acc | max | sum) or None.  lanes: the
    lane-per-item kernel (H = 4, C = 1; short items: block 0's point direction)."""
    ldStat = H if ldStat is None else ldStat
    fn = lib().gasfm_gat_attn_fwd_lanes if lanes else lib().gasfm_gat_attn_fwd
    st = fn(
        _p(XL), XL.stride(0), _p(XR), XR.stride(0), _p(att), _p(bias), _p(perm), _p(items), n_items, H, C,
        slope, int(finalize), _p(out), out.stride(0) if out is not None else 0, _p(seg_max), _p(seg_sum), ldStat,
        _p(part), _stream(XL))
    check(st, "gasfm_gat_attn_fwd")


def attn_combine(combine, n_combine, H, C, part, bias, finalize, out, seg_max, seg_sum, ldOut=None, ldStat=None):
    """Merge packed partial rows; out/seg_max/seg_sum may be views into a packed buffer (raw mode)."""
    ldOut = out.stride(0) if ldOut is None else ldOut
    ldStat = H if ldStat is None else ldStat
    st = lib().gasfm_gat_attn_combine(_p(combine), n_combine, H, C, _p(part), _p(bias), int(finalize), _p(out),
                                      ldOut, _p(seg_max), _p(seg_sum), ldStat, _stream(part))
    check(st, "gasfm_gat_attn_combine")


def attn_bwd_waves(n_items, H, C):
    return lib().gasfm_gat_attn_bwd_waves(n_items, H, C)


def attn_bwd(XL, XR, att, bias, perm, items, n_items, H, C, slope, out, seg_max, seg_sum, gout, dXL, dXR,
             part_dxr, datt_part, xl_by_position=False, lanes=False):
    fn = lib().gasfm_gat_attn_bwd_lanes if lanes else lib().gasfm_gat_attn_bwd
    st = fn(
        _p(XL), XL.stride(0), _p(XR), XR.stride(0), _p(att), _p(bias), _p(perm), _p(items), n_items, H, C,
        slope, _p(out), out.stride(0), _p(seg_max), _p(seg_sum), _p(gout), gout.stride(0), _p(dXL),
        dXL.stride(0), _p(dXR), dXR.stride(0), _p(part_dxr), _p(datt_part), int(xl_by_position), _stream(dXL))
    check(st, "gasfm_gat_attn_bwd")


def attn_bwd_combine(combine, n_combine, HC, part_dxr, dXR):
    st = lib().gasfm_gat_attn_bwd_combine(_p(combine), n_combine, HC, _p(part_dxr), _p(dXR), dXR.stride(0),
                                          _stream(dXR))
    check(st, "gasfm_gat_attn_bwd_combine")


def attn_bwd_combine2(combine, n_combine, HC, part_a, out_a, part_b, out_b):
    """attn_bwd_combine of two partial-row arrays over the same entries, one launch."""
    st = lib().gasfm_gat_attn_bwd_combine2(_p(combine), n_combine, HC, _p(part_a), _p(out_a), out_a.stride(0),
                                           _p(part_b), _p(out_b), out_b.stride(0), _stream(out_a))
    check(st, "gasfm_gat_attn_bwd_combine2")


_COUNTERS = {}
_COUNTER_POOL = 1 << 16


def _counters(device, n):
    """A range of n zeroed uint32 ticket counters for one colsum launch (self-resetting: the last
    arriver of each column chunk puts its counter back to 0).

    Every call gets its OWN range from a per-device pool, handed out round-robin, so colsums that
    run concurrently (on different streams, or on parallel branches of a captured graph) never
    share a ticket: a range comes back only after the other ~65k counters have been handed out.
    The pool is allocated once, large (a replacement allocated while a hipGraph is being captured
    would leave the nodes captured before it pointing at the freed array)."""
    n = max(1, int(n))
    if n > _COUNTER_POOL:
        raise ValueError(f"colsum counters: {n} requested, pool holds {_COUNTER_POOL}")
    c = _COUNTERS.get(device)
    if c is None:
        c = [torch.zeros(_COUNTER_POOL, dtype=torch.int32, device=device), 0]
        _COUNTERS[device] = c
    pool, at = c
    if at + n > _COUNTER_POOL:
        at = 0
    c[1] = at + n
    return pool[at:at + n]


def colsum(A, out=None):
    """Deterministic column sum of a 2-D fp32 CUDA tensor (row stride may exceed cols); one launch."""
    assert A.dim() == 2 and A.stride(1) == 1 and A.dtype == torch.float32
    rows, cols = A.shape
    if out is None:
        out = torch.empty(cols, dtype=torch.float32, device=A.device)
    L = lib()
    ws = torch.empty(int(L.gasfm_colsum_ws_floats(rows, cols)), dtype=torch.float32, device=A.device)
    cnt = _counters(A.device, L.gasfm_colsum_counters(cols))
    st = L.gasfm_colsum(_p(A), rows, cols, max(A.stride(0), cols), _p(ws), _p(out), _p(cnt), _stream(out))
    check(st, "gasfm_colsum")
    return out


def colsum_tall_ok(A):
    return (A.dim() == 2 and A.is_contiguous() and A.dtype == torch.float32
            and bool(lib().gasfm_colsum_tall_ok(A.shape[1])))


def colsum_tall(A, out=None):
    """Column sums of a contiguous tall [rows, cols] fp32 CUDA tensor (colsum_tall_ok)."""
    rows, cols = A.shape
    if out is None:
        out = torch.empty(cols, dtype=torch.float32, device=A.device)
    L = lib()
    ws = torch.empty(max(1, int(L.gasfm_colsum_tall_ws_floats(rows, cols))), dtype=torch.float32, device=A.device)
    cnt = _counters(A.device, 1)
    st = L.gasfm_colsum_tall(_p(A), rows, cols, _p(ws), _p(out), _p(cnt), _stream(out))
    check(st, "gasfm_colsum_tall")
    return out



# ---------------------------------------------------------------- batched weight-gradient sums
# A backward pass ends with ~150 column sums of per-workgroup weight-gradient partials (one per
# fused kernel).  Their results are parameter gradients that nothing reads before the backward
# pass returns, so inside a pass they are queued and run as ONE batched launch
# (gasfm_colsum_multi) from an autograd final callback: ~150 fewer kernel launches per step.
# Only when the model forward saw every parameter's .grad unset (AccumulateGrad then adopts the
# returned tensor instead of adding it to an existing gradient, so filling it later is safe);
# otherwise, and outside a backward pass, param_colsum is colsum.
_DEFER_FWD = False
_PENDING = {}
_SEEN = {}  # graph task -> ids of the parameters that already received a deferred sum in it
_PENDING_LOCK = threading.Lock()


def defer_token(*targets):
    """Captured by the fused Functions' forward (ctx.defer) and passed to param_colsum: in a
    deferring model forward, the tensors that receive the deferred sums when every one is a leaf
    (a parameter: no autograd node reads its gradient before the pass ends); else False."""
    if _DEFER_FWD and all(t is None or t.is_leaf for t in targets):
        return tuple(t for t in targets if t is not None) or True
    return False


class deferring_param_grads:
    """Set by GraphAttnSfMNet.forward for the duration of the forward."""

    def __init__(self, enabled):
        self.enabled = bool(enabled)

    def __enter__(self):
        global _DEFER_FWD
        self.prev, _DEFER_FWD = _DEFER_FWD, self.enabled
        return self

    def __exit__(self, *exc):
        global _DEFER_FWD
        _DEFER_FWD = self.prev
        return False


def param_colsum(A, defer):
    """colsum of weight-gradient partials; deferred to the end of the backward pass when
    ``defer`` (see above) and called inside one."""
    task = torch._C._current_graph_task_id() if defer else -1
    if task < 0:
        return colsum(A)
    if isinstance(defer, tuple) and any(t.grad is not None for t in defer):
        # the parameter already holds a gradient (retain_graph and a second backward, or two
        # forwards backpropagated separately): AccumulateGrad ADDS the returned tensor to it at
        # once, so it must be filled now
        return colsum(A)
    if isinstance(defer, tuple):
        # parameter -> the token (one per Function forward) whose sum it got first in this pass; the
        # same token again is another output of the same Function (e.g. both attention directions)
        with _PENDING_LOCK:
            seen = _SEEN.setdefault(task, {})
            again = any(seen.get(id(t), id(defer)) != id(defer) for t in defer)
            for t in defer:
                seen.setdefault(id(t), id(defer))
        if again and os.environ.get("GASFM_DEBUG_DEFER"):
            print("param_colsum: repeated targets", [tuple(t.shape) for t in defer], flush=True)
        if again:
            # a second contribution to these parameters in this pass (several forwards, one
            # backward: train.py sums the scenes' losses).  AccumulateGrad adopts one sum and adds
            # the other to it, so none may be left unfilled: fill the queued sums first (stream
            # order puts them before any later add), then sum this one now.
            _flush_param_colsums(task, final=False)
            return colsum(A)
    assert A.dim() == 2 and A.stride(1) == 1 and A.dtype == torch.float32
    rows, cols = A.shape
    L = lib()
    out = torch.empty(cols, dtype=torch.float32, device=A.device)
    ws = torch.empty(int(L.gasfm_colsum_ws_floats(rows, cols)), dtype=torch.float32, device=A.device)
    job = (A, ws, out, rows, cols, max(A.stride(0), cols), torch.cuda.current_stream(A.device))
    with _PENDING_LOCK:
        jobs = _PENDING.get(task)
        first = jobs is None
        if first:
            jobs = _PENDING[task] = []
        jobs.append(job)
    if first:
        torch.autograd.Variable._execution_engine.queue_callback(lambda: _flush_param_colsums(task))
    return out


def _flush_param_colsums(task, final=True):
    with _PENDING_LOCK:
        jobs = _PENDING.pop(task, [])
        if final:
            _SEEN.pop(task, None)
    if not jobs:
        return
    stream = jobs[0][6]
    assert all(j[6] == stream for j in jobs), "param_colsum: jobs queued on several streams"
    n = len(jobs)
    L = lib()
    arr = lambda ty, xs: (ty * n)(*xs)  # noqa: E731
    A = arr(ctypes.c_void_p, [j[0].data_ptr() for j in jobs])
    ws = arr(ctypes.c_void_p, [j[1].data_ptr() for j in jobs])
    out = arr(ctypes.c_void_p, [j[2].data_ptr() for j in jobs])
    rows = arr(ctypes.c_int64, [j[3] for j in jobs])
    cols = arr(ctypes.c_int32, [j[4] for j in jobs])
    ld = arr(ctypes.c_int64, [j[5] for j in jobs])
    dev = jobs[0][0].device
    cnt = _counters(dev, L.gasfm_colsum_multi_counters(n, cols))
    st = L.gasfm_colsum_multi(n, A, rows, cols, ld, ws, out, _p(cnt), ctypes.c_void_p(stream.cuda_stream))
    check(st, "gasfm_colsum_multi")
    # the partial buffers (jobs) are released only now, after the launch that reads them


# ---------------------------------------------------------------- fused per-edge block kernels
def _req(t, name, cols=None):
    if not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous():
        raise TypeError(f"{name}: expected a contiguous float32 CUDA tensor (no CPU fallback)")
    if cols is not None and t.shape[-1] != cols:
        raise ValueError(f"{name}: expected {cols} columns, got {tuple(t.shape)}")


def edge_part_floats(which, E, n_items=0):
    return lib().gasfm_edge_part_floats(which, E, n_items)


def edge_prologue_fwd(P, ln_w, ln_b, eps, W, b, Y, pos=None, W2=None, b2=None):
    """W [64,32] / b [64], or the halves W [32,32] + W2 [32,32] and b [32] + b2 [32]."""
    _req(P, "P", 32)
    st = lib().gasfm_edge_prologue_fwd(_p(P), P.shape[0], _p(ln_w), _p(ln_b), eps, _p(W), _p(W2), _p(b), _p(b2),
                                       _p(Y), Y.stride(0), _p(pos), _stream(P))
    check(st, "gasfm_edge_prologue_fwd")


def _rows32(t, name):
    """[rows, 32] float32 CUDA rows with unit column stride (row stride >= 32: a column slice of a
    gathered [SV | XR] block is fine); returns the row stride."""
    if not t.is_cuda or t.dtype != torch.float32 or t.dim() != 2 or t.shape[1] != 32 or t.stride(1) != 1 \
            or (t.shape[0] > 1 and t.stride(0) < 32):
        raise TypeError(f"{name}: expected [rows, 32] float32 CUDA rows with unit column stride")
    return t.stride(0) if t.shape[0] > 1 else 32


def edge_epilogue_fwd(P, P0, cam, pt, ln_w, ln_b, eps, Wp, bp, Sp, Sv, Sg, scale, out):
    _req(P, "P", 32)
    for t, n in ((Sp, "Sp"), (Sg, "Sg"), (Wp, "Wp")):
        _req(t, n)
    ldSv = _rows32(Sv, "Sv")
    st = lib().gasfm_edge_epilogue_fwd(_p(P), _p(P0), _p(cam), _p(pt), P.shape[0], _p(ln_w), _p(ln_b), eps, _p(Wp),
                                       Wp.shape[1], _p(bp), _p(Sp), _p(Sv), ldSv, _p(Sg), scale, _p(out),
                                       _stream(P))
    check(st, "gasfm_edge_epilogue_fwd")


def edge_epilogue_bwd(items, n_items, dPo, P, P0, ln_w, ln_b, eps, Wp, scale, dSv, part_dsv, dP0, part_w):
    _req(dPo, "dP'", 32)
    st = lib().gasfm_edge_epilogue_bwd(_p(items), n_items, _p(dPo), _p(P), _p(P0), _p(ln_w), _p(ln_b), eps, _p(Wp),
                                       Wp.shape[1], scale, _p(dSv), _p(part_dsv), _p(dP0), _p(part_w), _stream(dPo))
    check(st, "gasfm_edge_epilogue_bwd")


def edge_prologue_bwd(dXL, P, dRes, ln_w, ln_b, eps, W, Wp, scale, dP, part, W2=None, dXLc=None):
    """dXLc: the camera half of dXL in its own [E, 32] buffer (dXL then holds the point half)."""
    _req(P, "P", 32)
    st = lib().gasfm_edge_prologue_bwd(_p(dXL), dXL.stride(0), _p(P), _p(dRes), P.shape[0], _p(ln_w), _p(ln_b), eps,
                                       _p(W), _p(W2), _p(Wp), Wp.shape[1] if Wp is not None else 0, scale, _p(dP),
                                       _p(part), _p(dXLc), dXLc.stride(0) if dXLc is not None else 0, _stream(P))
    check(st, "gasfm_edge_prologue_bwd")


def edge_cam_fwd(P, ln_w, ln_b, eps, Wpt, bpt, Wc, bc, XLp, pos, XR, att, bias, slope, plan_items, n_items,
                 finalize, out, seg_max, seg_sum, part, ldStat=4):
    """Edge prologue + camera-direction attention forward (csrc/edge_cam.hip): XLp [E, 32] (point
    half of lin_l, written through pos), camera aggregates into out / seg_max / seg_sum (complete
    items) or packed partial rows part [slots, 40]."""
    _req(P, "P", 32)
    ldXR = _rows32(XR, "XR")
    st = lib().gasfm_edge_cam_fwd(_p(P), _p(ln_w), _p(ln_b), eps, _p(Wpt), _p(bpt), _p(Wc), _p(bc), _p(XLp),
                                  XLp.stride(0), _p(pos), _p(XR), ldXR, _p(att), _p(bias), slope, _p(plan_items),
                                  n_items, int(finalize), _p(out), out.stride(0) if out is not None else 0,
                                  _p(seg_max), _p(seg_sum), ldStat, _p(part), _stream(P))
    check(st, "gasfm_edge_cam_fwd")


def edge_cam_bwd_part_shape(n_items):
    L = lib()
    return int(L.gasfm_edge_cam_bwd_part_rows(n_items)), int(L.gasfm_edge_cam_bwd_part_cols())


def edge_cam_bwd(P, ln_w, ln_b, eps, Wc, bc, XR, att, bias, slope, out, seg_max, seg_sum, gout, plan_items, n_items,
                 dXLc, dXR, part_dxr, part, ldStat=4):
    """Camera-attention backward with XLc recomputed from P: dXLc [E, 32], dXR, [datt | dbias] partials."""
    _req(P, "P", 32)
    ldXR = _rows32(XR, "XR")
    st = lib().gasfm_edge_cam_bwd(_p(P), _p(ln_w), _p(ln_b), eps, _p(Wc), _p(bc), _p(XR), ldXR, _p(att), _p(bias),
                                  slope, _p(out), out.stride(0), _p(seg_max), _p(seg_sum), ldStat, _p(gout),
                                  gout.stride(0), _p(plan_items), n_items, _p(dXLc), dXLc.stride(0), _p(dXR),
                                  dXR.stride(0), _p(part_dxr), _p(part), _stream(P))
    check(st, "gasfm_edge_cam_bwd")


def _ld_stat(seg_max):
    """row stride of the [N, heads] statistics (4 for their own tensors; the partial-row stride when
    they are columns of a packed partial buffer)"""
    return seg_max.stride(0) if seg_max is not None else 4


def edge_seam_fwd(Pb, P0, pt, lnw_b, lnb_b, eps_b, Wp, bp, Sp, Sv, Sg, scale, Pout, ln_w, ln_b, eps, Wpt, bpt, Wc, bc,
                  XLp, pos, XR, att, bias, slope, plan_items, n_items, finalize, out, seg_max, seg_sum, part):
    """Block b's edge epilogue (P' = Pout) + block b+1's prologue and camera attention forward in one
    pass (csrc/edge_cam.hip edge_seam_fwd); outputs as edge_cam_fwd's plus Pout."""
    _req(Pb, "Pb", 32)
    ldXR = _rows32(XR, "XR")
    ldSv = _rows32(Sv, "Sv")
    st = lib().gasfm_edge_seam_fwd(_p(Pb), _p(P0), _p(pt), _p(lnw_b), _p(lnb_b), eps_b, _p(Wp), Wp.stride(0), _p(bp),
                                   _p(Sp), _p(Sv), ldSv, _p(Sg), scale, _p(Pout), _p(ln_w), _p(ln_b), eps, _p(Wpt),
                                   _p(bpt), _p(Wc), _p(bc), _p(XLp), XLp.stride(0), _p(pos), _p(XR), ldXR, _p(att),
                                   _p(bias), slope, _p(plan_items), n_items, int(finalize), _p(out),
                                   out.stride(0) if out is not None else 0, _p(seg_max), _p(seg_sum), _ld_stat(seg_max),
                                   _p(part), _stream(Pb))
    check(st, "gasfm_edge_seam_fwd")


def edge0_seam_fwd(P, pt, lna_w, lna_b, lnb_w, lnb_b, eps0, Wp, bp, Wsk, bsk, Sp, Sv, Sg, scale, Pout, ln_w, ln_b, eps,
                   Wpt, bpt, Wc, bc, XLp, pos, XR, att, bias, slope, plan_items, n_items, finalize, out, seg_max,
                   seg_sum, part):
    """Block 0's edge epilogue (2-wide P, edge0_epilogue_fwd) + block 1's prologue and camera
    attention forward in one pass (csrc/edge_cam.hip edge_seam_fwd, EP0); outputs as
    edge_seam_fwd's."""
    _req(P, "P", 2)
    ldXR = _rows32(XR, "XR")
    ldSv = _rows32(Sv, "Sv")
    st = lib().gasfm_edge0_seam_fwd(_p(P), _p(pt), _p(lna_w), _p(lna_b), _p(lnb_w), _p(lnb_b), eps0, _p(Wp), _p(bp),
                                    _p(Wsk), _p(bsk), _p(Sp), _p(Sv), ldSv, _p(Sg), scale, _p(Pout), _p(ln_w), _p(ln_b),
                                    eps, _p(Wpt), _p(bpt), _p(Wc), _p(bc), _p(XLp), XLp.stride(0), _p(pos), _p(XR),
                                    ldXR, _p(att), _p(bias), slope, _p(plan_items), n_items, int(finalize), _p(out),
                                    out.stride(0) if out is not None else 0, _p(seg_max), _p(seg_sum),
                                    _ld_stat(seg_max), _p(part), _stream(P))
    check(st, "gasfm_edge0_seam_fwd")


def edge_cam_pbwd_part_shape(n_items, dwp_cols=0):
    """(rows, cols) of edge_cam_pbwd's part buffer; dwp_cols = 32 or 34 with the dWp block (dwp)."""
    L = lib()
    return int(L.gasfm_edge_cam_pbwd_part_rows(n_items)), int(L.gasfm_edge_cam_pbwd_part_cols()) + 32 * dwp_cols


def edge_cam_pbwd(P, ln_w, ln_b, eps, Wpt, Wc, bc, Wp, scale, XR, att, bias, slope, out, seg_max, seg_sum, gout,
                  plan_items, n_items, dXLp, dRes, dP, dXR, part_dxr, part, ldStat=4, epi=None, dwp=None):
    """The camera attention's backward and the block's edge prologue backward in one pass
    (csrc/edge_cam.hip edge_cam_pbwd): dP, dXR (+ split partials), part rows
    [dW 64x32 | db 64 | dgamma 32 | dbeta 32 | datt 32 | 0 (32)] per workgroup (the attention bias
    gradient is the caller's column sum of gout).

    epi = (We, scale_e, dSv, part_dsv, dP0 or None): also the previous block's edge-epilogue
    gradients from this dP (dSv rows / split-camera partial rows of the same plan, dP0).
    dwp = P0 or None (requires ln_w and dRes): also this block's lin_proj weight gradient,
    [32 x (32 | 34)] appended to each part row (part has edge_cam_pbwd_part_shape(n, dwp=...) columns)."""
    _req(P, "P", 32)
    ldXR = _rows32(XR, "XR")
    We = dSv = part_dsv = dP0 = None
    scale_e, ldWe = 0.0, 0
    if epi is not None:
        We, scale_e, dSv, part_dsv, dP0 = epi
        _req(dSv, "dSv", 32)
        if dP0 is not None:
            _req(dP0, "dP0", 2)
        ldWe = We.stride(0)
    P0, ldWpo = None, 0
    if dwp is not False and dwp is not None:
        P0 = dwp if isinstance(dwp, torch.Tensor) else None
        ldWpo = 34 if P0 is not None else 32
    if P0 is not None:
        _req(P0, "P0", 2)
    st = lib().gasfm_edge_cam_pbwd_ex(_p(P), _p(ln_w), _p(ln_b), eps, _p(Wpt), _p(Wc), _p(bc), _p(Wp),
                                      Wp.stride(0) if Wp is not None else 0, scale, _p(XR), ldXR, _p(att), _p(bias),
                                      slope, _p(out), out.stride(0), _p(seg_max), _p(seg_sum), ldStat, _p(gout),
                                      gout.stride(0), _p(plan_items), n_items, _p(dXLp), dXLp.stride(0), _p(dRes),
                                      _p(dP), _p(dXR), dXR.stride(0), _p(part_dxr), _p(part), part.stride(0), _p(We),
                                      ldWe, scale_e, _p(dSv), _p(part_dsv), _p(dP0), _p(P0), ldWpo, _stream(P))
    check(st, "gasfm_edge_cam_pbwd")


def segment_rowsum(items, n_items, perm, X, scale, out, part):
    st = lib().gasfm_segment_rowsum(_p(items), n_items, _p(perm), _p(X), X.stride(0), scale, _p(out), _p(part),
                                    _stream(X))
    check(st, "gasfm_segment_rowsum")


# ---------------------------------------------------------------- block 0 (2-wide) edge kernels
def edge0_part_rows(which, E, n_items=0):
    return lib().gasfm_edge0_part_rows(which, E, n_items)


def edge0_prologue_fwd(P, ln_w, ln_b, eps, W0, b0, XL, pos=None):
    _req(P, "P", 2)
    st = lib().gasfm_edge0_prologue_fwd(_p(P), P.shape[0], _p(ln_w), _p(ln_b), eps, _p(W0), _p(b0), _p(XL),
                                        _p(pos), _stream(P))
    check(st, "gasfm_edge0_prologue_fwd")


def edge0_prologue_fwd_rows(P, ln_w, ln_b, eps, W0, b0, XL, perm):
    _req(P, "P", 2)
    if perm.dtype != torch.int32 or perm.numel() != P.shape[0] or perm.device != P.device:
        raise ValueError("edge0_prologue_fwd_rows: perm must be int32 [E] on P's device")
    st = lib().gasfm_edge0_prologue_fwd_rows(_p(P), P.shape[0], _p(ln_w), _p(ln_b), eps, _p(W0), _p(b0), _p(XL),
                                             _p(perm), _stream(P))
    check(st, "gasfm_edge0_prologue_fwd_rows")


def edge0_epilogue_fwd(P, cam, pt, lna_w, lna_b, lnb_w, lnb_b, eps, Wp, bp, Wsk, bsk, Sp, Sv, Sg, scale, out):
    _req(P, "P", 2)
    for t, n in ((Sp, "Sp"), (Sg, "Sg")):
        _req(t, n)
    ldSv = _rows32(Sv, "Sv")
    st = lib().gasfm_edge0_epilogue_fwd(_p(P), _p(cam), _p(pt), P.shape[0], _p(lna_w), _p(lna_b), _p(lnb_w),
                                        _p(lnb_b), eps, _p(Wp), _p(bp), _p(Wsk), _p(bsk), _p(Sp), _p(Sv), ldSv,
                                        _p(Sg), scale, _p(out), _stream(P))
    check(st, "gasfm_edge0_epilogue_fwd")


def edge0_epilogue_bwd(items, n_items, dPo, P, lna_w, lna_b, lnb_w, lnb_b, eps, Wp, Wsk, scale, dSv, part_dsv, aux,
                       part):
    _req(dPo, "dP'", 32)
    st = lib().gasfm_edge0_epilogue_bwd(_p(items), n_items, _p(dPo), _p(P), _p(lna_w), _p(lna_b), _p(lnb_w),
                                        _p(lnb_b), eps, _p(Wp), _p(Wsk), scale, _p(dSv), _p(part_dsv), _p(aux),
                                        _p(part), _stream(dPo))
    check(st, "gasfm_edge0_epilogue_bwd")


def edge0_prologue_bwd(dXL, P, aux, ln_w, ln_b, eps, W0, dP, part):
    _req(dXL, "dXL0", 8)
    st = lib().gasfm_edge0_prologue_bwd(_p(dXL), _p(P), _p(aux), P.shape[0], _p(ln_w), _p(ln_b), eps, _p(W0),
                                        _p(dP), _p(part), _stream(P))
    check(st, "gasfm_edge0_prologue_bwd")


# ---------------------------------------------------------------- point-node LayerNorm -> ReLU -> Linear
def node_part_rows(N, n_out, residual):
    return lib().gasfm_node_part_rows(N, n_out, int(residual))


def node_ln_linear_fwd(X, ln_w, ln_b, eps, W, b, residual, Y):
    _req(X, "X")
    N, n_in = X.shape
    st = lib().gasfm_node_ln_linear_fwd(_p(X), N, n_in, _p(ln_w), _p(ln_b), eps, _p(W), _p(b), W.shape[0],
                                        int(residual), _p(Y), Y.stride(0), _stream(X))
    check(st, "gasfm_node_ln_linear_fwd")


def node_ln_linear_bwd(dY, X, ln_w, ln_b, eps, W, residual, dX, part):
    _req(dY, "dY", W.shape[0])
    _req(X, "X")
    N, n_in = X.shape
    st = lib().gasfm_node_ln_linear_bwd(_p(dY), _p(X), N, n_in, _p(ln_w), _p(ln_b), eps, _p(W), W.shape[0],
                                        int(residual), _p(dX), _p(part), _stream(X))
    check(st, "gasfm_node_ln_linear_bwd")


# ---------------------------------------------------------------- global node (one row)
def gvec_bwd_chunks(N):
    return lib().gasfm_gvec_bwd_chunks(N)


def gvec_fwd(x, ln_w, ln_b, eps, W, b, res, y):
    _req(x, "x")
    _req(W, "W")
    st = lib().gasfm_gvec_fwd(_p(x), W.shape[1], _p(ln_w), _p(ln_b), eps, _p(W), _p(b), W.shape[0], _p(res), _p(y),
                              _stream(x))
    check(st, "gasfm_gvec_fwd")


def gvec_bwd(dy, x, ln_w, ln_b, eps, W, resid, dx, dW, db, dgam, dbet, part):
    _req(dy, "dy")
    st = lib().gasfm_gvec_bwd(_p(dy), _p(x), W.shape[1], _p(ln_w), _p(ln_b), eps, _p(W), W.shape[0], int(resid),
                              _p(dx), _p(dW), _p(db), _p(dgam), _p(dbet), _p(part), _stream(x))
    check(st, "gasfm_gvec_bwd")


# ---------------------------------------------------------------- scene-point block chains (point_block.hip)
def point_tail_part_shape(N, has_prev):
    cols = ctypes.c_int32(0)
    rows = lib().gasfm_point_tail_part_shape(N, int(has_prev), ctypes.byref(cols))
    return rows, cols.value


def point_hub_part_shape(N, which, has_res):
    cols = ctypes.c_int32(0)
    rows = lib().gasfm_point_hub_part_shape(N, int(which), int(has_res), ctypes.byref(cols))
    return rows, cols.value


def point_tail_fwd(prev, agg, Wp, bp, ln_w, ln_b, eps, Wm, bm, out):
    _req(agg, "agg", 32)
    if prev is not None:
        _req(prev, "prev", 64)
    st = lib().gasfm_point_tail_fwd(_p(prev), _p(agg), agg.shape[0], _p(Wp), _p(bp), _p(ln_w), _p(ln_b), eps,
                                    _p(Wm), _p(bm), _p(out), _stream(agg))
    check(st, "gasfm_point_tail_fwd")


def point_tail_bwd(dout, prev, agg, Wp, bp, ln_w, ln_b, eps, Wm, dx, dagg, part):
    _req(dout, "dout", 64)
    _req(agg, "agg", 32)
    if prev is not None:
        _req(prev, "prev", 64)
    st = lib().gasfm_point_tail_bwd(_p(dout), _p(prev), _p(agg), agg.shape[0], _p(Wp), _p(bp), _p(ln_w), _p(ln_b),
                                    eps, _p(Wm), _p(dx), _p(dagg), _p(part), _stream(agg))
    check(st, "gasfm_point_tail_bwd")


def point_hub_fwd(X, eps, gA, bA, WA, SA, WB, bB, XL, gC, bC, WC, bWC, WD, bD, XR):
    _req(X, "X", 64)
    st = lib().gasfm_point_hub_fwd(_p(X), X.shape[0], eps, _p(gA), _p(bA), _p(WA), _p(SA), _p(WB), _p(bB), _p(XL),
                                   _p(gC), _p(bC), _p(WC), _p(bWC), _p(WD), _p(bD), _p(XR), _stream(X))
    check(st, "gasfm_point_hub_fwd")


def point_tail_hub_fwd(prev, agg, Wp, bp, ln_w, ln_b, eps, Wm, bm, out, eps_h, gA, bA, WA, SA, WB, bB, XL, gC, bC,
                       WC, bWC, WD, bD, XR):
    """point_tail_fwd + point_hub_fwd on its output in one launch (out = p)."""
    _req(agg, "agg", 32)
    _req(out, "out", 64)
    if prev is not None:
        _req(prev, "prev", 64)
    st = lib().gasfm_point_tail_hub_fwd(_p(prev), _p(agg), agg.shape[0], _p(Wp), _p(bp), _p(ln_w), _p(ln_b), eps,
                                        _p(Wm), _p(bm), _p(out), eps_h, _p(gA), _p(bA), _p(WA), _p(SA), _p(WB), _p(bB),
                                        _p(XL), _p(gC), _p(bC), _p(WC), _p(bWC), _p(WD), _p(bD), _p(XR), _stream(agg))
    check(st, "gasfm_point_tail_hub_fwd")


def point_hub_bwd_c(X, eps, gC, bC, WC, bWC, WD, dXR, dRes, dX, part):
    _req(X, "X", 64)
    _req(dXR, "dXR", 32)
    if dRes is not None:
        _req(dRes, "dRes", 64)
    st = lib().gasfm_point_hub_bwd_c(_p(X), X.shape[0], eps, _p(gC), _p(bC), _p(WC), _p(bWC), _p(WD), _p(dXR),
                                     _p(dRes), _p(dX), _p(part), _stream(X))
    check(st, "gasfm_point_hub_bwd_c")


def point_hub_bwd_ab(X, eps, gA, bA, WA, WB, dSA, dXL, dRes, dX, part):
    _req(X, "X", 64)
    _req(dSA, "dSA", 32)
    _req(dXL, "dXL", 64)
    if dRes is not None:
        _req(dRes, "dRes", 64)
    st = lib().gasfm_point_hub_bwd_ab(_p(X), X.shape[0], eps, _p(gA), _p(bA), _p(WA), _p(WB), _p(dSA), _p(dXL),
                                      _p(dRes), _p(dX), _p(part), _stream(X))
    check(st, "gasfm_point_hub_bwd_ab")


def point_hub_bwd(X, eps, gA, bA, WA, WB, gC, bC, WC, bWC, WD, dSA, dXL, dXR, dRes, dX, part_a, part_c):
    """The whole point-hub backward in one pass (gasfm_point_hub_bwd)."""
    _req(X, "X", 64)
    _req(dSA, "dSA", 32)
    _req(dXL, "dXL", 64)
    _req(dXR, "dXR", 32)
    if dRes is not None:
        _req(dRes, "dRes", 64)
    st = lib().gasfm_point_hub_bwd(_p(X), X.shape[0], eps, _p(gA), _p(bA), _p(WA), _p(WB), _p(gC), _p(bC), _p(WC),
                                   _p(bWC), _p(WD), _p(dSA), _p(dXL), _p(dXR), _p(dRes), _p(dX), _p(part_a),
                                   _p(part_c), _stream(X))
    check(st, "gasfm_point_hub_bwd")


# ---------------------------------------------------------------- input embedding (embed.hip)
def embed2_fwd(X, W, b, Y):
    _req(X, "values", 2)
    _req(Y, "P", 2)
    st = lib().gasfm_embed2_fwd(_p(X), X.shape[0], _p(W), _p(b), _p(Y), _stream(X))
    check(st, "gasfm_embed2_fwd")


def embed2_bwd(X, dY, defer=False):
    """(dW [2, 2], db [2]) of P = X W^T + b from dP; column sums through param_colsum."""
    _req(X, "values", 2)
    _req(dY, "dP", 2)
    E = X.shape[0]
    rows = lib().gasfm_embed2_part_rows(E)
    if rows == 0:
        tot = torch.zeros(6, dtype=torch.float32, device=X.device)
    else:
        part = torch.empty((rows, 6), dtype=torch.float32, device=X.device)
        st = lib().gasfm_embed2_bwd(_p(X), _p(dY), E, _p(part), _stream(X))
        check(st, "gasfm_embed2_bwd")
        tot = param_colsum(part, defer)
    return tot[:4].view(2, 2), tot[4:]


# ---------------------------------------------------------------- scene-point head (point_head.hip)
def point_head_part_shape(N, which):
    cols = ctypes.c_int32(0)
    rows = lib().gasfm_point_head_part_shape(N, int(which), ctypes.byref(cols))
    return rows, cols.value


def _head_weights(W1, b1, W2, b2, W3, b3=None):
    shapes = ((W1, (64, 64)), (b1, (64,)), (W2, (64, 64)), (b2, (64,)), (W3, (3, 64))) + \
        (((b3, (3,)),) if b3 is not None else ())
    for t, shape in shapes:
        if tuple(t.shape) != shape or not t.is_contiguous() or t.dtype != torch.float32:
            raise ValueError(f"point head: weight {tuple(t.shape)} is not a contiguous fp32 {shape}")


def point_head_fwd(P, W1, b1, W2, b2, W3, b3, out):
    _req(P, "P", 64)
    _head_weights(W1, b1, W2, b2, W3, b3)
    N = P.shape[0]
    if tuple(out.shape) != (4, N) or not out.is_contiguous():
        raise ValueError("point_head_fwd: out must be a contiguous [4, N]")
    st = lib().gasfm_point_head_fwd(_p(P), N, _p(W1), _p(b1), _p(W2), _p(b2), _p(W3), _p(b3), _p(out), _stream(P))
    check(st, "gasfm_point_head_fwd")


def point_head_bwd(P, W1, b1, W2, b2, W3, dout, dP, part_a, part_b):
    _req(P, "P", 64)
    _req(dP, "dP", 64)
    _head_weights(W1, b1, W2, b2, W3)
    N = P.shape[0]
    if tuple(dout.shape) != (4, N) or not dout.is_contiguous():
        raise ValueError("point_head_bwd: dout must be a contiguous [4, N]")
    for part, which in ((part_a, 0), (part_b, 1)):
        if tuple(part.shape) != point_head_part_shape(N, which) or not part.is_contiguous():
            raise ValueError("point_head_bwd: partial buffer of the wrong shape")
    st = lib().gasfm_point_head_bwd(_p(P), N, _p(W1), _p(b1), _p(W2), _p(b2), _p(W3), _p(dout), _p(dP),
                                    _p(part_a), _p(part_b), _stream(P))
    check(st, "gasfm_point_head_bwd")


# ---------------------------------------------------------------- camera-side block chains (view_block.hip)
def view_tail_part_cols(D):
    return lib().gasfm_view_tail_part_cols(D)


def view_hub_part_cols(D):
    return lib().gasfm_view_hub_part_cols(D)


def view_scratch(m, D, device):
    return torch.empty(max(1, int(lib().gasfm_view_scratch_floats(m, D))), dtype=torch.float32, device=device)


def view_tail_fwd(prev, agg, Wp, bp, ln_w, ln_b, eps, bm, x, xb, h, rs, scratch):
    _req(agg, "agg", 32)
    D = x.shape[1]
    if prev is not None:
        _req(prev, "prev", D)
    st = lib().gasfm_view_tail_fwd(_p(prev), _p(agg), agg.shape[0], D, _p(Wp), _p(bp), _p(ln_w), _p(ln_b), eps,
                                   _p(bm), _p(x), _p(xb), _p(h), _p(rs), _p(scratch), _stream(agg))
    check(st, "gasfm_view_tail_fwd")


def view_tail_bwd(dv, dh, x, rs, agg, Wp, ln_w, ln_b, dx, dagg, part, scratch):
    D = x.shape[1]
    for t, n in ((dv, "dv"), (dh, "dh"), (x, "x")):
        _req(t, n, D)
    _req(agg, "agg", 32)
    st = lib().gasfm_view_tail_bwd(_p(dv), _p(dh), _p(x), _p(rs), _p(agg), agg.shape[0], D, _p(Wp), _p(ln_w),
                                   _p(ln_b), _p(dx), _p(dagg), _p(part), _p(scratch), _stream(agg))
    check(st, "gasfm_view_tail_bwd")


def view_hub_fwd(v, eps, gC, bC, Wv, gA, bA, Wa, ba, Wr, br, sv, t, xr, rs, scratch):
    """sv / xr: [m, 32] with a common row stride (two column halves of one [m, 64] block, or two
    contiguous tensors)."""
    _req(v, "v")
    ldo = _rows32(sv, "sv")
    if _rows32(xr, "xr") != ldo:
        raise ValueError("view_hub_fwd: sv and xr need the same row stride")
    st = lib().gasfm_view_hub_fwd(_p(v), v.shape[0], v.shape[1], eps, _p(gC), _p(bC), _p(Wv), _p(gA), _p(bA), _p(Wa),
                                  _p(ba), _p(Wr), _p(br), _p(sv), _p(t), _p(xr), ldo, _p(rs), _p(scratch), _stream(v))
    check(st, "gasfm_view_hub_fwd")


def view_chain_ok(m, D):
    return bool(lib().gasfm_view_chain_ok(m, D))


def _vc_scratch(m, D, device):
    return torch.empty(max(1, int(lib().gasfm_view_chain_scratch_floats(m, D))), dtype=torch.float32, device=device)


def view_chain_tail_fwd(prev, agg, Wp, bp, ln_w, ln_b, eps, Wm, bm, view, x, h, rs):
    _req(agg, "agg", 32)
    m, D = view.shape
    for t, n in ((view, "view"), (x, "x"), (h, "h"), (Wm, "Wm"), (Wp, "Wp")) + (((prev, "prev"),) if prev is not None else ()):
        _req(t, n)
    st = lib().gasfm_view_chain_tail_fwd(_p(prev), _p(agg), m, D, _p(Wp), _p(bp), _p(ln_w), _p(ln_b), eps, _p(Wm),
                                         _p(bm), _p(view), _p(x), _p(h), _p(rs), _stream(agg))
    check(st, "gasfm_view_chain_tail_fwd")


def view_chain_hub_fwd(v, eps, Wl, bl, gC, bC, Wv, gA, bA, Wa, ba, Wr, br, XL, sv, t, xr, rs):
    _req(v, "v")
    ldo = _rows32(sv, "sv")
    if _rows32(xr, "xr") != ldo:
        raise ValueError("view_chain_hub_fwd: sv and xr need the same row stride")
    for a, n in ((Wl, "Wl"), (Wv, "Wv"), (Wa, "Wa"), (XL, "XL")):
        _req(a, n)
    st = lib().gasfm_view_chain_hub_fwd(_p(v), v.shape[0], v.shape[1], eps, _p(Wl), _p(bl), _p(gC), _p(bC), _p(Wv),
                                        _p(gA), _p(bA), _p(Wa), _p(ba), _p(Wr), _p(br), _p(XL), _p(sv), _p(t), _p(xr),
                                        ldo, _p(rs), _stream(v))
    check(st, "gasfm_view_chain_hub_fwd")


def view_chain_hub_bwd(v, rs, gC, bC, Wv, gA, bA, Wa, t, Wr, Wl, dsv, dxr, dxl, dres, dacc, dWl, part):
    _req(v, "v")
    m, D = v.shape
    for a, n, w in ((t, "t", 32), (dsv, "dsv", 32), (dxr, "dxr", 32), (dxl, "dxl", D), (dacc, "dacc", D),
                    (dWl, "dWl", D)):
        _req(a, n, w)
    if dres is not None:
        _req(dres, "dres", D)
    scratch = _vc_scratch(m, D, v.device)
    st = lib().gasfm_view_chain_hub_bwd(_p(v), _p(rs), m, D, _p(gC), _p(bC), _p(Wv), _p(gA), _p(bA), _p(Wa), _p(t),
                                        _p(Wr), _p(Wl), _p(dsv), _p(dxr), _p(dxl), _p(dres), _p(dacc), _p(dWl),
                                        _p(part), _p(scratch), _stream(v))
    check(st, "gasfm_view_chain_hub_bwd")


def view_chain_tail_bwd(dv, x, h, rs, agg, Wp, ln_w, ln_b, Wm, dh, dWm, dx, dagg, part):
    m, D = x.shape
    for a, n in ((dv, "dv"), (x, "x"), (h, "h"), (dh, "dh"), (dx, "dx"), (dWm, "dWm")):
        _req(a, n, D)
    _req(agg, "agg", 32)
    scratch = _vc_scratch(m, D, x.device)
    cnt = _counters(x.device, lib().gasfm_view_chain_counters(m))
    st = lib().gasfm_view_chain_tail_bwd(_p(dv), _p(x), _p(h), _p(rs), _p(agg), m, D, _p(Wp), _p(ln_w), _p(ln_b),
                                         _p(Wm), _p(dh), _p(dWm), _p(dx), _p(dagg), _p(part), _p(scratch), _p(cnt),
                                         _stream(x))
    check(st, "gasfm_view_chain_tail_bwd")


def view_hub_bwd(v, rs, gC, bC, Wv, gA, bA, Wa, t, Wr, dsv, dxr, dxl, dacc, part, scratch, dres=None):
    """dres (d skip, or None) is added to dacc in the kernel's second pass."""
    _req(v, "v")
    D = v.shape[1]
    for a, n, w in ((t, "t", 32), (dsv, "dsv", 32), (dxr, "dxr", 32), (dxl, "dxl", D), (dacc, "dacc", D)):
        _req(a, n, w)
    if dres is not None:
        _req(dres, "dres", D)
    st = lib().gasfm_view_hub_bwd(_p(v), _p(rs), v.shape[0], D, _p(gC), _p(bC), _p(Wv), _p(gA), _p(bA), _p(Wa),
                                  _p(t), _p(Wr), _p(dsv), _p(dxr), _p(dxl), _p(dres), _p(dacc), _p(part),
                                  _p(scratch), _stream(v))
    check(st, "gasfm_view_hub_bwd")


# ---------------------------------------------------------------- calibrated camera head (pose_head.hip)
def pose_fwd(x, P):
    if not x.is_cuda or x.dtype != torch.float32 or x.stride(1) != 1:
        raise TypeError("pose x: expected a float32 CUDA tensor with unit column stride (no CPU fallback)")
    check(lib().gasfm_pose_fwd(_p(x), x.stride(0), x.shape[0], _p(P), _stream(x)), "gasfm_pose_fwd")


def pose_bwd(x, dP, dx):
    _req(dP, "dP")
    check(lib().gasfm_pose_bwd(_p(x), x.stride(0), x.shape[0], _p(dP), _p(dx), dx.stride(0), _stream(x)),
          "gasfm_pose_bwd")


# ---------------------------------------------------------------- ESFMLoss (esfm_loss.hip)
def _i32vec(t, name):
    if not t.is_cuda or t.dtype != torch.int32 or t.dim() != 1 or not t.is_contiguous():
        raise TypeError(f"{name}: expected a contiguous int32 CUDA vector")


def esfm_part_rows(E):
    return lib().gasfm_esfm_part_rows(E)


def esfm_fwd(cam, pt, vals, P, X, margin, hinge_w, hinge, part):
    E, n = cam.shape[0], X.shape[1]
    _i32vec(cam, "cam"), _i32vec(pt, "pt")
    _req(vals, "vals", 2), _req(P, "P", 12), _req(X, "pts3D", n)
    if X.shape[0] != 4 or pt.shape[0] != E or vals.shape[0] != E:
        raise ValueError("esfm_fwd: expected pts3D [4, n] and E-long cam / pt / values")
    st = lib().gasfm_esfm_fwd(_p(cam), _p(pt), _p(vals), E, _p(P), _p(X), n, margin, hinge_w, int(hinge), _p(part),
                              _stream(X))
    check(st, "gasfm_esfm_fwd")


def esfm_bwd(cptr, pptr, perm, cam, pt, vals, P, X, margin, hinge_w, hinge, equalize, valid_only, dloss, tot, dP,
             dX, E_norm=None):
    """E_norm: the edge count of the mean (default the local E; the global count on a sharded scene)."""
    E, n, m = cam.shape[0], X.shape[1], P.shape[0]
    E_norm = E if E_norm is None else int(E_norm)
    for t, name in ((cptr, "cam_ptr"), (pptr, "pt_ptr"), (cam, "cam"), (pt, "pt")):
        _i32vec(t, name)
    if perm is not None:
        _i32vec(perm, "perm")
    if cptr.shape[0] != m + 1 or pptr.shape[0] != n + 1 or (perm is not None and perm.shape[0] != E):
        raise ValueError("esfm_bwd: CSR shapes do not match m / n / E")
    _req(dP, "dP", 12), _req(dX, "dX", n)
    st = lib().gasfm_esfm_bwd(_p(cptr), m, _p(pptr), _p(perm) if perm is not None else None, _p(cam), _p(pt),
                              _p(vals), E, E_norm, _p(P), _p(X), n, margin, hinge_w, int(hinge), int(equalize),
                              int(valid_only), _p(dloss), _p(tot), _p(dP), _p(dX), _stream(X))
    check(st, "gasfm_esfm_bwd")


def reproj_error(cam, pt, xy, P, X, err=None):
    """Per-workgroup (sum, count) of the non-NaN reprojection errors (and err[e] if given)."""
    E, n = cam.shape[0], X.shape[1]
    _i32vec(cam, "cam"), _i32vec(pt, "pt")
    _req(xy, "xy", 2), _req(P, "P", 12), _req(X, "pts3D", n)
    if X.shape[0] != 4 or pt.shape[0] != E or xy.shape[0] != E or (err is not None and err.shape[0] != E):
        raise ValueError("reproj_error: expected pts3D [4, n] and E-long cam / pt / xy / err")
    part = torch.empty((esfm_part_rows(E), 2), dtype=torch.float32, device=X.device)
    st = lib().gasfm_reproj_error(_p(cam), _p(pt), _p(xy), E, _p(P), _p(X), n, _p(err), _p(part), _stream(X))
    check(st, "gasfm_reproj_error")
    return part


def _seg_args(eoff, S, name):
    if eoff.dtype != torch.int32 or not eoff.is_contiguous() or eoff.numel() != S + 1:
        raise TypeError(f"{name}: eoff must be a contiguous int32 [S + 1] tensor")


def esfm_seg_fwd(cam, pt, vals, eoff, weight, P, X, margin, hinge_w, hinge):
    """Union-batch ESFMLoss forward (gasfm_esfm_seg_fwd): (loss [1], tot [S, 2])."""
    S = int(weight.numel())
    _seg_args(eoff, S, "esfm_seg_fwd")
    n = X.shape[1]
    if X.shape[0] != 4 or cam.shape != pt.shape or vals.shape != (cam.shape[0], 2):
        raise ValueError("esfm_seg_fwd: expected pts3D [4, n] and E-long cam / pt / values")
    dev = X.device
    part = torch.empty((lib().gasfm_esfm_seg_part_rows(S), 2), dtype=torch.float32, device=dev)
    tot = torch.empty((S, 2), dtype=torch.float32, device=dev)
    loss = torch.empty(1, dtype=torch.float32, device=dev)
    st = lib().gasfm_esfm_seg_fwd(_p(cam), _p(pt), _p(vals), _p(eoff), S, _p(weight), _p(P), _p(X), n, margin, hinge_w,
                                  int(hinge), _p(part), _p(tot), _p(loss), _stream(X))
    check(st, "gasfm_esfm_seg_fwd")
    return loss, tot


def esfm_seg_bwd(cptr, pptr, perm, cam, pt, vals, eoff, scene_of_cam, scene_of_pt, weight, P, X, margin, hinge_w,
                 hinge, equalize, valid_only, dloss, tot, dP, dX):
    """Union-batch ESFMLoss backward (gasfm_esfm_seg_bwd) into dP [m, 12] and dX [4, n]."""
    S = int(weight.numel())
    _seg_args(eoff, S, "esfm_seg_bwd")
    m, n = P.shape[0], X.shape[1]
    if cptr.numel() != m + 1 or pptr.numel() != n + 1 or scene_of_cam.numel() != m or scene_of_pt.numel() != n:
        raise ValueError("esfm_seg_bwd: CSR / scene map shapes do not match m / n")
    st = lib().gasfm_esfm_seg_bwd(_p(cptr), m, _p(pptr), _p(perm), _p(cam), _p(pt), _p(vals), _p(eoff), S,
                                  _p(scene_of_cam), _p(scene_of_pt), _p(weight), _p(P), _p(X), n, margin, hinge_w,
                                  int(hinge), int(equalize), int(valid_only), _p(dloss), _p(tot), _p(dP), _p(dX),
                                  _stream(X))
    check(st, "gasfm_esfm_seg_bwd")


def reproj_error_seg(cam, pt, xy, eoff, S, P, X):
    """Per scene of a union batch: tot [S, 2] = (sum of the non-NaN reprojection errors, count)."""
    _seg_args(eoff, S, "reproj_error_seg")
    dev = X.device
    part = torch.empty((lib().gasfm_esfm_seg_part_rows(S), 2), dtype=torch.float32, device=dev)
    tot = torch.empty((S, 2), dtype=torch.float32, device=dev)
    st = lib().gasfm_reproj_error_seg(_p(cam), _p(pt), _p(xy), _p(eoff), S, _p(P), _p(X), X.shape[1], _p(part),
                                      _p(tot), _stream(X))
    check(st, "gasfm_reproj_error_seg")
    return tot


class UnionScene(ctypes.Structure):
    _fields_ = ([("idx", _vp), ("ld_idx", _i64)] + [(k, _vp) for k in (
        "vals", "vals_loss", "cptr", "pptr", "perm", "pos", "cam_per_pts", "pts_per_cam", "M")] + [("ldM", _i64),
        ("Ns", _vp)] + [(k, _i64) for k in ("E", "m", "n", "e0", "c0", "p0", "item0")] + [("scene", _i32)])


class UnionOut(ctypes.Structure):
    _fields_ = ([("indices", _vp), ("ld_indices", _i64)] + [(k, _vp) for k in (
        "cam32", "pt32", "values", "values_loss", "xy", "perm", "pos", "cam_ptr", "pt_ptr", "cam_per_pts",
        "pts_per_cam", "soc", "soc32", "sop32", "Ns_inv", "items_c", "comb_c", "items_p")] + [("piece", _i32)])


class UnionPad(ctypes.Structure):
    _fields_ = [(k, _i64) for k in ("M", "N", "E", "mp", "npd", "ep", "dI", "item0")] + [("scene", _i32)]


def union_fill_scene(sc, out, stream_of):
    check(lib().gasfm_union_fill_scene(ctypes.byref(sc), ctypes.byref(out), _stream(stream_of)),
          "gasfm_union_fill_scene")


def fold_scene_rows_fwd(sv, sg, soc):
    """sv [m, w] + sg[soc] (gasfm_fold_scene_rows_fwd); unit column strides."""
    out = torch.empty((sv.shape[0], sv.shape[1]), dtype=torch.float32, device=sv.device)
    check(lib().gasfm_fold_scene_rows_fwd(_p(sv), sv.stride(0), _p(sg), sg.stride(0), _p(soc), sv.shape[0],
                                          sv.shape[1], _p(out), out.stride(0), _stream(sv)), "gasfm_fold_scene_rows_fwd")
    return out


def fold_scene_rows_bwd(dout, soc, S):
    """[S, w] per-scene sums of dout's rows in camera order (gasfm_fold_scene_rows_bwd)."""
    dsg = torch.empty((S, dout.shape[1]), dtype=torch.float32, device=dout.device)
    check(lib().gasfm_fold_scene_rows_bwd(_p(dout), dout.stride(0), _p(soc), dout.shape[0], S, dout.shape[1], _p(dsg),
                                          dsg.stride(0), _stream(dout)), "gasfm_fold_scene_rows_bwd")
    return dsg


ADAM_CHUNK = 4096  # GASFM_ADAM_CHUNK


def adam_step(tensors, chunks, n_chunks, lr, beta1, beta2, eps, weight_decay, step, stream_of):
    """gasfm_adam_step over device tables (uint8 tensors holding gasfm_adam_tensor / _chunk rows)."""
    check(lib().gasfm_adam_step(_p(tensors), _p(chunks), int(n_chunks), float(lr), float(beta1), float(beta2),
                                float(eps), float(weight_decay), int(step), _stream(stream_of)), "gasfm_adam_step")


def union_fill_pad(pd, out, stream_of):
    check(lib().gasfm_union_fill_pad(ctypes.byref(pd), ctypes.byref(out), _stream(stream_of)), "gasfm_union_fill_pad")


# ---------------------------------------------------------------- batched single-row problems (global hub)
def _ptrs(ts):
    return (ctypes.c_void_p * len(ts))(*[None if t is None else t.data_ptr() for t in ts])


def _ints(v):
    return (ctypes.c_int32 * len(v))(*v)


def gvec_multi_fwd(probs, eps):
    """probs: [(x, ln_w, ln_b, W, b, res, y)]; x / res / y 1-D rows, W [N, K]."""
    cols = list(zip(*probs))
    for W in cols[3]:
        _req(W, "W")
    K = [W.shape[1] for W in cols[3]]
    N = [W.shape[0] for W in cols[3]]
    st = lib().gasfm_gvec_multi_fwd(len(probs), *[_ptrs(c) for c in cols], _ints(K), _ints(N), eps,
                                    _stream(cols[0][0]))
    check(st, "gasfm_gvec_multi_fwd")


def gvec_multi_bwd(probs, groups, eps):
    """probs: [(dy, x, ln_w, ln_b, W, dW, db, dgam, dbet, part)]; groups: [(p0, np, dres, dx)]."""
    dy, x, lw, lb, W, dW, db, dg, dbt, part = (list(c) for c in zip(*probs))
    K = [w.shape[1] for w in W]
    N = [w.shape[0] for w in W]
    p0, npr, dres, dx = (list(c) for c in zip(*groups))
    st = lib().gasfm_gvec_multi_bwd(len(probs), _ptrs(dy), _ptrs(x), _ptrs(lw), _ptrs(lb), _ptrs(W), _ints(K),
                                    _ints(N), _ptrs(dW), _ptrs(db), _ptrs(dg), _ptrs(dbt), _ptrs(part), len(groups),
                                    _ints(p0), _ints(npr), _ptrs(dres), _ptrs(dx), eps, _stream(x[0]))
    check(st, "gasfm_gvec_multi_bwd")


# ---------------------------------------------------------------- the global node's chain (global_chain.hip)
_GC_DIMS = ("G", "Kc", "NA", "NB", "NC", "ND", "NE")
_GC_W = ("W1", "b1", "gM", "bM", "W2", "b2", "gA", "bA", "WA", "gB", "bB", "WB", "bWB", "gC", "bC", "WC", "bWC",
         "WD", "bD", "WE", "bE")
_GC_D = tuple("d" + k for k in _GC_W)


_GC_SHADOW = ("W1", "W2", "WA", "WB", "WC", "WD", "WE")  # the weights with an optional bf16 shadow


class _GChain(ctypes.Structure):
    _fields_ = ([(k, _i32) for k in _GC_DIMS] + [("eps_m", _f32), ("eps_h", _f32)] + [(k, _vp) for k in _GC_W]
                + [(k + "h", _vp) for k in _GC_SHADOW] + [("rows", _i32)])


GCHAIN_MAX_ROWS = 7  # GASFM_GCHAIN_MAX_ROWS


class _GChainGrads(ctypes.Structure):
    _fields_ = [(k, _vp) for k in _GC_D]


def gchain_struct(w, eps_m, eps_h, shadows=None, rows=1):
    """gasfm_gchain of the weights dict w (keys _GC_W; the hub's B..E absent for the last block);
    shadows: dict weight key -> its bf16 shadow (BASELINE config 5) or None."""
    c = _GChain()
    W1, WA = w["W1"], w["WA"]
    hub = w.get("WB") is not None
    dims = dict(G=W1.shape[0], Kc=W1.shape[1], NA=WA.shape[0], NB=w["WB"].shape[0] if hub else 0,
                NC=w["WC"].shape[0] if hub else 0, ND=w["WD"].shape[0] if hub else 0,
                NE=w["WE"].shape[0] if hub else 0)
    for k, v in dims.items():
        setattr(c, k, int(v))
    c.eps_m, c.eps_h = float(eps_m), float(eps_h)
    for k in _GC_W:
        t = w.get(k)
        if t is not None:
            _req(t, k)
            setattr(c, k, t.data_ptr())
    for k, t in (shadows or {}).items():
        if t is not None:
            if t.dtype != torch.bfloat16 or not t.is_contiguous() or t.shape != w[k].shape:
                raise ValueError(f"gchain: the bf16 shadow of {k} must be a contiguous bf16 tensor of its shape")
            setattr(c, k + "h", t.data_ptr())
    if not 1 <= rows <= GCHAIN_MAX_ROWS:
        raise ValueError(f"gchain: {rows} rows (1..{GCHAIN_MAX_ROWS})")
    c.rows = int(rows)
    return c


def gchain_fwd(c, xcat, prev, x1, g, sg, xv, xp, xrv, xrp):
    st = lib().gasfm_gchain_fwd(ctypes.addressof(c), _p(xcat), _p(prev), _p(x1), _p(g), _p(sg), _p(xv), _p(xp),
                                _p(xrv), _p(xrp), _stream(g))
    check(st, "gasfm_gchain_fwd")


def gchain_bwd(c, xcat, x1, g, xv, xp, dskip, dsg, dxrv, dxrp, dxcat, dprev, grads):
    """grads: dict d<weight> -> tensor (gradient buffers to fill)."""
    d = _GChainGrads()
    for k in _GC_D:
        t = grads.get(k)
        if t is not None:
            setattr(d, k, t.data_ptr())
    L = lib()
    ws = torch.empty(int(L.gasfm_gchain_scratch_floats(ctypes.addressof(c))), dtype=torch.float32, device=g.device)
    cnt = _counters(g.device, L.gasfm_gchain_counters(ctypes.addressof(c)))
    st = L.gasfm_gchain_bwd(ctypes.addressof(c), _p(xcat), _p(x1), _p(g), _p(xv), _p(xp), _p(dskip), _p(dsg),
                            _p(dxrv), _p(dxrp), _p(dxcat), _p(dprev), ctypes.addressof(d), _p(ws), _p(cnt),
                            _stream(g))
    check(st, "gasfm_gchain_bwd")


# ---------------------------------------------------------------- global GATv2 convs (global_attn.hip)
class _GattProb(ctypes.Structure):
    _fields_ = [("XL", _vp), ("ldXL", _i64), ("src", _vp), ("S", _i32), ("HC", _i32), ("XR", _vp), ("att", _vp),
                ("bias", _vp), ("out", _vp), ("smax", _vp), ("ssum", _vp), ("part", _vp), ("gout", _vp),
                ("dXL", _vp), ("ldDXL", _i64), ("dXR", _vp), ("datt", _vp)]


def _gatt_probs(probs):
    """probs: dicts with XL [rows, HC] (unit column stride), src (int32 CUDA vector or None), S, XR,
    att, bias and the outputs of the direction; returns a ctypes array."""
    arr = (_GattProb * len(probs))()
    for q, d in enumerate(probs):
        XL = d["XL"]
        if not XL.is_cuda or XL.dtype != torch.float32 or XL.stride(1) != 1:
            raise TypeError("gatt: XL must be a float32 CUDA tensor with unit column stride")
        src = d.get("src")
        if src is not None and (src.dtype != torch.int32 or not src.is_contiguous()):
            raise TypeError("gatt: src must be a contiguous int32 tensor")
        a = arr[q]
        a.XL, a.ldXL, a.src, a.S, a.HC = XL.data_ptr(), XL.stride(0), _p(src), int(d["S"]), int(d["att"].numel())
        for k in ("XR", "att", "bias", "out", "smax", "ssum", "part", "gout", "dXR", "datt"):
            setattr(a, k, _p(d.get(k)))
        dXL = d.get("dXL")
        if dXL is not None:
            if dXL.stride(1) != 1:
                raise TypeError("gatt: dXL must have unit column stride")
            a.dXL, a.ldDXL = dXL.data_ptr(), dXL.stride(0)
    return arr


def gatt_fwd(probs, slope):
    """One launch: both global convs' forward (gasfm_gatt_fwd)."""
    arr = _gatt_probs(probs)
    L = lib()
    dev = probs[0]["XL"].device
    ws = torch.empty(int(L.gasfm_gatt_scratch_floats(len(probs), ctypes.addressof(arr))), dtype=torch.float32, device=dev)
    cnt = _counters(dev, int(L.gasfm_gatt_counters(len(probs), ctypes.addressof(arr))))
    check(L.gasfm_gatt_fwd(len(probs), ctypes.addressof(arr), float(slope), _p(ws), _p(cnt), _stream(probs[0]["XL"])),
          "gasfm_gatt_fwd")


def gatt_bwd(probs, slope):
    """One launch: both global convs' backward (gasfm_gatt_bwd)."""
    arr = _gatt_probs(probs)
    L = lib()
    dev = probs[0]["XL"].device
    ws = torch.empty(int(L.gasfm_gatt_scratch_floats(len(probs), ctypes.addressof(arr))), dtype=torch.float32, device=dev)
    cnt = _counters(dev, int(L.gasfm_gatt_counters(len(probs), ctypes.addressof(arr))))
    check(L.gasfm_gatt_bwd(len(probs), ctypes.addressof(arr), float(slope), _p(ws), _p(cnt), _stream(probs[0]["XL"])),
          "gasfm_gatt_bwd")


def gatt_merge(probs, nrows, stride, unpack=None):
    """One launch: merge the nrows gathered partial rows of each problem (probs[q]["part"]: the first
    row; rank r's at + r * stride floats) into its out / smax / ssum (gasfm_gatt_merge).  unpack =
    (G, blk, roff, chunk, dst [m, width]): the same launch also copies every rank's own rows out of
    the gathered send blocks G (gasfm_gatt_merge_unpack)."""
    arr = (_GattProb * len(probs))()
    for q, d in enumerate(probs):
        a = arr[q]
        a.HC = int(d["bias"].numel())
        for k in ("bias", "out", "smax", "ssum", "part"):
            setattr(a, k, _p(d[k]))
    if unpack is None:
        check(lib().gasfm_gatt_merge(len(probs), ctypes.addressof(arr), int(nrows), int(stride), _stream(d["bias"])),
              "gasfm_gatt_merge")
        return
    G, blk, roff, chunk, dst = unpack
    _exchange_args(G, dst, None)
    check(lib().gasfm_gatt_merge_unpack(len(probs), ctypes.addressof(arr), int(nrows), int(stride), _p(G), int(nrows),
                                        int(blk), int(roff), int(chunk), int(dst.shape[1]), int(dst.shape[0]), _p(dst),
                                        dst.stride(0) if dst.shape[0] > 1 else dst.shape[1], _stream(G)),
          "gasfm_gatt_merge_unpack")


def _exchange_args(G, rows_dst, sum_dst):
    for t, nm in ((G, "G"), (rows_dst, "rows_dst"), (sum_dst, "sum_dst")):
        if t is not None and (not t.is_cuda or t.dtype != torch.float32 or t.stride(-1) != 1):
            raise TypeError(f"exchange_unpack: {nm} must be float32 CUDA with unit column stride")


def exchange_unpack(G, W, blk, rows=None, sums=None):
    """Unpack W gathered send blocks of blk floats (gasfm_exchange_unpack): rows = (roff, chunk, dst
    [m, width]) copies every rank's own rows into dst, sums = (soff, dst [sn]) the rank-order sum of
    the W partial vectors."""
    roff, chunk, rdst = rows if rows is not None else (0, 1, None)
    soff, sdst = sums if sums is not None else (0, None)
    _exchange_args(G, rdst, sdst)
    width = int(rdst.shape[1]) if rdst is not None else 4
    m = int(rdst.shape[0]) if rdst is not None else 0
    ld = (rdst.stride(0) if m > 1 else width) if rdst is not None else 4
    check(lib().gasfm_exchange_unpack(_p(G), int(W), int(blk), int(roff), int(chunk), width, m, _p(rdst), ld,
                                      int(soff), int(sdst.numel()) if sdst is not None else 0, _p(sdst), _stream(G)),
          "gasfm_exchange_unpack")


# ---------------------------------------------------------------- device scene builder (scene_build.hip)
def scan_i32(x):
    """Exclusive scan of an int32 CUDA vector: returns out[L + 1] (out[L] = total)."""
    _i32vec(x, "scan input")
    out = torch.empty(x.shape[0] + 1, dtype=torch.int32, device=x.device)
    check(lib().gasfm_scan_i32(_p(x), x.shape[0], _p(out), _stream(x)), "gasfm_scan_i32")
    return out


# ---------------------------------------------------------------- outlier injection (outliers.hip)
def _dev_check(what, *ts):
    for name, t, dt in ts:
        if t is not None and (not t.is_cuda or t.dtype != dt or not t.is_contiguous()):
            raise TypeError(f"{what}: {name} must be a contiguous {dt} CUDA tensor")


def outlier_counts(state, cam_ptr, pt_ptr, perm, m, n):
    """Inliers per view / per point and their minima: (cam_in [m], pt_in [n], mins [2]) int32."""
    _dev_check("outlier_counts", ("state", state, torch.uint8), ("cam_ptr", cam_ptr, torch.int32),
               ("pt_ptr", pt_ptr, torch.int32), ("perm", perm, torch.int32))
    if cam_ptr.shape[0] != m + 1 or pt_ptr.shape[0] != n + 1:
        raise ValueError("outlier_counts: cam_ptr / pt_ptr must have m + 1 / n + 1 entries")
    dev = state.device
    cam_in = torch.empty(m, dtype=torch.int32, device=dev)
    pt_in = torch.empty(n, dtype=torch.int32, device=dev)
    mins = torch.empty(2, dtype=torch.int32, device=dev)
    check(lib().gasfm_outlier_counts(_p(state), _p(cam_ptr), _p(pt_ptr), _p(perm), m, n, _p(cam_in), _p(pt_in),
                                     _p(mins), _stream(state)), "gasfm_outlier_counts")
    return cam_in, pt_in, mins


def outlier_mark(state, cam, pt, cam_in, pt_in, mode, counts=None):
    """init (mode 0) / blacklist (mode 1) pass over the edge classes; returns counts [4] int32."""
    _dev_check("outlier_mark", ("state", state, torch.uint8), ("cam", cam, torch.int64), ("pt", pt, torch.int64),
               ("cam_in", cam_in, torch.int32), ("pt_in", pt_in, torch.int32))
    E = state.shape[0]
    if cam.shape[0] != E or pt.shape[0] != E:
        raise ValueError("outlier_mark: cam / pt must have one entry per edge")
    if counts is None:
        counts = torch.empty(4, dtype=torch.int32, device=state.device)
    check(lib().gasfm_outlier_mark(_p(state), _p(cam), _p(pt), _p(cam_in), _p(pt_in), E, mode, _p(counts),
                                   _stream(state)), "gasfm_outlier_mark")
    return counts


def outlier_moments(values, state, cam_ptr, m):
    """(mu [m, 2], sigma [m, 2, 2], scale_tril [m, 2, 2], pivots [m, 2] int32) of the inliers."""
    _dev_check("outlier_moments", ("values", values, torch.float32), ("state", state, torch.uint8),
               ("cam_ptr", cam_ptr, torch.int32))
    if values.dim() != 2 or values.shape[1] != 2 or values.shape[0] != state.shape[0] or cam_ptr.shape[0] != m + 1:
        raise ValueError("outlier_moments: values [E, 2], state [E], cam_ptr [m + 1]")
    dev = values.device
    mu = torch.empty((m, 2), dtype=torch.float32, device=dev)
    sigma = torch.empty((m, 2, 2), dtype=torch.float32, device=dev)
    tril = torch.empty((m, 2, 2), dtype=torch.float32, device=dev)
    piv = torch.empty((m, 2), dtype=torch.int32, device=dev)
    check(lib().gasfm_outlier_moments(_p(values), _p(state), _p(cam_ptr), m, _p(mu), _p(sigma), _p(tril), _p(piv),
                                      _stream(values)), "gasfm_outlier_moments")
    return mu, sigma, tril, piv


def outlier_apply(idx, cam, pt, z, mu, tril, M, pix=None):
    """Write mu[cam] + scale_tril[cam] z[k] for the outlier edges idx (ascending) into M (and pix)."""
    _dev_check("outlier_apply", ("idx", idx, torch.int64), ("cam", cam, torch.int64), ("pt", pt, torch.int64),
               ("z", z, torch.float32), ("mu", mu, torch.float32), ("scale_tril", tril, torch.float32),
               ("pix", pix, torch.float32))
    _check_M(M, "outlier_apply")
    k = idx.shape[0]
    if z.numel() != 2 * k:
        raise ValueError(f"outlier_apply: z has {z.numel()} values for {k} outliers")
    m = M.shape[0] // 2
    if mu.shape != (m, 2) or tril.shape != (m, 2, 2):
        raise ValueError("outlier_apply: mu [m, 2], scale_tril [m, 2, 2]")
    check(lib().gasfm_outlier_apply(_p(idx), k, _p(cam), _p(pt), _p(z), _p(mu), _p(tril), _p(M), M.stride(0),
                                    _p(pix), _stream(M)), "gasfm_outlier_apply")


def _check_M(M, what):
    if not M.is_cuda or M.dtype != torch.float32 or M.dim() != 2 or M.stride(1) != 1 or M.shape[0] % 2:
        raise TypeError(f"{what}: M must be a float32 CUDA [2m, n] matrix with unit column stride "
                        "(no CPU fallback)")


def scene_mask(M):
    """gasfm_scene_mask on a dense M: (mask [m*W] int64 bits, pt_valid [W], pt_count int32 [n] (views of
    points with >= 2, else 0), tile_base int32 [tiles + 1])."""
    _check_M(M, "scene_mask")
    m, n = M.shape[0] // 2, M.shape[1]
    L = lib()
    dev = M.device
    W, T = L.gasfm_scene_mask_words(n), L.gasfm_scene_tiles(m, n)
    i32 = dict(dtype=torch.int32, device=dev)
    mask = torch.empty(m * W, dtype=torch.int64, device=dev)
    pt_valid = torch.empty(W, dtype=torch.int64, device=dev)
    view_count, pt_count = torch.empty(n, **i32), torch.empty(n, **i32)
    tile_count, tile_base = torch.empty(T, **i32), torch.empty(T + 1, **i32)
    check(L.gasfm_scene_mask(_p(M), M.stride(0), m, n, _p(mask), _p(view_count), _p(pt_valid), _p(pt_count),
                             _p(tile_count), _p(tile_base), _stream(M)), "gasfm_scene_mask")
    return mask, pt_valid, pt_count, tile_base


def scene_homography(M, Ns, R, Ninv):
    """Rotational homography augmentation of a dense M (gasfm_scene_homography): new [2m, n] M."""
    _check_M(M, "scene_homography")
    m, n = M.shape[0] // 2, M.shape[1]
    for t, name in ((Ns, "Ns"), (R, "R"), (Ninv, "Ninv")):
        if not t.is_cuda or t.dtype != torch.float32 or tuple(t.shape) != (m, 3, 3) or not t.is_contiguous():
            raise TypeError(f"scene_homography: {name} must be a contiguous float32 CUDA [m, 3, 3] tensor")
    mask, pt_valid, _, _ = scene_mask(M)
    out = torch.empty_like(M)
    check(lib().gasfm_scene_homography(_p(M), M.stride(0), m, n, _p(mask), _p(pt_valid), _p(Ns), _p(R), _p(Ninv),
                                       _p(out), out.stride(0), _stream(M)), "gasfm_scene_homography")
    return out


def scene_build(M, Ns=None):
    """Dense M [2m, n] (CUDA fp32) -> dict of device tensors: cam, pt (int64 [E]), values [E, 2],
    pt_count (int32 [n], the reference's cam_per_pts), cam_ptr (int32 [m+1]), pt_ptr (int32 [n+1]),
    perm / pos (int32 [E]).  One host sync (E sizes the edge buffers)."""
    _check_M(M, "scene_build")
    m, n = M.shape[0] // 2, M.shape[1]
    if Ns is not None:
        if not Ns.is_cuda or Ns.dtype != torch.float32 or tuple(Ns.shape) != (m, 3, 3):
            raise TypeError("scene_build: Ns must be a float32 CUDA [m, 3, 3] tensor")
        Ns = Ns.contiguous()
    L = lib()
    dev = M.device
    T = L.gasfm_scene_tiles(m, n)
    i32 = dict(dtype=torch.int32, device=dev)
    mask, pt_valid, pt_count, tile_base = scene_mask(M)
    st = _stream(M)
    W = L.gasfm_scene_mask_words(n)
    E = int(tile_base[T].item())
    cam = torch.empty(E, dtype=torch.int64, device=dev)
    pt = torch.empty(E, dtype=torch.int64, device=dev)
    vals = torch.empty((E, 2), dtype=torch.float32, device=dev)
    word_base = torch.empty(m * W, **i32)
    check(L.gasfm_scene_emit(_p(M), M.stride(0), _p(Ns) if Ns is not None else None, m, n, _p(mask), _p(pt_valid),
                             _p(tile_base), _p(cam), _p(pt), _p(vals), _p(word_base), st), "gasfm_scene_emit")
    pt_ptr = scan_i32(pt_count)
    perm, pos = torch.empty(E, **i32), torch.empty(E, **i32)
    if E:
        check(L.gasfm_scene_point_csr(_p(mask), _p(pt_valid), _p(word_base), _p(pt_ptr), m, n, _p(perm), _p(pos),
                                      st), "gasfm_scene_point_csr")
    cam_ptr = tile_base[0::T // m].contiguous() if T else torch.zeros(m + 1, **i32)
    return {"cam": cam, "pt": pt, "values": vals, "pt_count": pt_count, "cam_ptr": cam_ptr, "pt_ptr": pt_ptr,
            "perm": perm, "pos": pos}


def sum_n(tensors):
    """Elementwise sum of same-shape contiguous fp32 CUDA tensors in one pass (gasfm_sum_n)."""
    t0 = tensors[0]
    for t in tensors:
        _req(t, "sum_n input")
        if t.shape != t0.shape:
            raise ValueError("sum_n: shapes differ")
    if t0.numel() % 4:  # the kernel streams float4s (odd E): pairwise adds on the device
        out = tensors[0].clone()
        for t in tensors[1:]:
            out += t
        return out
    out = torch.empty_like(t0)
    st = lib().gasfm_sum_n(len(tensors), _ptrs(tensors), t0.numel(), _p(out), _stream(t0))
    check(st, "gasfm_sum_n")
    return out


def _gemm(fn, what, a, b, cin=None, bias=None, out=None):
    for t, nm in ((a, what + " a"), (b, what + " b")):
        if not (t.is_cuda and t.dtype == torch.float32 and t.dim() == 2):
            raise ValueError(f"{nm}: fp32 CUDA matrix required")
    M, K = a.shape
    K2, N = b.shape
    if K2 != K:
        raise ValueError(f"{what}: inner dimensions {K} and {K2} differ")
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    if cin is not None and (cin.shape != (M, N) or cin.stride(1) != 1):
        raise ValueError(f"{what}: cin must be [M, N] with unit column stride")
    if bias is not None and (bias.shape != (N,) or not bias.is_contiguous()):
        raise ValueError(f"{what}: bias must be a contiguous [N] vector")
    if out.shape != (M, N) or out.stride(1) != 1:
        raise ValueError(f"{what}: out must be [M, N] with unit column stride")
    st = fn(M, N, K, _p(a), a.stride(0), a.stride(1), _p(b), b.stride(0), b.stride(1), _p(cin),
            cin.stride(0) if cin is not None else 0, _p(bias), _p(out), out.stride(0), _stream(out))
    check(st, what)
    return out


def gemm_bf16(a, b, cin=None, bias=None, out=None):
    """out = a @ b (+ cin) (+ bias) on bf16 MFMA with fp32 accumulation (gasfm_gemm_bf16).

    a [M, K], b [K, N]: fp32 CUDA tensors, each with a unit stride along one dimension (plain
    row-major tensors and their .t() views both qualify: x @ W.t(), dy @ W, dy.t() @ x)."""
    return _gemm(lib().gasfm_gemm_bf16, "gasfm_gemm_bf16", a, b, cin, bias, out)


def gemm_f32_smallm(a, b, cin=None, bias=None, out=None):
    """out = a @ b (+ cin) (+ bias) on the small-row-count fp32 MFMA kernels (csrc/gemm_smallm.hip),
    or None when the operand form / shape is not one of theirs: a @ W.t() (mode 0: a, W row-major),
    a @ W (mode 1, no epilogue), A.t() @ B (mode 2: A, B row-major, short K, no epilogue)."""
    if not (a.is_cuda and b.is_cuda and a.dtype == torch.float32 and b.dtype == torch.float32
            and a.dim() == 2 and b.dim() == 2 and a.shape[1] == b.shape[0]):
        return None
    M, K = a.shape
    N = b.shape[1]
    L = lib()
    if a.stride(1) == 1 and a.stride(0) % 4 == 0:
        if b.stride(0) == 1 and b.stride(1) % 4 == 0:  # b = W.t(), W [N, K] row-major
            mode, A, lda, B, ldb = 0, a, a.stride(0), b, b.stride(1)
        elif b.stride(1) == 1 and cin is None and bias is None:  # b = W [K, N] row-major
            mode, A, lda, B, ldb = 1, a, a.stride(0), b, b.stride(0)
        else:
            return None
        I, J = M, N
    elif a.stride(0) == 1 and b.stride(1) == 1 and cin is None and bias is None:  # a = A.t(), A [K, M]
        mode, A, lda, B, ldb = 2, a, a.stride(1), b, b.stride(0)
        I, J = M, N
    else:
        return None
    # modes 0 / 1 read float4 runs of A (and of W in mode 0): a misaligned view falls back to hipBLASLt
    if mode in (0, 1) and (A.data_ptr() % 16 or (mode == 0 and B.data_ptr() % 16)):
        return None
    if not L.gasfm_gemm_f32_smallm_ok(mode, I, J, K):
        return None
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    if out.shape != (M, N) or out.stride(1) != 1 or (cin is not None and (cin.shape != (M, N) or cin.stride(1) != 1)):
        return None
    if bias is not None and (bias.shape != (N,) or not bias.is_contiguous()):
        return None
    st = L.gasfm_gemm_f32_smallm(mode, I, J, K, _p(A), lda, _p(B), ldb, _p(bias), _p(cin),
                                 cin.stride(0) if cin is not None else 0, _p(out), out.stride(0), _stream(out))
    check(st, "gasfm_gemm_f32_smallm")
    return out


def gemm_f32(a, b, cin=None, bias=None, out=None):
    """out = a @ b (+ cin) (+ bias) in fp32 on v_mfma_f32_16x16x4_f32 (gasfm_gemm_f32); same
    operand rules as gemm_bf16.  out may be cin (accumulate in place)."""
    return _gemm(lib().gasfm_gemm_f32, "gasfm_gemm_f32", a, b, cin, bias, out)
