"""ctypes binding of libjabd.so (the C-ABI declared in include/jabd.h).

This is the Python side of the drop-in boundary: every function of the
header is declared here with its exact C signature, and `call()` turns a
non-zero status into a RuntimeError carrying `jabd_last_error()`.

There is no fallback: if libjabd.so is missing or the HIP runtime is not
usable, `lib()` raises.  The library is loaded *after* torch so that its
libamdhip64.so.7 dependency binds to the HIP runtime torch already loaded
(one runtime per process, so torch streams are valid handles here).
"""
import ctypes
import os
import threading

import torch  # noqa: F401  (load torch's HIP runtime first; see docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
# JABD_LIB: an alternative build of the same ABI (A/B timing of kernel variants)
LIB_PATH = os.environ.get("JABD_LIB") or os.path.join(_HERE, "libjabd.so")

c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_f32 = ctypes.c_float
c_f64 = ctypes.c_double
c_size = ctypes.c_size_t
c_vp = ctypes.c_void_p
c_sizep = ctypes.POINTER(ctypes.c_size_t)

c_i32 = ctypes.c_int32
c_fp = ctypes.POINTER(ctypes.c_float)


class ConvArgs(ctypes.Structure):
    """Mirror of `jabd_conv_args` (include/jabd.h) — field order is the ABI."""
    _fields_ = [
        ("x", c_vp), ("x_bs", c_i64), ("x_ps", c_i32), ("x_c0", c_i32),
        ("B", c_i32), ("H", c_i32), ("W", c_i32), ("Cin", c_i32),
        ("x2", c_vp), ("x2_bs", c_i64), ("x2_ps", c_i32), ("Cin2", c_i32),
        ("x2_W", c_i32), ("x2_stride", c_i32),
        ("ascale", c_vp), ("ascale_bs", c_i64),
        ("w", c_vp), ("bias", c_vp),
        ("res", c_vp), ("res_bs", c_i64), ("res_ps", c_i32), ("res_c0", c_i32),
        ("y", c_vp), ("y_bs", c_i64), ("y_ps", c_i32), ("y_c0", c_i32),
        ("OH", c_i32), ("OW", c_i32), ("Cout", c_i32), ("Ntiles", c_i32), ("tn", c_i32),
        ("Kc", c_i32),
        ("KH", c_i32), ("KW", c_i32), ("stride", c_i32), ("pad", c_i32),
        ("act", c_i32), ("slope", c_f32),
        ("nchw_in", c_i32), ("tconv", c_i32),
        ("flags", c_i32), ("reserved1", c_i32),
        ("M", c_i64),
        ("w32", c_vp), ("ntiles32", c_i32), ("tn32", c_i32),
        ("y2", c_vp), ("y2_bs", c_i64), ("y2_ps", c_i32), ("y2_c0", c_i32), ("nsplit", c_i32),
        ("act2", c_i32), ("slope2", c_f32), ("reserved2", c_i32),
        ("ws", c_vp), ("ws_bytes", c_i64),
    ]


class DwArgs(ctypes.Structure):
    """Mirror of `jabd_dw_args` (include/jabd.h)."""
    _fields_ = [
        ("x", c_vp), ("x_bs", c_i64), ("x_ps", c_i32), ("reserved0", c_i32),
        ("B", c_i32), ("H", c_i32), ("W", c_i32), ("C", c_i32),
        ("w", c_vp), ("bias", c_vp),
        ("y", c_vp), ("y_bs", c_i64), ("y_ps", c_i32), ("reserved1", c_i32),
        ("OH", c_i32), ("OW", c_i32), ("k", c_i32), ("stride", c_i32), ("pad", c_i32),
        ("act", c_i32),
        ("slope", c_f32), ("nblk", c_i32),
        ("part", c_vp),
    ]


class ExpDwArgs(ctypes.Structure):
    """Mirror of `jabd_expdw_args` (include/jabd.h)."""
    _fields_ = [
        ("x", c_vp), ("x_bs", c_i64), ("x_ps", c_i32), ("Cin", c_i32),
        ("B", c_i32), ("H", c_i32), ("W", c_i32), ("E", c_i32),
        ("we", c_vp), ("be", c_vp), ("Ntiles", c_i32), ("Kc", c_i32),
        ("wd", c_vp), ("bd", c_vp),
        ("k", c_i32), ("stride", c_i32), ("act", c_i32), ("nblk", c_i32),
        ("y", c_vp), ("y_bs", c_i64), ("y_ps", c_i32), ("OH", c_i32), ("OW", c_i32),
        ("reserved0", c_i32),
        ("part", c_vp),
        ("sw", c_vp), ("sb", c_vp), ("sy", c_vp), ("sy_bs", c_i64), ("sy_ps", c_i32),
        ("reserved1", c_i32),
        ("pw", c_vp), ("pb", c_vp), ("pg", c_vp), ("pres", c_vp), ("pg_bs", c_i32), ("pact", c_i32),
    ]


class WindowCopy(ctypes.Structure):
    """Mirror of `jabd_window_copy` (include/jabd.h)."""
    _fields_ = [
        ("src", c_vp), ("dst", c_vp),
        ("s0", c_i32), ("s1", c_i32), ("s2", c_i32),
        ("d0", c_i32), ("d1", c_i32), ("d2", c_i32),
        ("off2", c_i32), ("fill", c_f32), ("scale", c_f32), ("reserved", c_i32),
    ]


WINDOW_MAX = 32  # JABD_WINDOW_MAX


# name -> argtypes (every function returns int status unless listed in _RESTYPE)
SIGNATURES = {
    "jabd_version": [],
    "jabd_abi_struct_size": [c_i32],
    "jabd_last_error": [ctypes.c_char_p, c_size],
    "jabd_decode_f32": [c_vp, c_vp, c_i64, c_i64, c_f32, c_f32, c_vp, c_vp],
    "jabd_decode_landm_f32": [c_vp, c_vp, c_i64, c_i64, c_f32, c_vp, c_vp],
    "jabd_nms_workspace_size": [c_i64, c_i64, c_sizep],
    "jabd_batched_nms_f32": [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64,
                             c_f64, c_f32, c_vp, c_vp, c_vp, c_size, c_vp],
    "jabd_nms_pair_stats": [c_vp, c_size, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp],
    "jabd_sort_workspace_size": [c_i64, c_i32, c_sizep],
    "jabd_sort_u64": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_vp, c_size, c_vp],
    "jabd_scan_workspace_size": [c_i64, c_sizep],
    "jabd_scan_excl_i32": [c_vp, c_vp, c_i64, c_vp, c_size, c_vp],
    "jabd_detect_workspace_size": [c_i64, c_i64, c_sizep],
    "jabd_detect_f32": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_f32, c_f32, c_f32, c_f64,
                        c_vp, c_vp, c_vp, c_size, c_vp],
    "jabd_match_workspace_size": [c_i64, c_i64, c_sizep],
    "jabd_match_encode_f32": [c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_f32, c_f32, c_f32,
                              c_vp, c_vp, c_vp, c_vp, c_size, c_vp],
    "jabd_multibox_workspace_size": [c_i64, c_i64, c_sizep],
    "jabd_multibox_loss_fwd_f32": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_int,
                                   c_vp, c_vp, c_vp, c_vp, c_size, c_vp],
    "jabd_multibox_loss_bwd_f32": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                   c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "jabd_multibox_loss_finalize_f32": [c_vp, c_vp, c_vp, c_vp],
    "jabd_letterbox_f32": [c_vp, c_i64, c_int, c_int, c_vp, c_int, c_int, c_f32, c_vp, c_int,
                           c_vp],
    "jabd_correct_boxes_f32": [c_vp, c_i64, c_int, c_int, c_int, c_int, c_int, c_int, c_vp],
    "jabd_augment_workspace_size": [c_int, c_int, c_sizep],
    "jabd_augment_u8": [c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                        c_f64, c_f32, c_f32, c_vp, c_vp, c_size, c_vp],
    "jabd_wider_eval_workspace_size": [c_i64, c_i64, c_sizep],
    "jabd_wider_eval_f64": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_f64, c_int,
                            c_vp, c_vp, c_size, c_vp],
    "jabd_upsample_bicubic_ac_f32": [c_vp, c_i64, c_int, c_int, c_int, c_vp, c_int, c_int, c_vp],
    "jabd_upsample_bicubic_ac_bwd_f32": [c_vp, c_i64, c_int, c_int, c_int, c_vp, c_int, c_int,
                                         c_vp],
    "jabd_nlm_attn_fwd_f32": [c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp],
    "jabd_nlm_attn_bwd_f32": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32,
                              c_vp, c_vp, c_vp, c_vp],
    "jabd_window_copy_multi_f32": [c_i32, ctypes.POINTER(WindowCopy), c_vp],
    "jabd_transpose_f32": [c_vp, c_i32, c_i32, c_vp, c_vp],
    "jabd_colsum_f32": [c_vp, c_i64, c_i32, c_vp, c_vp],
    "jabd_sum_multi_f32": [c_i32, ctypes.POINTER(c_vp), c_i64, c_vp, c_vp],
    "jabd_weighted_sum3_f32": [c_vp, c_vp, c_vp, c_f32, c_vp, c_vp],
    "jabd_conv_w2d_f32": [c_vp, c_i32, c_i32, c_i32, c_vp, c_vp],
    "jabd_heads_wpack_f32": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32,
                             c_vp, c_i32, c_vp, c_i32, c_vp],
    "jabd_nlm_attn_dkv_ws_floats": [c_i32, c_i32, c_i32, c_i32],
    "jabd_nlm_attn_dkv_f32": [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_i64,
                              c_vp, c_vp, c_vp],
    "jabd_add3_f32": [c_vp, c_vp, c_vp, c_i64, c_vp, c_vp],
    "jabd_beca_ws_floats": [c_i64, c_i64, c_int],
    "jabd_conv_pack_multi_f32": [c_vp, c_vp, c_i32, c_i64, c_vp],
    "jabd_ssh_tail_weight_floats": [],
    "jabd_ssh_tail_heads_f32": [c_vp, c_i64, c_i32, c_vp, c_i64, c_i32, c_i32, c_i32, c_vp, c_f32,
                                c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp],
    "jabd_conv_pack_f32": [c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_i32,
                           c_i32, c_vp, c_vp],
    "jabd_beca_fwd_f32": [c_vp, c_i64, c_i64, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_i64, c_vp],
    "jabd_beca_bwd_f32": [c_vp, c_vp, c_i64, c_i64, c_int, c_vp, c_int, c_vp, c_vp, c_vp, c_vp,
                          c_vp, c_i64, c_vp],
    "jabd_match_iou_f32": [c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, c_f32, c_f32, c_f32,
                           c_vp, c_vp, c_vp, c_vp, c_size, c_vp],
    "jabd_multibox_diou_loss_fwd_f32": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32,
                                        c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_vp, c_size,
                                        c_vp],
    "jabd_multibox_diou_loss_bwd_f32": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32,
                                        c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "jabd_conv_pack_tn": [c_int],
    "jabd_conv_pack_tn32": [c_int],
    "jabd_conv2d_nhwc_f32": [ctypes.POINTER(ConvArgs), c_vp],
    "jabd_conv1x1_bn_stats_nblk": [ctypes.POINTER(ConvArgs)],
    "jabd_conv1x1_bn_stats_f32": [ctypes.POINTER(ConvArgs), c_vp, c_i64, c_vp, c_vp],
    "jabd_conv_workspace_size": [ctypes.POINTER(ConvArgs)],
    "jabd_conv_bn_stats_part_floats": [ctypes.POINTER(ConvArgs)],
    "jabd_conv_bn_bwd_part_floats": [ctypes.POINTER(ConvArgs)],
    "jabd_conv_bn_bwd_sums_f32": [ctypes.POINTER(ConvArgs), c_vp, c_i32, c_vp, c_vp, c_vp, c_vp,
                                  c_i32, c_f32, c_vp, c_i64, c_vp],
    "jabd_conv_bn_bwd_sums_res_f32": [ctypes.POINTER(ConvArgs), c_vp, c_i32, c_vp, c_i32, c_vp,
                                      c_vp, c_vp, c_i64, c_vp],
    "jabd_bn_act_bwd_rows_f32": [c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_i32,
                                 c_f32, c_vp, c_vp, c_vp, c_vp],
    "jabd_conv_bn_stats_f32": [ctypes.POINTER(ConvArgs), c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                               c_f32, c_f32, c_vp],
    "jabd_stem_nchw_f32": [c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_i32, c_vp, c_vp],
    "jabd_dw_nblk": [c_i64, c_i64, c_i64, c_i64],
    "jabd_dwconv_nhwc_f32": [ctypes.POINTER(DwArgs), c_vp],
    "jabd_dwconv_stats_nblk": [c_i64, c_i64, c_i64, c_i64],
    "jabd_dwconv_stats_f32": [ctypes.POINTER(DwArgs), c_vp, c_vp, c_vp],
    "jabd_dwconv_bnin_stats_f32": [ctypes.POINTER(DwArgs), c_vp, c_vp, c_vp, c_vp, c_i32, c_f32,
                                   c_vp, c_vp, c_vp],
    "jabd_bn_stats_final_f32": [c_vp, c_vp, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_f32,
                                c_f32, c_vp],
    "jabd_expand_dw_nblk": [c_i32, c_i32, c_i32, c_i32],
    "jabd_expand_dw_nhwc_f32": [ctypes.POINTER(ExpDwArgs), c_vp],
    "jabd_expand_dw_select": [c_i32],
    "jabd_channel_sum_f32": [c_vp, c_i64, c_i32, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp],
    "jabd_partial_reduce_f32": [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp],
    "jabd_eca_gate_f32": [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i32, c_i32, c_vp, c_vp,
                          c_vp],
    "jabd_nlm_pool_f32": [c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp,
                          c_vp, c_vp, c_vp, c_i32, ctypes.POINTER(c_i32), c_i32, c_vp, c_vp,
                          c_vp, c_vp],
    "jabd_nlm_apply_f32": [c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp,
                           c_vp, c_vp, c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                           c_vp],
    "jabd_maxpool_nhwc_f32": [c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp],
    "jabd_heads_scatter_f32": [c_vp, c_i32, c_i64, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp],
    "jabd_heads_f32": [c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_i64, c_i64, c_i32,
                       c_vp, c_vp, c_vp, c_vp],
    # training (A11)
    "jabd_bn_nblk": [c_i64, c_i32],
    "jabd_bn_stats_f32": [c_vp, c_i32, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_f32,
                          c_vp],
    "jabd_bn_act_fwd_f32": [c_vp, c_i32, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32,
                            c_i32, c_f32, c_vp, c_i32, c_i32, c_vp],
    "jabd_bn_act_bwd_f32": [c_vp, c_i32, c_i32, c_vp, c_i32, c_vp, c_i32, c_i64, c_i32, c_vp,
                            c_vp, c_vp, c_vp, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "jabd_conv_wgrad_part_floats": [ctypes.POINTER(ConvArgs)],
    "jabd_conv_wgrad_f32": [ctypes.POINTER(ConvArgs), c_vp, c_vp, c_vp],
    "jabd_eca_pool_gate_multi_f32": [c_i32, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                     c_vp, c_i32, c_vp, c_vp],
    "jabd_bn_sum_nblk": [c_i64, c_i32],
    "jabd_bn_act_fwd_sum_f32": [c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_vp, c_i32, c_f32, c_vp,
                                c_i64, c_vp, c_vp],
    "jabd_conv_wgrad_eca_part_floats": [ctypes.POINTER(ConvArgs)],
    "jabd_conv_wgrad_eca_f32": [ctypes.POINTER(ConvArgs), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "jabd_eca_gate_bwd_f32": [c_vp, c_i32, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_i32, c_i32,
                              c_vp, c_vp, c_vp, c_vp],
    "jabd_dw_dgrad_f32": [c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32,
                          c_i32, c_vp, c_vp],
    "jabd_dw_wgrad_part_floats": [c_i64, c_i32, c_i32],
    "jabd_dw_dgrad_bn_part_floats": [c_i32, c_i32, c_i32, c_i32],
    "jabd_dw_dgrad_bn_bwd_f32": [c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32,
                                 c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_f32, c_vp,
                                 c_vp, c_vp, c_vp, c_vp, c_vp],
    "jabd_dw_wgrad_f32": [c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32,
                          c_i32, c_vp, c_vp, c_vp],
    "jabd_dw_wgrad_bnin_f32": [c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32,
                               c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i32, c_f32, c_vp, c_vp,
                               c_vp],
    "jabd_eca_bwd_f32": [c_vp, c_vp, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_i32, c_i32, c_vp,
                         c_i32, c_vp, c_vp, c_vp, c_vp, c_vp],
    "jabd_scale_bwd_f32": [c_vp, c_vp, c_i64, c_i64, c_i32, c_vp, c_vp, c_i32, c_vp, c_vp],
    "jabd_eca_bwd_terms_f32": [c_vp, c_vp, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_i32, c_i32,
                               c_vp, c_i32, c_vp, c_vp, c_vp, c_vp],
    "jabd_bn_act_bwd_ex_f32": [c_vp, c_i32, c_i32, c_vp, c_i32, c_vp, c_i32, c_i64, c_i32, c_vp,
                               c_vp, c_vp, c_vp, c_i32, c_f32, c_vp, c_vp, c_i64, c_vp, c_vp,
                               c_vp, c_vp, c_vp, c_vp],
    "jabd_heads_gather_f32": [c_vp, c_vp, c_vp, c_i32, c_i64, c_i64, c_i32, c_vp, c_vp],
    "jabd_nlm_bwd_attn_f32": [c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_i32, c_vp,
                              c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "jabd_nlm_bwd_proj_f32": [c_vp, c_vp, c_i32, c_i32, ctypes.POINTER(c_i32), c_i32, c_i32,
                              c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp],
    "jabd_upsample_nearest_bwd_f32": [c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32,
                                      c_vp, c_vp],
    "jabd_upsample_nearest_f32": [c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp],
    "jabd_maxpool_bwd_f32": [c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp,
                             c_vp],
    "jabd_maxpool_idx_nhwc_f32": [c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp,
                                  c_vp, c_vp],
    "jabd_maxpool_bwd_idx_f32": [c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32,
                                 c_vp, c_vp],
    "jabd_adam_num_chunks": [c_vp, c_i64],
    "jabd_adam_fill_chunks": [c_vp, c_i64, c_vp],
    "jabd_adam_step_f32": [c_vp, c_vp, c_i64, c_f64, c_f64, c_f64, c_f64, c_f64, c_f64, c_f64,
                           c_vp],
    # module-level ops (csrc/modules.hip)
    "jabd_act_f32": [c_vp, c_i64, c_i32, c_f32, c_vp, c_vp],
    "jabd_act_bwd_f32": [c_vp, c_vp, c_i64, c_i32, c_f32, c_vp, c_vp],
    "jabd_bn_eval_f32": [c_vp, c_i64, c_i32, c_vp, c_vp, c_f32, c_vp, c_vp, c_i32, c_f32, c_vp,
                         c_vp],
    "jabd_channel_scale_f32": [c_vp, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp],
    "jabd_adaptive_pool_ws_floats": [c_i32, c_i32, c_i32, ctypes.POINTER(c_i32), c_i32],
    "jabd_adaptive_pool_f32": [c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, ctypes.POINTER(c_i32),
                               c_i32, c_vp, c_vp, c_i64, c_vp],
    "jabd_upsample_nearest_add_f32": [c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp,
                                      c_vp],
    "jabd_adaptive_pool_bwd_f32": [c_vp, c_i32, c_i32, c_i32, c_i32, ctypes.POINTER(c_i32),
                                   c_i32, c_vp, c_vp],
}
_RESTYPE = {"jabd_version": ctypes.c_char_p, "jabd_dw_nblk": ctypes.c_int64,
            "jabd_expand_dw_nblk": ctypes.c_int64,
            "jabd_bn_nblk": ctypes.c_int64, "jabd_conv_wgrad_part_floats": ctypes.c_int64,
            "jabd_conv_wgrad_eca_part_floats": ctypes.c_int64, "jabd_bn_sum_nblk": ctypes.c_int64,
            "jabd_dw_wgrad_part_floats": ctypes.c_int64,
            "jabd_dw_dgrad_bn_part_floats": ctypes.c_int64,
            "jabd_dwconv_stats_nblk": ctypes.c_int64,
            "jabd_conv1x1_bn_stats_nblk": ctypes.c_int64,
            "jabd_conv_bn_stats_part_floats": ctypes.c_int64,
            "jabd_conv_bn_bwd_part_floats": ctypes.c_int64,
            "jabd_adam_num_chunks": ctypes.c_int64, "jabd_beca_ws_floats": ctypes.c_int64,
            "jabd_adaptive_pool_ws_floats": ctypes.c_int64,
            "jabd_abi_struct_size": ctypes.c_int64, "jabd_conv_workspace_size": ctypes.c_int64,
            "jabd_ssh_tail_weight_floats": ctypes.c_int64,
            "jabd_nlm_attn_dkv_ws_floats": ctypes.c_int64}

_lock = threading.Lock()
_lib = None


def lib():
    """Load libjabd.so once (thread-safe) and declare every signature."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"libjabd.so not built at {LIB_PATH}; run __graft_entry__.build() "
                    "(the HIP path has no CPU fallback)")
            h = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
            for name, args in SIGNATURES.items():
                fn = getattr(h, name)
                fn.argtypes = args
                fn.restype = _RESTYPE.get(name, ctypes.c_int)
            _lib = h
    return _lib


def last_error() -> str:
    buf = ctypes.create_string_buffer(512)
    lib().jabd_last_error(buf, 512)
    return buf.value.decode(errors="replace")


def call(name, *args):
    st = getattr(lib(), name)(*args)
    if st != 0:
        raise RuntimeError(f"{name} failed (status {st}): {last_error()}")


def exported_symbols():
    """Names declared in include/jabd.h that the loaded library must export."""
    return list(SIGNATURES)
