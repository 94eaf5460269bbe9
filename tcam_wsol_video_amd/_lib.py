"""ctypes binding of libtcam_hip.so (the C ABI declared in include/tcam_hip.h).

The library is built in-tree by ``__graft_entry__.build()`` (or
``python -m tcam_wsol_video_amd.build``).  There is no CPU fallback: if the
library is missing every op raises :class:`NativeLibraryError`.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# TCAM_LIB_PATH: another build of the same ABI (A/B timing of two builds on one box)
LIB_PATH = os.environ.get("TCAM_LIB_PATH") or os.path.join(_HERE, "libtcam_hip.so")

_lib = None


class NativeLibraryError(RuntimeError):
    pass


class tcam_conv_src(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("C", C.c_int), ("H", C.c_int), ("W", C.c_int),
                ("stride", C.c_int), ("up2", C.c_int)]


class tcam_pack_item(C.Structure):
    _fields_ = [("w", C.c_void_p), ("out", C.c_void_p), ("wscale", C.c_void_p),
                ("kdiv", C.c_void_p), ("mode", C.c_int), ("CoutW", C.c_int), ("CtotW", C.c_int),
                ("KH", C.c_int), ("KW", C.c_int), ("c0", C.c_int), ("cout_sel", C.c_int),
                ("cin_pad", C.c_int)]


class tcam_conv_dst(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("c_begin", C.c_int), ("cstride", C.c_int),
                ("coff", C.c_int)]


class tcam_conv_prob(C.Structure):
    _fields_ = [("src", tcam_conv_src), ("wt", C.c_void_p), ("wscale", C.c_void_p),
                ("bias", C.c_void_p), ("out", C.c_void_p)] + [
        (n, C.c_int) for n in ("Cout", "Hout", "Wout", "KH", "KW", "pad_h", "pad_w", "relu",
                               "out_cstride", "out_coff")]


_P = C.c_void_p
_I = C.c_int
_F = C.c_float

# name -> (restype, argtypes); must mirror include/tcam_hip.h.
SIGNATURES = {
    "tcam_abi_version": (_I, []),
    "tcam_arch": (C.c_char_p, []),
    "tcam_conv2d": (_I, [C.POINTER(tcam_conv_src), _I, _I, _P, _P, _P, _P, _I, _I, _I,
                         _I, _I, _I, _I, _P]),
    "tcam_conv_weight_dims": (_I, [_I, _I, C.POINTER(_I), C.POINTER(_I)]),
    "tcam_conv_force_tile": (_I, [_I]),
    "tcam_conv2d_x6": (_I, [C.POINTER(tcam_conv_src), _I, _I, _P, _P, _P, _P, _I, _I, _I,
                            _I, _I, _I, _I, _I, _I, _I, _P, C.c_size_t, _P]),
    "tcam_conv2d_x6_multi": (_I, [C.POINTER(tcam_conv_src), _I, _I, _P, _P, _I, _I, _I, _I,
                                  _I, _I, _I, _I, C.POINTER(tcam_conv_dst), _I, _P, C.c_size_t,
                                  _P]),
    "tcam_conv2d_f16x3": (_I, [C.POINTER(tcam_conv_src), _I, _I, _P, _P, _P, _P, _P, _I, _I,
                               _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, C.c_size_t, _P]),
    "tcam_conv2d_f16x3_multi": (_I, [C.POINTER(tcam_conv_src), _I, _I, _P, _P, _P, _I, _I,
                                     _I, _I, _I, _I, _I, _I, C.POINTER(tcam_conv_dst), _I, _P,
                                     _P, C.c_size_t, _P]),
    "tcam_conv2d_group": (_I, [C.POINTER(tcam_conv_prob), _I, _I, _I, _I, _P, _P]),
    "tcam_conv_x6_ws_bytes": (C.c_size_t, []),
    "tcam_conv_x6_weight_dims": (_I, [_I, _I, C.POINTER(_I), C.POINTER(_I)]),
    "tcam_conv_x6_force_tile": (_I, [_I]),
    "tcam_wgrad_force_fp32": (_I, [_I]),
    "tcam_resample_coeffs": (_I, [_I, _I, _P, _P]),
    "tcam_frames_preprocess": (_I, [_P, _I, _I, _I, _P, _P, _I, _I, _P, _P, _I, _I, _P, _P,
                                    _I, _I, C.POINTER(_F), C.POINTER(_F), _P, _P, _P, _P]),
    "tcam_jpeg_pack": (_I, [_P, _P, _I, _P, C.c_size_t, _P, _P]),
    "tcam_jpeg_decode": (_I, [_P, _P, _P, C.c_size_t, _P, _P]),
    "tcam_jpeg_debug_rounds": (_I, [_P, _P]),
    "tcam_conv_x6_force_streamk": (_I, [_I]),
    "tcam_conv_x6_debug": (_I, [_I]),
    "tcam_s3_from_nchw": (_I, [_P, _P, _I, _I, _I, _I, _I, _P]),
    "tcam_s3_to_nchw": (_I, [_P, _P, _I, _I, _I, _I, _P]),
    "tcam_maxpool3x3s2_s3": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_up2_resize_s3": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_pool2d_s3": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_wgap_s3_ws_bytes": (C.c_size_t, [_I, _I, _I]),
    "tcam_wgap_s3": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "tcam_seghead_cam_s3": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "tcam_resize_cam": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_resize_ac_bwd": (_I, [_P, _P, _I, _I, _I, _I, _I, _P]),
    "tcam_std_cam_s3": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_s2_from_nchw": (_I, [_P, _P, _I, _I, _I, _I, _I, _P]),
    "tcam_s2_to_nchw": (_I, [_P, _P, _I, _I, _I, _I, _P]),
    "tcam_maxpool3x3s2_s2": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_up2_resize_s2": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_pool2d_s2": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_wgap_s2": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "tcam_seghead_cam_s2": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "tcam_std_cam_s2": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_maxpool3x3s2": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_up2_resize": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_wgap": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "tcam_seghead_cam": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "tcam_std_cam": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_temporal_max": (_I, [_P, _P, _P, _I, _I, _I, _F, _P]),
    "tcam_temporal_cam": (_I, [_P, _I, _P, _P, _P, _I, _I, _I, _F, _P, _P]),
    "tcam_topk_flags": (_I, [_P, _P, _P, _P, _I, _I, _P]),
    "tcam_bbox_ws_bytes": (C.c_size_t, [_I, _I, _I]),
    "tcam_bbox_multi_ws_bytes": (C.c_size_t, [_I, _I, _I]),
    "tcam_bbox_multi_iou": (_I, [_P, _P, _P, _I, _P, _P, _P, _P, _I, _I, _I, _P]),
    "tcam_box_accumulate_multi": (_I, [_P, _P, _P, _P, _I, _P, _P, _I, _P, _P, _P, _I, _P, _P,
                                       _I, _P]),
    "tcam_bbox_contours_ws_bytes": (C.c_size_t, [_I, _I]),
    "tcam_bbox_contours": (_I, [_P, _I, _P, _I, _P, _P, _I, _I, _P]),
    "tcam_flag_count": (_I, [_P, _I, _P, _P]),
    "tcam_bbox_levels": (_I, [_P, _P, _P, _P, _I, _I, _I, _P]),
    "tcam_bbox_scan_line": (_I, [_P, _P, _P, _I, _I, _P]),
    "tcam_s2_to_s3": (_I, [_P, _P, C.c_long, _P]),
    "tcam_s3_to_s2": (_I, [_P, _P, C.c_long, _P]),
    "tcam_bbox_set_debug": (_I, [_P]),
    "tcam_bbox_fill_variant": (_I, [_I]),
    "tcam_bbox_level_variant": (_I, [_I]),
    "tcam_bbox_set_inc_debug": (_I, [_P]),
    "tcam_box_accumulate": (_I, [_P, _P, _P, _I, _P, _P, _I, _P, _P, _P, _I, _P, _P, _I,
                                 _P]),
    "tcam_bilateral_ws_bytes": (C.c_size_t, [_I, _I, _I, _I, _I]),
    "tcam_bilateral_batch": (_I, [_P, _P, _P, _P, C.c_size_t, _I, _I, _I, _I, _F, _F, _P]),
    "tcam_bilateral_prepare": (_I, [_P, _P, C.c_size_t, _I, _I, _I, _I, _F, _F, _P]),
    "tcam_bilateral_apply": (_I, [_P, _P, _P, C.c_size_t, _I, _I, _I, _I, _F, _F, _P]),
    "tcam_colorbilateral_batch": (_I, [_P, _P, _P, _P, C.c_size_t, _I, _I, _I, _I, _F, _I,
                                       _P]),
    "tcam_bilateral_status": (_I, [_P, _I, C.POINTER(_I)]),
    "tcam_bilateral_set_debug": (None, [_P]),
    "tcam_crf_energy_ws_bytes": (C.c_size_t, []),
    "tcam_bn_ws_bytes": (C.c_size_t, [C.c_long, _I]),
    "tcam_bn_stats_s3": (_I, [_P, C.c_long, _I, _F, _F, _P, _P, _P, _P, _P, _P]),
    "tcam_bn_relu_s3": (_I, [_P, _P, _P, _P, _P, _P, C.c_long, _I, _P]),
    "tcam_bn_relu_bwd_s3": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, C.c_long, _I, _P, _P]),
    "tcam_up2_bwd_s3": (_I, [_P, _P, _I, _I, _I, _I, _P]),
    "tcam_conv_wgrad_ws_bytes": (C.c_size_t, [C.POINTER(tcam_conv_src), _I, _I, _I, _I, _I,
                                              _I, _I]),
    "tcam_conv_wgrad_s3": (_I, [C.POINTER(tcam_conv_src), _I, _I, _P, _I, _I, _I, _I, _I, _I,
                                _I, _I, _P, _P, C.c_size_t, _P]),
    "tcam_timer_arm": (_I, [_P, _P]),
    "tcam_bn_stats_s2": (_I, [_P, C.c_long, _I, _F, _F, _P, _P, _P, _P, _P, _P]),
    "tcam_bn_relu_s2": (_I, [_P, _P, _P, _P, _P, _P, C.c_long, _I, _P]),
    "tcam_bn_relu_bwd_s3s2": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, C.c_long, _I, _P, _P,
                                   _P]),
    "tcam_dy_scaled_s2": (_I, [_P, C.c_long, _I, _P, _I, _P, _P, _P]),
    "tcam_bn_bwd_scaled_ws_bytes": (C.c_size_t, [C.c_long, _I]),
    "tcam_bn_relu_bwd_scaled_s3s2": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                          C.c_long, _I, _P, _P]),
    "tcam_bn_relu_bwd_fused_s1": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, C.c_long, _I,
                                       _P, _P]),
    "tcam_conv_wgrad_s2_f16x3": (_I, [C.POINTER(tcam_conv_src), _I, _I, _P, _P, _I, _I, _I, _I,
                                      _I, _I, _I, _I, _P, _P, C.c_size_t, _P]),
    "tcam_pack_weight_f16x3": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    "tcam_pack_table_bytes": (C.c_size_t, [_I]),
    "tcam_pack_weights": (_I, [_P, _I, _I, _P, _P]),
    "tcam_bottleneck_set_debug": (None, [_P]),
    "tcam_bbox_set_chunks": (None, [_I]),
    "tcam_bottleneck_f16": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _P, _P]),
    "tcam_bottleneck_f16x3": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I,
                                   _P, _P, _P]),
    "tcam_conv2d_f16x3_s3out": (_I, [C.POINTER(tcam_conv_src), _I, _I, _P, _P, _P, _P, _I, _I,
                                     _I, _I, _I, _I, _I, _I, _I, _I, _P, C.c_size_t, _P]),
    "tcam_conv_wgrad_s3_f16x3": (_I, [C.POINTER(tcam_conv_src), _I, _I, _P, _I, _I, _I, _I, _I,
                                      _I, _I, _I, _P, _P, C.c_size_t, _P, _P]),
    "tcam_pack_weight_x6": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_up2_resize_bwd_s3": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_chansum_ws_bytes": (C.c_size_t, [_I, _I, C.c_long]),
    "tcam_chansum_nchw": (_I, [_P, _I, _I, C.c_long, _P, _P, _P]),
    "tcam_softmax2": (_I, [_P, _P, _I, C.c_long, _P]),
    "tcam_tcam_loss_ws_bytes": (C.c_size_t, [_I, C.c_long]),
    "tcam_tcam_losses": (_I, [_P, _P, _P, _P, _I, C.c_long, _F, _F, _F, _F, _P, _P, _P, _P]),
    "tcam_tcam_losses_ex": (_I, [_P, _P, _P, _P, _P, _P, _I, C.c_long, _F, _F, _F, _F, _P, _P,
                                 _P, _P]),
    "tcam_mosaic_gather": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P]),
    "tcam_mosaic_scatter": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _F, _I, _P, _P]),
    "tcam_sgd_step": (_I, [_P, _P, _P, C.c_long, _F, _F, _F, _F, _I, _I, _F, _P]),
    "tcam_sgd_step_gated": (_I, [_P, _P, _P, C.c_long, _F, _F, _F, _F, _I, _F, _P, _P, _P,
                                 _P]),
    "tcam_seeder_ws_bytes": (C.c_size_t, [_I, _I, _I]),
    "tcam_prepare_std_cams": (_I, [_P, _P, _I, _I, _I, _I, _I, _P]),
    "tcam_tcam_seeder": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _F, _F, _I, _I, _I, _I, _I,
                              C.c_double, _I, C.c_ulonglong, C.c_ulonglong, _P, _P, _P,
                              C.c_size_t, _P]),
    "tcam_get_roi": (_I, [_P, _I, _I, _I, _I, C.c_double, C.c_double, _P, _P, _P, _P, _P,
                          C.c_size_t, _P]),
    "tcam_stotsu_roi_thresh": (_I, [_P, _I, _I, _I, _I, _P, _P]),
    "tcam_crf_energy": (_I, [_P, _P, C.c_long, _I, _P, _P, _P]),
    "tcam_crf_grad": (_I, [_P, _P, C.c_long, _I, _P, _P]),
    "tcam_stem_window": (_I, [_I, _I, _I, C.POINTER(_I), C.POINTER(_I)]),
    "tcam_stem_f16x3": (_I, [_P, _P, _P, _P, _P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I,
                             _P, _P]),
    # AMP path (S1 activations, fp16 convolutions, GradScaler)
    "tcam_conv2d_f16": (_I, [C.POINTER(tcam_conv_src), _I, _I, _P, _P, _P, _P, _I, _I, _I,
                             _I, _I, _I, _I, _I, _I, _I, _P, C.c_size_t, _P]),
    "tcam_s1_from_nchw": (_I, [_P, _P, _I, _I, _I, _I, _I, _P]),
    "tcam_s1_to_nchw": (_I, [_P, _P, _I, _I, _I, _I, _P]),
    "tcam_maxpool3x3s2_s1": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_up2_resize_s1": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_pool2d_s1": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_wgap_s1": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "tcam_seghead_cam_s1": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "tcam_std_cam_s1": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_bn_stats_s1": (_I, [_P, C.c_long, _I, _F, _F, _P, _P, _P, _P, _P, _P]),
    "tcam_bn_relu_s1": (_I, [_P, _P, _P, _P, _P, _P, C.c_long, _I, _P]),
    "tcam_bn_relu_bwd_s1": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, C.c_long, _I, _P, _P]),
    "tcam_up2_bwd_s1": (_I, [_P, _P, _I, _I, _I, _I, _P]),
    "tcam_up2_resize_bwd_s1": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_conv_wgrad_s1": (_I, [C.POINTER(tcam_conv_src), _I, _I, _P, _I, _I, _I, _I, _I, _I,
                                _I, _I, _P, _P, C.c_size_t, _P]),
    "tcam_pack_weight_f16": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_amp_unscale": (_I, [_P, C.c_long, _P, _P, _P]),
    "tcam_sgd_step_amp": (_I, [_P, _P, _P, C.c_long, _F, _F, _F, _F, _I, _F, _P, _P, _P, _P,
                               _P, _F, _F, _I, _P]),
    # encoder training step (stage 1, STD_CL; csrc/enc_train.hip)
    "tcam_bn_add_relu_s2": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, C.c_long, _I,
                                 _P]),
    "tcam_bn_add_relu_s1": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, C.c_long, _I,
                                 _P]),
    "tcam_grad_add_mask_s3s2": (_I, [_P, _P, _P, _P, C.c_long, _I, _P]),
    "tcam_grad_add_mask_s1": (_I, [_P, _P, _P, _P, C.c_long, _I, _P]),
    "tcam_maxpool_bwd_ws_bytes": (C.c_size_t, [_I, _I, _I, _I]),
    "tcam_maxpool3x3s2_bwd_s3s2": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_maxpool3x3s2_bwd_s1": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_zero_up2": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_im2col": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "tcam_wgrad11_ws_bytes": (C.c_size_t, [_I, _I, _I, _I, _I, _I, _I, _I]),
    "tcam_wgrad11_s2_f16x3": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _I, _I, _I, _P, _P,
                                   C.c_size_t, _P]),
    "tcam_wgrad11_s1": (_I, [_P, _I, _I, _I, _I, _I, _P, _I, _I, _I, _P, _P, C.c_size_t, _P]),
    "tcam_conv_wgrad_generic_ws_bytes": (C.c_size_t, [C.POINTER(tcam_conv_src), _I, _I, _I, _I,
                                                      _I, _I, _I]),
    "tcam_conv_wgrad_s3s2": (_I, [C.POINTER(tcam_conv_src), _I, _I, _P, _I, _I, _I, _I, _I, _I,
                                  _I, _I, _P, _P, C.c_size_t, _P]),
    "tcam_cls_pool_ws_bytes": (C.c_size_t, [_I, _I]),
    "tcam_cls_fwd_s2": (_I, [_P, _I, C.c_long, _I, _P, _P, _I, _P, _P, _P, _P]),
    "tcam_cls_fwd_s1": (_I, [_P, _I, C.c_long, _I, _P, _P, _I, _P, _P, _P, _P]),
    "tcam_ce_loss": (_I, [_P, _P, _I, _I, _F, _P, _P, _P, _P]),
    "tcam_cls_bwd": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P]),
    "tcam_pool_bwd_s3": (_I, [_P, _I, C.c_long, _I, _P, _P]),
    "tcam_pool_bwd_s1": (_I, [_P, _I, C.c_long, _I, _P, _P]),
    "bilateralfilter_batch": (None, [_P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _F, _F]),
    "colorbilateralfilter_batch": (None, [_P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _F, _I]),
}


def load(path: str = LIB_PATH):
    """Load (once) and return the native library; raise loudly if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise NativeLibraryError(
            f"{path} not found: build it with `python -c 'import __graft_entry__ as g; "
            f"g.build()'` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with code {rc}")
