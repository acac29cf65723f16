"""Signature table of every exported launcher in _C_hip.so (see csrc/kernels/*.hip).

Single source of truth for both launch paths: ``_loader`` sets the ctypes argtypes from it, and
``tools/build_native.py`` generates the native METH_FASTCALL entry points of ``_C_dispatch`` from it
(csrc/dispatch/dispatch_gen.inc). Pure ctypes, no package imports, so the build can load it by path.
"""
import ctypes

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int
_f32 = ctypes.c_float
_u64 = ctypes.c_uint64

SIGS = {
    # norms
    "pa_rms_norm_fwd": [_vp, _vp, _vp, _vp, _i64, _i64, _f32, _i32, _vp],
    "pa_rms_norm_bwd": [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _vp],
    "pa_rms_norm_bwd_res": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _vp],
    "pa_layer_norm_fwd": [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _f32, _i32, _vp],
    "pa_layer_norm_bwd": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _vp],
    "pa_reduce_parts": [_vp, _vp, _vp, _vp, _i32, _i64, _i32, _i32, _vp],
    # softmax / cross entropy
    "pa_softmax_fwd": [_vp, _vp, _i64, _i64, _i32, _vp],
    "pa_softmax_bwd": [_vp, _vp, _vp, _i64, _i64, _i32, _vp],
    "pa_softmax_ce_fwd": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp],
    "pa_softmax_ce_bwd": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp],
    "pa_ce_slice_fwd": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp],
    "pa_ce_slice_bwd": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i32, _vp],
    # activations
    "pa_gelu_fwd": [_vp, _vp, _i64, _i32, _i32, _vp],
    "pa_gelu_bwd": [_vp, _vp, _vp, _i64, _i32, _i32, _vp],
    "pa_swiglu_fwd": [_vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp],
    "pa_swiglu_bwd": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp],
    "pa_bias_gelu_fwd": [_vp, _vp, _vp, _i64, _i64, _i32, _vp],
    # rope
    "pa_rope_fwd": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i32, _i32, _vp],
    "pa_rope_rows": [_vp, _i64, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _vp],
    # optimizer
    "pa_adamw_multi": [_vp, _vp, _i64, _vp, _f32, _f32, _f32, _f32, _f32, _f32, _f32, _vp, _vp],
    "pa_adam_hyper_step": [_vp, _f32, _f32, _vp],
    "pa_sq_norm_multi": [_vp, _vp, _i64, _vp, _vp],
    "pa_scale_multi": [_vp, _i64, _vp, _vp],
    "pa_write_i64": [_vp, _vp, _i64, _vp],
    "pa_bn_set_target_wgs": [_i32],
    "pa_momentum_multi": [_vp, _vp, _i64, _vp, _f32, _f32, _f32, _i32, _vp],
    # attention
    "pa_flash_attn_fwd": [_vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _f32, _i32, _vp],
    "pa_flash_attn_bwd": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                          _i32, _i32, _i32, _i32, _i32, _i32, _f32, _i32, _vp],
    "pa_flash_attn_fwd_ex": [_vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _f32, _i32, _vp,
                             _vp],
    "pa_flash_attn_bwd_ex": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                             _i32, _i32, _i32, _i32, _i32, _i32, _f32, _i32, _i64, _vp, _vp],
    "pa_flash_attn_bwd_ds": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                             _i32, _i32, _i32, _i32, _i32, _i32, _f32, _i32, _vp, _vp],
    "pa_flash_attn_bwd_ds_ok": [_i32, _i32, _i32, _i32, _i32],
    "pa_flash_attn_bwd_ds_bytes": [_i32, _i32, _i32, _i32],
    "pa_fa_fm_stats": [_vp, _i32, _i32, _i32, _i32, _i32, _i64, _i64, _i32, _vp, _vp],
    "pa_paged_decode_attn": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32,
                             _i64, _i64, _f32, _vp],
    # gemm epilogue companions
    "pa_colsum": [_vp, _vp, _vp, _i64, _i64, _i32, _vp],
    "pa_dwconv_fwd": [_vp, _vp, _vp, _vp, _vp, _i32, _vp],
    "pa_dwconv_dgrad": [_vp, _vp, _vp, _vp, _vp, _i32, _vp],
    "pa_dwconv_wgrad_parts": [_vp, _vp],
    "pa_dwconv_wgrad": [_vp, _vp, _vp, _vp, _i32, _vp],
    "pa_gemm_bf16": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _f32,
                     _i32, _i32, _vp],
    "pa_gemm_bf16_pp": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _f32,
                        _vp, _vp],
    "pa_gemm_bf16_4w": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _f32,
                        _vp, _vp],
    "pa_gemm_bf16_res": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _vp, _vp],
    "pa_gemm_bf16_dgelu": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _vp],
    "pa_gemm_bf16_pp_segs": [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32,
                             _i32, _f32, _vp, _vp],
    "pa_gemm_pp_ws_bytes": [_i64, _i64, _i64],
    "pa_gemm_pp_splitk_ws_bytes": [_i64, _i64, _i32],
    "pa_gemm_bf16_pp_splitk": [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _f32, _i32, _vp,
                               _vp],
    "pa_gemm_fp8": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _f32, _i32, _i32, _vp],
    "pa_gemm_fp8_set_kernel": [_i32],
    "pa_gemm_fp8_ws": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _f32, _i32, _i32, _vp, _vp],
    "pa_gemm_fp8_ws_bytes": [_i64, _i64, _i64],
    "pa_gemm_bf16_4w_abl": [_vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp],
    "pa_gemm_small_m": [_vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _vp],
    "pa_gemm_skinny": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _vp],
    # weight-only int8 / int4 GEMM and LLM.int8 (csrc/kernels/wo_gemm.hip)
    "pa_wo_gemm": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp],
    "pa_wo_gemm_splits": [_i64, _i64, _i64, _i32],
    "pa_wo_dequant": [_vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp],
    "pa_gemm_skinny_ok": [_i64, _i64],
    "pa_gemm_skinny_stats_chunks": [_i64, _i64, _i64],
    "pa_gemm_skinny_stats": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _vp, _vp],
    "pa_conv_skinny_stats_chunks": [_i64, _i64, _i64],
    "pa_conv_skinny_stats": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _vp, _vp],
    "pa_conv_skinny": [_vp, _vp, _vp, _vp, _vp] + [_i64] * 11 + [_vp],
    "pa_conv_skinny_ok": [_i64, _i64, _i64, _i64],
    "pa_conv_skinny_wgrad": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _vp],
    "pa_conv2d_nhwc_fwd": [_vp, _vp, _vp, _vp, _vp] + [_i32] * 13 + [_vp],
    "pa_conv3d_ndhwc_fwd": [_vp, _vp, _vp, _vp, _vp] + [_i32] * 17 + [_vp],
    "pa_conv2d_nhwc_fwd_stats": [_vp, _vp, _vp, _vp, _vp] + [_i32] * 13 + [_vp, _vp],
    "pa_gemm_stats_chunks": [_i64, _i32],
    "pa_slab_reduce_bf16": [_vp, _vp, _i64, _i64, _i64, _i32, _vp],
    "pa_gemm_bf16_bnbwd": [_vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _vp, _vp, _vp, _vp,
                           _vp],
    "pa_conv2d_nhwc_fwd_bnbwd": [_vp, _vp, _vp, _vp] + [_i32] * 13 + [_vp, _vp, _vp, _vp, _vp],
    "pa_gemm_bf16_stats": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _i32, _vp,
                           _vp],
    "pa_conv2d_nhwc_wgrad": [_vp, _vp, _vp, _vp] + [_i32] * 15 + [_vp],
    "pa_bias_gelu_bwd": [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _vp],
    "pa_dropout_add_fwd": [_vp, _vp, _vp, _i64, _f32, _u64, _i32, _vp],
    "pa_dropout_bwd": [_vp, _vp, _i64, _f32, _u64, _i32, _vp],
    "pa_dropout_bwd_colsum": [_vp, _vp, _vp, _i64, _i64, _f32, _u64, _i32, _vp],
    "pa_colsum_nparts": [_i64],
    "pa_fold_partials": [_vp, _vp, _i64, _i64, _i32, _vp],
    # batch norm (NHWC)
    "pa_bn_chunks": [_i64, _i32],
    "pa_bn_fwd_nhwc": [_vp] * 11 + [_i64, _i32, _f32, _f32, _i32, _i32, _vp],
    "pa_bn_bwd_nhwc": [_vp] * 12 + [_i64, _i32, _i32, _i32, _vp, _vp],
    "pa_bn_reduce_nhwc": [_i32] + [_vp] * 7 + [_i64, _i32, _i32, _vp],
    "pa_bn_fwd_nhwc_mask": [_vp] * 12 + [_i64, _i32, _f32, _f32, _i32, _vp],
    "pa_bn_bwd_nhwc_mask": [_vp] * 12 + [_i64, _i32, _i32, _vp],
    "pa_bn_bwd_apply_nhwc": [_vp] * 6 + [_i64, _i32, _i32, _vp, _vp],
    "pa_bn_pre_ws": [_i32, _i32],
    "pa_bn_bwd_nhwc_pre": [_vp] * 9 + [_i32, _vp, _vp, _i64, _i32, _i32, _vp, _vp],
    "pa_bn_fwd_nhwc_pre": [_vp] * 10 + [_i32, _vp, _vp, _vp, _i64, _i32, _f32, _f32, _i32, _vp],
    # fused decode step
    "pa_add_rms_norm_fwd": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _f32, _i32, _vp],
    "pa_decode_rope_cache": [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _i64, _i32, _vp],
    # pooling
    "pa_maxpool_nhwc_fwd": [_vp, _vp, _vp] + [_i32] * 10 + [_vp],
    "pa_maxpool_nhwc_bwd": [_vp, _vp, _vp] + [_i32] * 10 + [_vp],
    # MoE
    "pa_grouped_gemm": [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i64, _i32, _i32, _i32, _i64, _i64, _i64, _i32,
                        _vp],
    "pa_moe_route": [_vp, _i32, _i32, _vp, _vp, _vp, _vp],
    "pa_version": [],
}

RET_I64 = {"pa_flash_attn_bwd_ds_bytes", "pa_gemm_pp_ws_bytes", "pa_gemm_fp8_ws_bytes", "pa_gemm_pp_splitk_ws_bytes", "pa_bn_pre_ws", "pa_gemm_skinny_stats_chunks", "pa_conv_skinny_stats_chunks",
           "pa_colsum_nparts"}
