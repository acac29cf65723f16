"""Loader for the hand-written CDNA4 (gfx950) HIP kernel library ``_C_hip.so``.

The library is a plain C-ABI shared object compiled by ``tools/build_native.py`` with
``hipcc --offload-arch=gfx950``. It is loaded with ctypes *after* torch so that it binds to
the HIP runtime instance that torch already loaded (same soname ``libamdhip64.so.7``).

On a machine with a HIP device the kernels are the path that runs; if the library is missing
there we fail loudly (set ``PADDLE_AMD_ALLOW_FALLBACK=1`` to permit the ATen fallback, e.g. for
debugging). On CPU-only hosts the ATen/CPU reference implementations run.
"""
from __future__ import annotations

import ctypes
import os

import torch

from ..framework.flags import flag

_LIB = None
_LIB_ERR = None
_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "_C_hip.so")


def _load():
    global _LIB, _LIB_ERR
    if _LIB is not None or _LIB_ERR is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        _LIB_ERR = f"{LIB_PATH} not built (run: python tools/build_native.py)"
        return None
    try:
        import torch  # noqa: F401  (bind to torch's HIP runtime first)
        _LIB = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover
        _LIB_ERR = str(e)
        return None
    _declare(_LIB)
    return _LIB


def lib():
    l = _load()
    if l is None:
        raise RuntimeError(f"paddlepaddle_amd HIP kernels unavailable: {_LIB_ERR}")
    return l


def hip_enabled_for(t: torch.Tensor) -> bool:
    """True if a HIP kernel should run for a tensor on this device."""
    if not t.is_cuda or not flag("FLAGS_use_hip_kernels", True):
        return False
    if type(t) is not torch.Tensor and type(t) is not torch.nn.Parameter:
        return False  # distributed / wrapper tensors (auto-parallel DTensor) take the sharding-aware path
    if _load() is None:
        if os.environ.get("PADDLE_AMD_ALLOW_FALLBACK", "0") == "1":
            return False
        raise RuntimeError(f"HIP device present but native kernels missing: {_LIB_ERR}")
    return True


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int
_f32 = ctypes.c_float


def _declare(L):
    """Argument types of every exported launcher (see csrc/kernels/*.hip)."""
    sigs = {
        # norms
        "pa_rms_norm_fwd": [_vp, _vp, _vp, _vp, _i64, _i64, _f32, _i32, _vp],
        "pa_rms_norm_bwd": [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _vp],
        "pa_layer_norm_fwd": [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _f32, _i32, _vp],
        "pa_layer_norm_bwd": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _vp],
        "pa_reduce_parts": [_vp, _vp, _vp, _vp, _i32, _i64, _i32, _i32, _vp],
        # softmax / cross entropy
        "pa_softmax_fwd": [_vp, _vp, _i64, _i64, _i32, _vp],
        "pa_softmax_bwd": [_vp, _vp, _vp, _i64, _i64, _i32, _vp],
        "pa_softmax_ce_fwd": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp],
        "pa_softmax_ce_bwd": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp],
        # activations
        "pa_gelu_fwd": [_vp, _vp, _i64, _i32, _i32, _vp],
        "pa_gelu_bwd": [_vp, _vp, _vp, _i64, _i32, _i32, _vp],
        "pa_swiglu_fwd": [_vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp],
        "pa_swiglu_bwd": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp],
        "pa_bias_gelu_fwd": [_vp, _vp, _vp, _i64, _i64, _i32, _vp],
        # rope
        "pa_rope_fwd": [_vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i32, _i32, _vp],
        # optimizer
        "pa_adamw_multi": [_vp, _vp, _i64, _vp, _f32, _f32, _f32, _f32, _f32, _f32, _f32, _vp, _vp],
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
        "pa_fa_fm_stats": [_vp, _i32, _i32, _i32, _i32, _i32, _i64, _i64, _i32, _vp, _vp],
        "pa_paged_decode_attn": [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32,
                                 _i64, _i64, _f32, _vp],
        # gemm epilogue companions
        "pa_colsum": [_vp, _vp, _vp, _i64, _i64, _i32, _vp],
        "pa_gemm_bf16": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _f32,
                         _i32, _i32, _vp],
        "pa_gemm_bf16_pp": [_vp, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _i32, _i32, _f32,
                            _vp, _vp],
        "pa_gemm_pp_ws_bytes": [_i64, _i64, _i64],
        "pa_gemm_small_m": [_vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _vp],
        "pa_conv2d_nhwc_fwd": [_vp, _vp, _vp, _vp, _vp] + [_i32] * 13 + [_vp],
        "pa_conv2d_nhwc_wgrad": [_vp, _vp, _vp, _vp] + [_i32] * 15 + [_vp],
        "pa_bias_gelu_bwd": [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i32, _vp],
        "pa_dropout_add_fwd": [_vp, _vp, _vp, _i64, _f32, ctypes.c_uint64, _i32, _vp],
        "pa_dropout_bwd": [_vp, _vp, _i64, _f32, ctypes.c_uint64, _i32, _vp],
        # batch norm (NHWC)
        "pa_bn_chunks": [_i64, _i32],
        "pa_bn_fwd_nhwc": [_vp] * 11 + [_i64, _i32, _f32, _f32, _i32, _i32, _vp],
        "pa_bn_bwd_nhwc": [_vp] * 12 + [_i64, _i32, _i32, _i32, _vp, _vp],
        "pa_bn_reduce_nhwc": [_i32] + [_vp] * 7 + [_i64, _i32, _i32, _vp],
        "pa_bn_bwd_apply_nhwc": [_vp] * 6 + [_i64, _i32, _i32, _vp, _vp],
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
    for name, args in sigs.items():
        fn = getattr(L, name, None)
        if fn is None:
            continue
        fn.argtypes = args
        fn.restype = _i64 if name in _RET_I64 else _i32


_RET_I64 = {"pa_gemm_pp_ws_bytes"}


def has(name):
    l = _load()
    return l is not None and hasattr(l, name)


# per-launcher dispatch counters: tests assert that the HIP path (not a fallback) ran
CALLS: dict = {}


def calls(name):
    return CALLS.get(name, 0)


def reset_calls():
    CALLS.clear()


def call(name, *args):
    CALLS[name] = CALLS.get(name, 0) + 1
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"HIP kernel {name} failed with code {rc}")


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


_DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}


def dcode(t):
    return _DT[t.dtype]
