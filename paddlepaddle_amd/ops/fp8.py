"""fp8 GEMM with a fused bias / activation epilogue on the gfx950 block-scaled MFMA (csrc/kernels/gemm_fp8.hip).

Reference: python/paddle/tensor/linalg.py fp8_fp8_half_gemm_fused, paddle/phi/kernels/fusion/fp8_gemm/.
OCP e4m3fn / e5m2 operands (gfx950's native encodings, not the fnuz variants), fp32 accumulation,
fp16 / bf16 output: out = act(alpha * x @ y + bias)."""
from __future__ import annotations

import torch

from . import _loader as L

_FMT = {torch.float8_e4m3fn: 0, torch.float8_e5m2: 1}
_ACT = {"identity": 0, "none": 0, "gelu": 1, "relu": 2}


def _ref(a, b_nk, bias, alpha, act, out_dtype):
    y = alpha * (a.float() @ b_nk.float().t())
    if bias is not None:
        y = y + bias.float()
    if act == "gelu":
        y = torch.nn.functional.gelu(y)
    elif act == "relu":
        y = torch.relu(y)
    return y.to(out_dtype)


def hip_ok(a, b_nk, bias, out_dtype):
    return (L.hip_enabled_for(a) and L.has("pa_gemm_fp8") and a.dtype in _FMT and b_nk.dtype in _FMT
            and a.dim() == 2 and b_nk.dim() == 2 and a.shape[1] % 128 == 0 and b_nk.shape[0] % 4 == 0
            and out_dtype in (torch.float16, torch.bfloat16) and a.stride(1) == 1 and b_nk.stride(1) == 1
            and a.stride(0) % 16 == 0 and b_nk.stride(0) % 16 == 0 and a.data_ptr() % 16 == 0
            and b_nk.data_ptr() % 16 == 0 and (bias is None or bias.is_contiguous()))


def set_kernel(kind):
    """fp8 GEMM kernel choice: "auto" (the ping-pong 256x256 schedule when N % 8 == 0, else the generic kernel) or
    "generic"; returns the previous choice (A/B measurements and tests)."""
    global _KERNEL
    old, _KERNEL = _KERNEL, kind
    L.call("pa_gemm_fp8_set_kernel", {"auto": 0, "generic": 1}[kind])
    return old


_KERNEL = "auto"


def gemm_fp8(a, b_nk, bias=None, alpha=1.0, act="identity", out_dtype=torch.float16):
    """a [M, K] and b_nk [N, K] fp8 (both K-major) -> [M, N] in out_dtype."""
    if act not in _ACT:
        raise ValueError(f"fp8 GEMM: unsupported activation {act!r} (identity / relu / gelu)")
    M, K = a.shape
    N = b_nk.shape[0]
    if b_nk.shape[1] != K:
        raise ValueError(f"fp8 GEMM: inner dimensions differ ({K} vs {b_nk.shape[1]})")
    if not hip_ok(a, b_nk, bias, out_dtype):
        if a.is_cuda and L.hip_enabled_for(a) and a.dtype in _FMT and a.shape[1] % 128 == 0 \
                and b_nk.shape[0] % 4 == 0:
            a, b_nk = a.contiguous(), b_nk.contiguous()
            if hip_ok(a, b_nk, bias, out_dtype):
                return gemm_fp8(a, b_nk, bias, alpha, act, out_dtype)
        return _ref(a, b_nk, bias, alpha, act, out_dtype)
    out = torch.empty(M, N, dtype=out_dtype, device=a.device)
    bias_c = None if bias is None else bias.to(out_dtype).contiguous()
    if L.has("pa_gemm_fp8_ws"):  # the ping-pong kernel's balanced tail: K-sliced last wave of tiles
        nb = int(L.lib().pa_gemm_fp8_ws_bytes(M, N, K))
        ws = torch.empty(nb // 4, dtype=torch.float32, device=a.device) if nb else None
        L.call("pa_gemm_fp8_ws", L.ptr(a), L.ptr(b_nk), L.ptr(out), L.ptr(bias_c), M, N, K, a.stride(0),
               b_nk.stride(0), out.stride(0), _FMT[a.dtype], _FMT[b_nk.dtype], float(alpha), _ACT[act],
               1 if out_dtype == torch.float16 else 0, L.ptr(ws), L.stream_ptr())
        return out
    L.call("pa_gemm_fp8", L.ptr(a), L.ptr(b_nk), L.ptr(out), L.ptr(bias_c), M, N, K, a.stride(0), b_nk.stride(0),
           out.stride(0), _FMT[a.dtype], _FMT[b_nk.dtype], float(alpha), _ACT[act],
           1 if out_dtype == torch.float16 else 0, L.stream_ptr())
    return out
