"""Weight-only quantized linears on the hand-written kernels of csrc/kernels/wo_gemm.hip.

Reference: paddle/phi/kernels/gpu/weight_only_linear_kernel.cu, llm_int8_linear_kernel.cu,
python/paddle/nn/quant/quantized_linear.py. Weights use the reference layout (weight_quantize): int8 [N, K] or
int4 pairs [N/2, K] (channels 2j / 2j+1 in the low / high nibble, stored +8), scales [N] or [K/G, N].

Decode shapes (M <= 64 rows) run ``pa_wo_gemm``: the weight bytes stream once and are dequantised in registers
in front of the MFMA. Longer inputs dequantise the weight once per call into a bf16 [N, K] image
(``pa_wo_dequant``) and run the bf16 MFMA GEMM on it (compute-bound there, the dequant pass is amortised).
"""
from __future__ import annotations

import torch

from . import _loader as L

DECODE_MAX_M = 64


def _scale_f32(scale):
    return scale if scale.dtype == torch.float32 else scale.float()


def available(x):
    return (x.is_cuda and L.has("pa_wo_gemm") and L.hip_enabled_for(x))


def dequantize(w, scale, bits, group, K, N):
    """bf16 [N, K] image of a quantized weight (device)."""
    out = torch.empty(N, K, dtype=torch.bfloat16, device=w.device)
    L.call("pa_wo_dequant", L.ptr(w.contiguous()), L.ptr(_scale_f32(scale).contiguous()), L.ptr(out), N, K, bits,
           group, L.stream_ptr())
    return out


def wo_linear(x, w, scale, bias, bits, group, llm=None):
    """y[..., N] = x[..., K] . dequant(w)^T (+ bias) for bf16 ``x``; ``llm`` = (xq, xo, sx) switches the decode
    kernel to LLM.int8 (x is then ignored)."""
    K = x.shape[-1]
    N = w.shape[0] * (2 if bits == 4 else 1)
    x2 = x.reshape(-1, K)
    M = x2.shape[0]
    if K % 64 or N % 16:
        raise ValueError(f"weight-only GEMM needs K % 64 == 0 and N % 16 == 0 (K={K}, N={N})")
    sc = _scale_f32(scale).contiguous()
    b = None if bias is None else bias.to(torch.bfloat16).contiguous()
    if M <= DECODE_MAX_M:
        y = torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
        nt = 1 if M <= 16 else (2 if M <= 32 else (2 if llm is not None else 4))
        if N % (16 * nt):
            raise ValueError(f"weight-only decode GEMM needs N % {16 * nt} == 0 at M = {M} (N={N})")
        splits = int(L.lib().pa_wo_gemm_splits(M, N, K, int(llm is not None)))
        ws = torch.empty(M * N, dtype=torch.float32, device=x.device) if splits > 1 else None
        if llm is not None:
            xq, xo, sx = llm
            L.call("pa_wo_gemm", L.ptr(xq), L.ptr(xo), L.ptr(sx), L.ptr(w), L.ptr(sc), L.ptr(b), L.ptr(y), L.ptr(ws),
                   M, N, K, K, N, 8, -1, splits, L.stream_ptr())
        else:
            x2 = x2.to(torch.bfloat16).contiguous()
            L.call("pa_wo_gemm", L.ptr(x2), L.ptr(None), L.ptr(None), L.ptr(w), L.ptr(sc), L.ptr(b), L.ptr(y),
                   L.ptr(ws), M, N, K, K, N, bits, group, splits, L.stream_ptr())
        return y.reshape(*x.shape[:-1], N)
    if llm is not None:
        raise ValueError("the LLM.int8 kernel takes decode shapes only (M <= 64)")
    from . import gemm as G
    wd = dequantize(w, scale, bits, group, K, N)        # [N, K]: B K-major
    x2 = x2.to(torch.bfloat16).contiguous()
    if G.supported(x2, wd.t()):
        y = G.gemm(x2, wd.t(), bias=b)
    else:
        y = x2 @ wd.t()
        if b is not None:
            y = y + b
    return y.reshape(*x.shape[:-1], N)
