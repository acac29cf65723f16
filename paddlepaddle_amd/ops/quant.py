"""Weight-only quantized linears on the hand-written kernels of csrc/kernels/wo_gemm.hip.

Reference: paddle/phi/kernels/gpu/weight_only_linear_kernel.cu, llm_int8_linear_kernel.cu,
python/paddle/nn/quant/quantized_linear.py. Weights use the reference layout (weight_quantize): int8 [N, K] or
int4 pairs [N/2, K] (channels 2j / 2j+1 in the low / high nibble, stored +8), scales [N] or [K/G, N].

Decode shapes (M <= 64 rows) run ``pa_wo_gemm`` — the weight bytes stream once and are dequantised in registers in
front of the MFMA — or the bf16 small-M GEMM on a cached dequantised image, whichever the per-shape timing
(ops.gemm.choose, key "wo_linear") finds faster: the decode kernel wins where the weight stream dominates, the bf16
GEMM where the activation rows make the product compute-bound (profiles/weight_only_gemm_r4.log). Longer inputs
run the bf16 MFMA GEMM on the cached image. The image cache (``dequantized``) is bounded by
FLAGS_weight_only_dequant_cache_mb (0: no cache — every long call dequantises, decode always streams the quantised
weight) and keyed by the weight / scale storage and version, so an updated weight is re-dequantised.
LLM.int8 above the decode shapes (``llm_int8_gemm``) also runs on the MFMA GEMM: the inlier columns enter as the
exact int8 values, the outlier columns as x / sx, against the cached bf16 copy of the int8 weight, with the
row / channel scales applied to the fp32 result.
"""
from __future__ import annotations

from collections import OrderedDict

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


_DQ_CACHE = OrderedDict()  # key -> bf16 image (LRU)


def _cache_budget():
    return int(L.flag("FLAGS_weight_only_dequant_cache_mb", 4096)) << 20


def dequantized(w, scale, bits, group, K, N, raw=False):
    """Cached bf16 [N, K] image of a quantized weight (``raw``: the int8 values without the scale, LLM.int8); None
    when the cache is off or the image does not fit its budget."""
    budget = _cache_budget()
    nbytes = N * K * 2
    if budget <= 0 or nbytes > budget:
        return None
    key = (w.data_ptr(), w._version, tuple(w.shape), None if raw else (scale.data_ptr(), scale._version),
           bits, group, raw)
    img = _DQ_CACHE.get(key)
    if img is not None:
        _DQ_CACHE.move_to_end(key)
        return img
    img = w.to(torch.bfloat16) if raw else dequantize(w, scale, bits, group, K, N)
    _DQ_CACHE[key] = img
    total = sum(v.numel() * 2 for v in _DQ_CACHE.values())
    while total > budget and len(_DQ_CACHE) > 1:
        _, old = _DQ_CACHE.popitem(last=False)
        total -= old.numel() * 2
    return img


def _bf16_linear(x2, wd, b):
    """x2 . wd^T (+ b) on the per-shape choice of the hand-written / vendor bf16 GEMM (ops/linear.py)."""
    from .linear import _fwd_mm
    return _fwd_mm(x2, wd.t(), b)


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
        nt = 1 if M <= 16 else (2 if M <= 32 else (2 if llm is not None else 4))
        if N % (16 * nt):
            raise ValueError(f"weight-only decode GEMM needs N % {16 * nt} == 0 at M = {M} (N={N})")
        splits = int(L.lib().pa_wo_gemm_splits(M, N, K, int(llm is not None)))
        if llm is None:
            x2 = x2.to(torch.bfloat16).contiguous()

        def decode():
            y = torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
            ws = torch.empty(M * N, dtype=torch.float32, device=x.device) if splits > 1 else None
            if llm is not None:
                xq, xo, sx = llm
                L.call("pa_wo_gemm", L.ptr(xq), L.ptr(xo), L.ptr(sx), L.ptr(w), L.ptr(sc), L.ptr(b), L.ptr(y),
                       L.ptr(ws), M, N, K, K, N, 8, -1, splits, L.stream_ptr())
            else:
                L.call("pa_wo_gemm", L.ptr(x2), L.ptr(None), L.ptr(None), L.ptr(w), L.ptr(sc), L.ptr(b), L.ptr(y),
                       L.ptr(ws), M, N, K, K, N, bits, group, splits, L.stream_ptr())
            return y
        # the bf16 GEMM on the cached image as the alternative (LLM.int8: its device path below)
        img = dequantized(w, scale, bits, group, K, N, raw=llm is not None)
        if img is not None:
            from . import gemm as G
            if llm is not None:
                alt = (lambda: llm_int8_gemm(None, w, scale, b, llm=llm, img=img))
            else:
                alt = (lambda: _bf16_linear(x2, img, b))
            key = ("wo_linear", M, N, K, bits if llm is None else "llm.int8", group)
            if G.choose(key, {"wo": decode, "bf16": alt}, cold=True) == "bf16":
                return alt().reshape(*x.shape[:-1], N)
        return decode().reshape(*x.shape[:-1], N)
    if llm is not None:
        return llm_int8_gemm(None, w, scale, b, llm=llm).reshape(*x.shape[:-1], N)
    x2 = x2.to(torch.bfloat16).contiguous()
    wd = dequantized(w, scale, bits, group, K, N)
    if wd is None:
        wd = dequantize(w, scale, bits, group, K, N)        # [N, K]: B K-major
    return _bf16_linear(x2, wd, b).reshape(*x.shape[:-1], N)


def llm_int8_gemm(x2, w, scale, bias, llm, img=None):
    """LLM.int8 on the MFMA GEMM for any row count: y = sw * sx * ((xq + xo / sx) . Wq^T) (+ bias). The inlier
    columns are the exact int8 values (xq; the outlier columns of xq are 0), the outlier columns enter as xo / sx,
    Wq is the bf16 copy of the int8 weight (exact), the product accumulates in fp32 and the row scale sx and channel
    scale sw multiply the fp32 result. ``llm`` = (xq, xo, sx) from nn.quant._llm_split."""
    xq, xo, sx = llm
    K = w.shape[1]
    N = w.shape[0]
    if img is None:
        img = dequantized(w, scale, 8, -1, K, N, raw=True)
        if img is None:
            img = w.to(torch.bfloat16)
    sxf = sx.float().reshape(-1, 1)
    a = (xq.float() + xo.float() / sxf).to(torch.bfloat16).contiguous()
    from . import gemm as G
    wt = img.t()
    if G.supported(a, wt):
        acc = G.gemm(a, wt, out_dtype=torch.float32)
    else:
        acc = a.float() @ wt.float()
    y = acc * sxf * _scale_f32(scale).reshape(1, -1)
    if bias is not None:
        y = y + bias.float()
    return y.to(torch.bfloat16)
