"""paddle.nn.quant — weight-only int8 / int4 and LLM.int8 linears (hand-written kernels: ops/quant.py), QAT /
PTQ layers. Reference: python/paddle/nn/quant/ (quantized_linear.py:56,183,276)."""
from __future__ import annotations

import torch

from ...framework.tensor import _wrap
from ...tensor._helpers import T


_ALGOS = ("weight_only_int8", "weight_only_int4", "llm.int8")


def _check_group(group_size):
    if group_size not in (-1, 64, 128):
        raise ValueError(f"group_size must be -1, 64 or 128, got {group_size}")


def weight_quantize(x, algo="weight_only_int8", arch=None, group_size=-1):
    """Symmetric weight quantisation of a [K, N] (in, out) weight, reference layout and rounding
    (phi/kernels/impl/weight_quantize_kernel_impl.h): ``out`` int8 [N, K] (int8 / llm.int8) or int4 pairs
    [N/2, K] (channels 2j / 2j+1 in the low / high nibble, values + 8 as on ROCm); ``scale`` [N] (per channel)
    or [ceil(K / group_size), N], in x's dtype. ``arch`` selects CUDA SM-specific interleavings in the
    reference; this framework has one layout for gfx950, so any value is accepted and has no effect."""
    if algo not in _ALGOS:
        raise ValueError(f"algo must be one of {_ALGOS}, got {algo!r}")
    _check_group(group_size)
    w = T(x)
    if w.dim() != 2 or w.shape[0] % 64 or w.shape[1] % 16:
        raise ValueError(f"weight_quantize needs a 2-D [K, N] weight with K % 64 == 0 and N % 16 == 0, got "
                         f"{list(w.shape)}")
    if algo == "llm.int8" and group_size != -1:
        raise ValueError("llm.int8 quantises per channel (group_size=-1)")
    K, N = w.shape
    bound = 7.0 if algo == "weight_only_int4" else 127.0
    wf = w.float()
    if group_size == -1:
        scale = wf.abs().amax(0) / bound                          # [N]
        s_full = scale.clamp_min(1e-30)[None, :]
    else:
        g = -(-K // group_size)
        pad = g * group_size - K
        wp = torch.nn.functional.pad(wf, (0, 0, 0, pad)) if pad else wf
        scale = wp.abs().reshape(g, group_size, N).amax(1) / bound  # [G, N]
        s_full = scale.clamp_min(1e-30).repeat_interleave(group_size, 0)[:K]
    # round half away from zero, as the reference's C round()
    r = wf / s_full
    q = torch.where(r >= 0, torch.floor(r + 0.5), torch.ceil(r - 0.5)).clamp(-bound, bound).to(torch.int32)
    if algo == "weight_only_int4":
        u = (q + 8).to(torch.uint8)                               # [K, N], 1..15
        packed = (u[:, 0::2] & 0xF) | ((u[:, 1::2] & 0xF) << 4)   # [K, N/2]
        out = packed.view(torch.int8).t().contiguous()            # [N/2, K]
    else:
        out = q.to(torch.int8).t().contiguous()                   # [N, K]
    return _wrap(out), _wrap(scale.to(w.dtype) if w.is_floating_point() else scale)


def _unpack(q, algo):
    """int8 [N, K] view of a quantized weight (int4 pairs unpacked, offset removed)."""
    if algo == "weight_only_int4" or algo == "int4":
        u = q.view(torch.uint8)
        lo = (u & 0xF).to(torch.int16) - 8
        hi = ((u >> 4) & 0xF).to(torch.int16) - 8
        return torch.stack([lo, hi], 1).reshape(-1, q.shape[1])   # rows 2j (lo), 2j+1 (hi)
    return q.to(torch.int16)


def weight_dequantize(x, scale, algo="weight_only_int8", out_dtype="float16", group_size=-1):
    """Inverse of weight_quantize: [K, N] in ``out_dtype``."""
    from ...framework.dtype import to_torch_dtype
    if algo not in _ALGOS:
        raise ValueError(f"algo must be one of {_ALGOS}, got {algo!r}")
    _check_group(group_size)
    q = _unpack(T(x), algo).float()                               # [N, K]
    s = T(scale).float()
    if group_size == -1:
        w = q * s[:, None]
    else:
        w = q * s.repeat_interleave(group_size, 0)[:q.shape[1]].t()
    return _wrap(w.t().to(to_torch_dtype(out_dtype)).contiguous())


def _bits(weight_dtype):
    if weight_dtype not in ("int8", "int4"):
        raise ValueError(f"weight_dtype must be 'int8' or 'int4', got {weight_dtype!r}")
    return 8 if weight_dtype == "int8" else 4


def weight_only_linear(x, weight, bias=None, weight_scale=None, weight_dtype="int8", arch=None, group_size=-1):
    """y = x . dequant(weight) (+ bias). bf16 inputs on the device run the hand-written kernels
    (ops/quant.py: in-register dequant for M <= 64 rows, dequant + MFMA GEMM above); other dtypes / the CPU
    compute the same product from the dequantised weight."""
    bits = _bits(weight_dtype)
    _check_group(group_size)
    if weight_scale is None:
        raise ValueError("weight_only_linear needs weight_scale")
    from ... import ops as _ops
    xt, w, s = T(x), T(weight), T(weight_scale)
    b = T(bias)
    if xt.dtype == torch.bfloat16 and _ops.quant.available(xt):
        return _wrap(_ops.quant.wo_linear(xt, w.contiguous(), s, b, bits, group_size))
    wd = T(weight_dequantize(_wrap(w), _wrap(s), "weight_only_int4" if bits == 4 else "weight_only_int8",
                             "float32", group_size))
    y = (xt.float() @ wd).to(xt.dtype)
    if b is not None:
        y = y + b.to(y.dtype)
    return _wrap(y)


def _llm_split(xt, threshold):
    """LLM.int8 decomposition of the activations: outlier columns (any |x| > threshold) kept in floating point,
    the rest quantised per row to int8 (absmax / 127)."""
    xf = xt.float()
    outl = (xf.abs() > threshold).any(0) if threshold > 0 else torch.zeros(xf.shape[-1], dtype=torch.bool,
                                                                          device=xf.device)
    inl = xf.masked_fill(outl, 0.0)
    sx = inl.abs().amax(-1).clamp_min(1e-30) / 127.0
    xq = torch.round(inl / sx[:, None]).clamp(-127, 127)
    xo = xf * outl
    return xq, xo, sx, outl


def llm_int8_linear(x, weight, bias=None, weight_scale=None, threshold=6.0):
    """LLM.int8 (reference llm_int8_linear_kernel.cu): columns of x holding any |value| > ``threshold`` multiply
    the dequantised weight in floating point; the remaining columns are quantised per row to int8 and multiply
    the int8 weight; y = sw * (sx * xq.Wq + xo.Wq) (+ bias). ``weight`` from weight_quantize(algo="llm.int8")."""
    if weight_scale is None:
        raise ValueError("llm_int8_linear needs weight_scale")
    from ... import ops as _ops
    xt, w, s, b = T(x), T(weight), T(weight_scale), T(bias)
    K = xt.shape[-1]
    x2 = xt.reshape(-1, K)
    xq, xo, sx, _ = _llm_split(x2, float(threshold))
    if xt.dtype == torch.bfloat16 and _ops.quant.available(xt):
        # device kernels at every row count: the decode kernel / cached-image GEMM up to 64 rows, the MFMA GEMM
        # form of the decomposition above (ops/quant.py llm_int8_gemm)
        y = _ops.quant.wo_linear(xt, w.contiguous(), s, b, 8, -1,
                                 llm=(xq.to(torch.bfloat16).contiguous(), xo.to(torch.bfloat16).contiguous(),
                                      sx.float().contiguous()))
        return _wrap(y)
    wq = w.float()                                                 # [N, K]
    y = (sx[:, None] * (xq @ wq.t()) + xo @ wq.t()) * s.float()[None, :]
    if b is not None:
        y = y + b.float()
    return _wrap(y.to(xt.dtype).reshape(*xt.shape[:-1], -1))


def apply_per_channel_scale(x, scales):
    """x * scales over the last dimension (reference: nn/quant/quantized_linear.py apply_per_channel_scale, the
    SmoothQuant pre-scale)."""
    xt, st = T(x), T(scales)
    return _wrap(xt * st.to(xt.dtype))


from ..layer.layers import Layer as _Layer  # noqa: E402


class Stub(_Layer):
    """Placeholder in a model's forward that QAT / PTQ replace with the configured observer / quanter
    (reference nn/quant/stub.py); identity until then."""

    def __init__(self, observer=None):
        super().__init__()
        self._observer = observer

    def forward(self, input):
        return input


from . import quant_layers  # noqa: E402,F401
from .format import (ConvertibleQuantedLayer, LinearDequanter, LinearQuanter,  # noqa: E402,F401
                     LinearQuanterDequanter)
from .quant_layers import (FakeQuantAbsMax, FakeQuantChannelWiseAbsMax,  # noqa: E402,F401
                           FakeQuantMovingAverageAbsMax, MovingAverageAbsMaxScale, QuantizedConv2D,
                           QuantizedConv2DTranspose, QuantizedLinear)
