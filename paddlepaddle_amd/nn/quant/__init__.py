"""paddle.nn.quant — weight-only int8/fp8 helpers. Reference: python/paddle/nn/quant/."""
from __future__ import annotations

import torch

from ...framework.tensor import _wrap
from ...tensor._helpers import T


def weight_quantize(x, algo="weight_only_int8", arch=None, group_size=-1):
    """Per-output-channel symmetric quantisation of a [in, out] weight."""
    w = T(x).float()
    if algo in ("weight_only_int8", "llm.int8"):
        scale = w.abs().amax(0).clamp_min(1e-8) / 127.0
        q = torch.round(w / scale).clamp(-127, 127).to(torch.int8)
        return _wrap(q.t().contiguous()), _wrap(scale)
    if algo == "weight_only_int4":
        scale = w.abs().amax(0).clamp_min(1e-8) / 7.0
        q = torch.round(w / scale).clamp(-7, 7).to(torch.int8)
        return _wrap(q.t().contiguous()), _wrap(scale)
    raise ValueError(algo)


def weight_dequantize(x, scale, algo="weight_only_int8", out_dtype="float16", group_size=-1):
    from ...framework.dtype import to_torch_dtype
    q = T(x).float().t()
    return _wrap((q * T(scale).float()).to(to_torch_dtype(out_dtype)))


def weight_only_linear(x, weight, bias=None, weight_scale=None, weight_dtype="int8", arch=None, group_size=-1):
    xt = T(x)
    w = (T(weight).float().t() * T(weight_scale).float()).to(xt.dtype)
    y = xt @ w
    if bias is not None:
        y = y + T(bias)
    return _wrap(y)


def llm_int8_linear(x, weight, bias=None, weight_scale=None, threshold=6.0):
    return weight_only_linear(x, weight, bias, weight_scale)


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
