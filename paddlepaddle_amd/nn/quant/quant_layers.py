"""Imperative QAT layers (fake quantisation in the forward, straight-through gradients).

Reference: python/paddle/nn/quant/quant_layers.py (FakeQuantAbsMax :69, FakeQuantMovingAverageAbsMax :172,
FakeQuantChannelWiseAbsMax :310, MovingAverageAbsMaxScale :424, QuantizedConv2D :544, QuantizedConv2DTranspose
:646, QuantizedLinear :769, QuantizedColumn/RowParallelLinear :850/:953, QuantizedMatmul :1060,
MAOutputScaleLayer :1126, FakeQuantMAOutputScaleLayer :1160).

Quantisation is symmetric: q = clip(round(x / s * Q), -Q, Q) * s / Q with Q = 2^(bits-1) - 1; the scale s is the
tensor's abs-max, a per-channel abs-max, or an abs-max moving average (state/accum buffers, updated in training,
frozen in eval). The rounding is a straight-through estimator (paddlepaddle_amd.quantization.fake_quant).
"""
from __future__ import annotations

import torch

from ...framework.tensor import Tensor, _wrap
from ...tensor._helpers import T
from ..layer.layers import Layer
from .. import functional as F


def _qmax(bits):
    return float(2 ** (bits - 1) - 1)


class _STE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scale, qmax):
        s = scale.clamp_min(1e-12)
        return torch.round(x / s * qmax).clamp(-qmax, qmax) * s / qmax

    @staticmethod
    def backward(ctx, g):
        return g, None, None


def _fq(x, scale, bits):
    return _STE.apply(x, scale.to(x.dtype), _qmax(bits))


class FakeQuantAbsMax(Layer):
    def __init__(self, name=None, quant_bits=8, dtype="float32", quant_on_weight=False, reduce_type=None):
        super().__init__()
        self._quant_bits = quant_bits
        self._reduce_type = reduce_type
        self.register_buffer("_scale", _wrap(torch.zeros(1)))

    def forward(self, input):
        x = T(input)
        s = x.detach().abs().amax().reshape(1).float()
        if self._reduce_type == "max" and torch.distributed.is_initialized():
            torch.distributed.all_reduce(s, op=torch.distributed.ReduceOp.MAX)
        self._scale._t.copy_(s.to(self._scale._t.device))
        return _wrap(_fq(x, s.to(x.device), self._quant_bits))


class FakeQuantMovingAverageAbsMax(Layer):
    """scale = accum / state with accum = rate * accum + max|x|, state = rate * state + 1 (training)."""

    def __init__(self, name=None, moving_rate=0.9, quant_bits=8, dtype="float32", reduce_type=None):
        super().__init__()
        self._moving_rate = moving_rate
        self._quant_bits = quant_bits
        self._reduce_type = reduce_type
        self.register_buffer("_scale", _wrap(torch.ones(1)))
        self.register_buffer("_state", _wrap(torch.ones(1)))
        self.register_buffer("_accum", _wrap(torch.ones(1)))

    def forward(self, input):
        x = T(input)
        if self.training:
            cur = x.detach().abs().amax().reshape(1).float().to(self._accum._t.device)
            if self._reduce_type == "max" and torch.distributed.is_initialized():
                torch.distributed.all_reduce(cur, op=torch.distributed.ReduceOp.MAX)
            r = self._moving_rate
            self._state._t.mul_(r).add_(1.0)
            self._accum._t.mul_(r).add_(cur)
            self._scale._t.copy_(self._accum._t / self._state._t)
        return _wrap(_fq(x, self._scale._t.to(x.device), self._quant_bits))


class FakeQuantChannelWiseAbsMax(Layer):
    def __init__(self, name=None, channel_num=None, quant_bits=8, quant_axis=0, dtype="float32",
                 quant_on_weight=False, reduce_type=None):
        super().__init__()
        self._quant_bits = quant_bits
        self._quant_axis = quant_axis
        self.register_buffer("_scale", _wrap(torch.zeros(channel_num or 1)))

    def forward(self, input):
        x = T(input)
        ax = self._quant_axis % x.dim()
        red = [d for d in range(x.dim()) if d != ax]
        s = x.detach().abs().amax(dim=red).float()
        if self._scale._t.shape != s.shape:
            self._scale._t = torch.zeros_like(s).to(self._scale._t.device)
        self._scale._t.copy_(s.to(self._scale._t.device))
        shape = [1] * x.dim()
        shape[ax] = -1
        return _wrap(_fq(x, s.reshape(shape).to(x.device), self._quant_bits))


class MovingAverageAbsMaxScale(Layer):
    """Tracks the moving-average abs-max of its input (an output-scale observer); returns the input."""

    def __init__(self, name=None, moving_rate=0.9, dtype="float32", reduce_type=None):
        super().__init__()
        self._moving_rate = moving_rate
        self._reduce_type = reduce_type
        self.register_buffer("_scale", _wrap(torch.zeros(1)))
        self.register_buffer("_state", _wrap(torch.zeros(1)))
        self.register_buffer("_accum", _wrap(torch.zeros(1)))

    def forward(self, input):
        x = T(input)
        if self.training:
            cur = x.detach().abs().amax().reshape(1).float().to(self._accum._t.device)
            r = self._moving_rate
            self._state._t.mul_(r).add_(1.0)
            self._accum._t.mul_(r).add_(cur)
            self._scale._t.copy_(self._accum._t / self._state._t)
        return input


def _weight_quanter(kind, bits, channels, axis):
    if kind == "channel_wise_abs_max":
        return FakeQuantChannelWiseAbsMax(channel_num=channels, quant_bits=bits, quant_axis=axis,
                                          quant_on_weight=True)
    if kind == "abs_max":
        return FakeQuantAbsMax(quant_bits=bits, quant_on_weight=True)
    raise ValueError(f"unsupported weight_quantize_type {kind!r}")


def _act_quanter(kind, bits, moving_rate):
    if kind == "moving_average_abs_max":
        return FakeQuantMovingAverageAbsMax(moving_rate=moving_rate, quant_bits=bits)
    if kind == "abs_max":
        return FakeQuantAbsMax(quant_bits=bits)
    raise ValueError(f"unsupported activation_quantize_type {kind!r}")


class _QuantizedBase(Layer):
    """Shared plumbing: optional pre-layers and user quant layers override the built-in fake quanters."""

    _w_axis = 0

    def __init__(self, layer, weight_bits=8, activation_bits=8, moving_rate=0.9, weight_quantize_type="abs_max",
                 activation_quantize_type="abs_max", weight_pre_layer=None, act_pre_layer=None,
                 weight_quant_layer=None, act_quant_layer=None):
        super().__init__()
        self._layer = layer
        self.weight = layer.weight
        self.bias = getattr(layer, "bias", None)
        ch = self.weight.shape[self._w_axis]
        self._fake_quant_weight = weight_quant_layer or _weight_quanter(weight_quantize_type, weight_bits, ch,
                                                                        self._w_axis)
        self._fake_quant_input = act_quant_layer or _act_quanter(activation_quantize_type, activation_bits,
                                                                 moving_rate)
        self._weight_preprocess = weight_pre_layer
        self._act_preprocess = act_pre_layer

    def _quant_io(self, input):
        x = input if isinstance(input, Tensor) else _wrap(input)
        if self._act_preprocess is not None:
            x = self._act_preprocess(x)
        x = self._fake_quant_input(x)
        w = self.weight
        if self._weight_preprocess is not None:
            w = self._weight_preprocess(w)
        return x, self._fake_quant_weight(w)


class QuantizedConv2D(_QuantizedBase):
    def forward(self, input):
        x, w = self._quant_io(input)
        L = self._layer
        return F.conv2d(x, w, self.bias, L._stride, L._padding, L._dilation, L._groups, L._data_format)


class QuantizedConv2DTranspose(_QuantizedBase):
    _w_axis = 1  # weight [in, out / groups, kh, kw]: per output channel

    def forward(self, input, output_size=None):
        x, w = self._quant_io(input)
        L = self._layer
        return F.conv2d_transpose(x, w, self.bias, L._stride, L._padding, L._output_padding, L._groups,
                                  L._dilation, output_size, L._data_format)


class QuantizedLinear(_QuantizedBase):
    _w_axis = 1  # paddle weight [in, out]

    def forward(self, input):
        x, w = self._quant_io(input)
        return F.linear(x, w, self.bias)


class QuantizedColumnParallelLinear(_QuantizedBase):
    _w_axis = 1

    def forward(self, input):
        from ...parallel import tensor_parallel as tp
        x, w = self._quant_io(input)
        L = self._layer
        t = tp.c_identity(x._t, L.group)
        y = F.linear(_wrap(t), w, self.bias)
        return _wrap(tp.c_concat(y._t, L.group)) if L.gather_output else y


class QuantizedRowParallelLinear(_QuantizedBase):
    _w_axis = 1

    def forward(self, input):
        from ...parallel import tensor_parallel as tp
        L = self._layer
        t = input._t if isinstance(input, Tensor) else input
        if not L.input_is_parallel:
            t = tp.c_split(t, L.group)
        x, w = self._quant_io(_wrap(t))
        y = F.linear(x, w, None)
        y = _wrap(tp.mp_allreduce(y._t, L.group))
        return y + self.bias if self.bias is not None else y


class QuantizedMatmul(Layer):
    def __init__(self, layer=None, weight_bits=8, activation_bits=8, moving_rate=0.9,
                 activation_quantize_type="abs_max", weight_pre_layer=None, act_pre_layer=None,
                 weight_quant_layer=None, act_quant_layer=None):
        super().__init__()
        self._fake_quant_x = act_quant_layer or _act_quanter(activation_quantize_type, activation_bits, moving_rate)
        self._fake_quant_y = act_quant_layer or _act_quanter(activation_quantize_type, activation_bits, moving_rate)
        self._act_preprocess_x = act_pre_layer
        self._act_preprocess_y = act_pre_layer

    def forward(self, x, y, transpose_x=False, transpose_y=False, name=None):
        from ...tensor.math import matmul
        if self._act_preprocess_x is not None:
            x = self._act_preprocess_x(x)
        if self._act_preprocess_y is not None:
            y = self._act_preprocess_y(y)
        return matmul(self._fake_quant_x(x), self._fake_quant_y(y), transpose_x, transpose_y)


class MAOutputScaleLayer(Layer):
    """Runs ``layer`` and tracks the moving-average abs-max of its (first) output."""

    def __init__(self, layer=None, moving_rate=0.9, name=None, dtype="float32", reduce_type=None):
        super().__init__()
        self._layer = layer
        self._ma_output_scale = MovingAverageAbsMaxScale(moving_rate=moving_rate, reduce_type=reduce_type)

    def forward(self, *inputs, **kwargs):
        out = self._layer(*inputs, **kwargs)
        if isinstance(out, (list, tuple)):
            return out
        return self._ma_output_scale(out)


class FakeQuantMAOutputScaleLayer(Layer):
    """Runs ``layer`` and fake-quantises its output with a moving-average abs-max scale."""

    def __init__(self, layer, weight_bits=8, activation_bits=8, moving_rate=0.9, name=None, reduce_type=None,
                 *args, **kwargs):
        super().__init__()
        self._layer = layer
        self._fake_quant_output = FakeQuantMovingAverageAbsMax(moving_rate=moving_rate, quant_bits=activation_bits,
                                                               reduce_type=reduce_type)

    def forward(self, *inputs, **kwargs):
        out = self._layer(*inputs, **kwargs)
        if isinstance(out, (list, tuple)):
            return out
        return self._fake_quant_output(out)
