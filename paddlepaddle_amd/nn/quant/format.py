"""Deployment form of quantised layers: explicit quantize / dequantize operators and the base class that
converts a QAT layer's quanters into them.

Reference: python/paddle/nn/quant/format.py (LinearQuanterDequanter :65, LinearQuanter :88,
LinearDequanter :250, ConvertibleQuantedLayer :408). Symmetric linear quantisation with an optional zero point:
q = clip(round(x / s * Q) + zp, -Q-1, Q) with Q = 2^(bits-1) - 1 (per tensor, or per channel along quant_axis);
dequant: (q - zp) * s / Q.
"""
from __future__ import annotations

import abc

import torch

from ...framework.tensor import _wrap
from ...tensor._helpers import T
from ..layer.layers import Layer


def _bnt(bits):
    return float(2 ** (bits - 1) - 1)


def _bcast(s, x, axis):
    if s.numel() == 1:
        return s.reshape([])
    shape = [1] * x.dim()
    shape[axis % x.dim()] = -1
    return s.reshape(shape)


class LinearQuanter(Layer):
    def __init__(self, scales, zero_point=None, quant_axis=None, bit_length=8, group_size=128):
        super().__init__()
        s = T(scales) if not isinstance(scales, (int, float, list, tuple)) else torch.tensor(scales)
        self.register_buffer("_scales", _wrap(torch.as_tensor(s, dtype=torch.float32).reshape(-1)))
        zp = torch.zeros_like(self._scales._t) if zero_point is None else \
            torch.as_tensor(T(zero_point) if not isinstance(zero_point, (int, float, list)) else zero_point,
                            dtype=torch.float32).reshape(-1)
        self.register_buffer("_zero_point", _wrap(zp))
        self._quant_axis = -1 if quant_axis is None else quant_axis
        self._bit_length = bit_length
        self._group_size = group_size

    def forward(self, input):
        x = T(input)
        q = _bnt(self._bit_length)
        s = _bcast(self._scales._t.to(x.device), x, self._quant_axis)
        zp = _bcast(self._zero_point._t.to(x.device), x, self._quant_axis)
        out = torch.round(x.float() / s.clamp_min(1e-12) * q) + zp
        return _wrap(out.clamp(-q - 1, q).to(x.dtype))

    @staticmethod
    def from_quanter(quanter):
        return LinearQuanter(quanter.scales(), zero_point=quanter.zero_points(), quant_axis=quanter.quant_axis(),
                             bit_length=quanter.bit_length())


class LinearDequanter(Layer):
    def __init__(self, scales, zero_point=None, quant_axis=None, bit_length=8, group_size=128):
        super().__init__()
        s = T(scales) if not isinstance(scales, (int, float, list, tuple)) else torch.tensor(scales)
        self.register_buffer("_scales", _wrap(torch.as_tensor(s, dtype=torch.float32).reshape(-1)))
        zp = torch.zeros_like(self._scales._t) if zero_point is None else \
            torch.as_tensor(T(zero_point) if not isinstance(zero_point, (int, float, list)) else zero_point,
                            dtype=torch.float32).reshape(-1)
        self.register_buffer("_zero_point", _wrap(zp))
        self._quant_axis = -1 if quant_axis is None else quant_axis
        self._bit_length = bit_length
        self._group_size = group_size

    def forward(self, input):
        x = T(input)
        q = _bnt(self._bit_length)
        s = _bcast(self._scales._t.to(x.device), x, self._quant_axis)
        zp = _bcast(self._zero_point._t.to(x.device), x, self._quant_axis)
        return _wrap(((x.float() - zp) * s / q).to(x.dtype if x.is_floating_point() else torch.float32))

    @staticmethod
    def from_quanter(quanter):
        return LinearDequanter(quanter.scales(), zero_point=quanter.zero_points(), quant_axis=quanter.quant_axis(),
                               bit_length=quanter.bit_length())


class LinearQuanterDequanter(Layer):
    def __init__(self, quanter, dequanter):
        super().__init__()
        self._quanter = quanter
        self._dequanter = dequanter

    def forward(self, input):
        out = input
        if self._quanter is not None:
            out = self._quanter(out)
        if self._dequanter is not None:
            out = self._dequanter(out)
        return out

    @staticmethod
    def from_quanter(quanter):
        assert quanter is not None
        return LinearQuanterDequanter(LinearQuanter.from_quanter(quanter), LinearDequanter.from_quanter(quanter))


class ConvertibleQuantedLayer(Layer, metaclass=abc.ABCMeta):
    """A QAT layer that knows which weights its quanters cover; ``_convert`` turns every quanter / observer
    into quantize-dequantize operators holding the learned scales (weights are fake-quantised once, in place)."""

    def __init__(self):
        super().__init__()
        self.converted = False

    @abc.abstractmethod
    def weights_to_quanters(self):
        """[(weight attribute name, quanter attribute name), ...]"""

    @abc.abstractmethod
    def activation_quanters(self):
        """[quanter attribute name, ...]"""

    def _convert_quanter_to_qdq(self, quanter_name):
        if not hasattr(self, quanter_name):
            return None
        quanter = getattr(self, quanter_name)
        if quanter is None:
            return None
        qdq = LinearQuanterDequanter.from_quanter(quanter)
        setattr(self, quanter_name, qdq)
        self._sub_layers[quanter_name] = qdq
        return qdq

    def _quant_weights(self, weight_name, quanter):
        w = getattr(self, weight_name)
        with torch.no_grad():
            w._t.copy_(T(quanter(w)).to(w._t.dtype))

    def _convert(self, remain_weight=False):
        for weight_name, quanter_name in self.weights_to_quanters():
            qdq = self._convert_quanter_to_qdq(quanter_name)
            if qdq is not None and not remain_weight:
                self._quant_weights(weight_name, qdq._quanter)
                qdq._quanter = None  # the weight now holds the quantised values
        for quanter_name in self.activation_quanters():
            self._convert_quanter_to_qdq(quanter_name)
        self.converted = True
