"""Convolution layers. Reference: python/paddle/nn/layer/conv.py.
With data_format NHWC the weight is kept channels-last-strided so MIOpen's NHWC solvers get it
without a per-step relayout."""
from __future__ import annotations

import math

import numpy as np
import torch

from .. import functional as F
from .. import initializer as I
from .layers import Layer


def _ntuple(v, n):
    return tuple(v) if isinstance(v, (list, tuple)) else (v,) * n


class _ConvNd(Layer):
    _nd = 2
    _transpose = False

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", weight_attr=None, bias_attr=None, data_format=None, output_padding=0):
        super().__init__()
        n = self._nd
        self._in_channels, self._out_channels = in_channels, out_channels
        self._kernel_size = _ntuple(kernel_size, n)
        self._stride, self._padding, self._dilation = stride, padding, dilation
        self._groups = groups
        self._padding_mode = padding_mode
        self._output_padding = output_padding
        self._data_format = data_format or {1: "NCL", 2: "NCHW", 3: "NCDHW"}[n]
        if self._transpose:
            shape = [in_channels, out_channels // groups, *self._kernel_size]
        else:
            shape = [out_channels, in_channels // groups, *self._kernel_size]
        fan_in = (in_channels // groups) * int(np.prod(self._kernel_size))
        std = math.sqrt(2.0 / fan_in)
        self.weight = self.create_parameter(shape, attr=weight_attr, default_initializer=I.Normal(0.0, std))
        if n == 2 and self._data_format == "NHWC":
            self.weight._t = self.weight._t.detach().contiguous(memory_format=torch.channels_last).requires_grad_(
                self.weight._t.requires_grad)
        self.bias = self.create_parameter([out_channels], attr=bias_attr, is_bias=True)

    def extra_repr(self):
        return (f"{self._in_channels}, {self._out_channels}, kernel_size={list(self._kernel_size)}, "
                f"stride={self._stride}, padding={self._padding}, data_format={self._data_format}")

    def _pad_input(self, x):
        if self._padding_mode != "zeros":
            p = self._padding
            pads = [p] * (2 * self._nd) if isinstance(p, int) else list(p)
            return F.pad(x, pads, mode=self._padding_mode, data_format=self._data_format), 0
        return x, self._padding


class Conv1D(_ConvNd):
    _nd = 1

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", weight_attr=None, bias_attr=None, data_format="NCL"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, padding_mode,
                         weight_attr, bias_attr, data_format)

    def forward(self, x):
        x, p = self._pad_input(x)
        return F.conv1d(x, self.weight, self.bias, self._stride, p, self._dilation, self._groups, self._data_format)


class Conv2D(_ConvNd):
    _nd = 2

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", weight_attr=None, bias_attr=None, data_format="NCHW"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, padding_mode,
                         weight_attr, bias_attr, data_format)

    def forward(self, x):
        x, p = self._pad_input(x)
        return F.conv2d(x, self.weight, self.bias, self._stride, p, self._dilation, self._groups, self._data_format)


class Conv3D(_ConvNd):
    _nd = 3

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", weight_attr=None, bias_attr=None, data_format="NCDHW"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, padding_mode,
                         weight_attr, bias_attr, data_format)

    def forward(self, x):
        x, p = self._pad_input(x)
        return F.conv3d(x, self.weight, self.bias, self._stride, p, self._dilation, self._groups, self._data_format)


class Conv1DTranspose(_ConvNd):
    _nd, _transpose = 1, True

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0, groups=1,
                 dilation=1, weight_attr=None, bias_attr=None, data_format="NCL"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, "zeros",
                         weight_attr, bias_attr, data_format, output_padding)

    def forward(self, x, output_size=None):
        return F.conv1d_transpose(x, self.weight, self.bias, self._stride, self._padding, self._output_padding,
                                  self._groups, self._dilation, output_size, self._data_format)


class Conv2DTranspose(_ConvNd):
    _nd, _transpose = 2, True

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0, dilation=1,
                 groups=1, weight_attr=None, bias_attr=None, data_format="NCHW"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, "zeros",
                         weight_attr, bias_attr, data_format, output_padding)

    def forward(self, x, output_size=None):
        return F.conv2d_transpose(x, self.weight, self.bias, self._stride, self._padding, self._output_padding,
                                  self._dilation, self._groups, output_size, self._data_format)


class Conv3DTranspose(_ConvNd):
    _nd, _transpose = 3, True

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0, dilation=1,
                 groups=1, weight_attr=None, bias_attr=None, data_format="NCDHW"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, "zeros",
                         weight_attr, bias_attr, data_format, output_padding)

    def forward(self, x, output_size=None):
        return F.conv3d_transpose(x, self.weight, self.bias, self._stride, self._padding, self._output_padding,
                                  self._groups, self._dilation, output_size, self._data_format)
