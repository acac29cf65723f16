"""paddle.sparse.nn: activations, batch norm, sparse (submanifold) convolutions and pooling on COO
tensors in NDHWC / NHWC layout. Reference: python/paddle/sparse/nn/{layer,functional}/."""
from __future__ import annotations

import math

import torch
import torch.nn.functional as TF

from .. import nn as _nn
from ..framework.tensor import Tensor, _wrap
from ..nn import initializer as I
from . import _core as K


def _vals(x, fn):
    return _wrap(K.map_values(x._t, fn))


class functional:  # namespace object: paddle.sparse.nn.functional.*
    @staticmethod
    def relu(x, name=None):
        return _vals(x, torch.relu)

    @staticmethod
    def relu6(x, name=None):
        return _vals(x, lambda v: v.clamp(0, 6))

    @staticmethod
    def leaky_relu(x, negative_slope=0.01, name=None):
        return _vals(x, lambda v: TF.leaky_relu(v, negative_slope))

    @staticmethod
    def softmax(x, axis=-1, name=None):
        out = K.softmax(x._t, axis)
        return _wrap(K.same_layout(out, x._t))

    @staticmethod
    def _conv(x, weight, bias, stride, padding, dilation, groups, subm, nd):
        """Rulebook convolution on the active sites (sparse/_core.py sparse_conv); submanifold convs keep
        the input's active set with a centred kernel."""
        def lst(v):
            return [int(v)] * nd if isinstance(v, int) else [int(a) for a in v]
        w = weight._t  # [*k, Cin / groups, Cout]
        dil = lst(dilation)
        if subm:
            st = [1] * nd
            pad = [(int(kk) - 1) // 2 * dil[i] for i, kk in enumerate(w.shape[:nd])]
        else:
            st, pad = lst(stride), lst(padding)
        out = K.sparse_conv(x._t, w, None if bias is None else bias._t, st, pad, dil, groups, subm)
        return _wrap(out)

    @staticmethod
    def conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NDHWC", name=None):
        return functional._conv(x, weight, bias, stride, padding, dilation, groups, False, 3)

    @staticmethod
    def subm_conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NDHWC", key=None,
                    name=None):
        return functional._conv(x, weight, bias, stride, padding, dilation, groups, True, 3)

    @staticmethod
    def conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NHWC", name=None):
        return functional._conv(x, weight, bias, stride, padding, dilation, groups, False, 2)

    @staticmethod
    def subm_conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NHWC", key=None,
                    name=None):
        return functional._conv(x, weight, bias, stride, padding, dilation, groups, True, 2)

    @staticmethod
    def max_pool3d(x, kernel_size, stride=None, padding=0, ceil_mode=False, data_format="NDHWC", name=None):
        """Max over the active sites of each window (rulebook), output sites = windows with any active input."""
        def lst(v):
            return [int(v)] * 3 if isinstance(v, int) else [int(a) for a in v]
        ks = lst(kernel_size)
        st = lst(stride if stride is not None else kernel_size)
        return _wrap(K.sparse_max_pool(x._t, ks, st, lst(padding)))

    @staticmethod
    def attention(query, key, value, sparse_mask, key_padding_mask=None, attn_mask=None, name=None):
        """Attention whose score matrix is evaluated only at sparse_mask's nonzeros (CSR [B*H, S, S]):
        SDDMM -> per-row softmax over the stored scores -> SpMM (no dense S x S matrix)."""
        return _wrap(K.sparse_attention(query._t, key._t, value._t, sparse_mask._t,
                                        None if key_padding_mask is None else key_padding_mask._t,
                                        None if attn_mask is None else attn_mask._t))


class ReLU(_nn.Layer):
    def forward(self, x):
        return functional.relu(x)


class ReLU6(_nn.Layer):
    def forward(self, x):
        return functional.relu6(x)


class LeakyReLU(_nn.Layer):
    def __init__(self, negative_slope=0.01, name=None):
        super().__init__()
        self.negative_slope = negative_slope

    def forward(self, x):
        return functional.leaky_relu(x, self.negative_slope)


class Softmax(_nn.Layer):
    def __init__(self, axis=-1, name=None):
        super().__init__()
        self.axis = axis

    def forward(self, x):
        return functional.softmax(x, self.axis)


class BatchNorm(_nn.Layer):
    """Batch norm over the values (channels last) of a COO tensor's active sites."""

    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format="NDHWC", use_global_stats=None, name=None):
        super().__init__()
        self.weight = self.create_parameter([num_features], attr=weight_attr, default_initializer=I.Constant(1.0))
        self.bias = self.create_parameter([num_features], attr=bias_attr, is_bias=True)
        self.register_buffer("_mean", _wrap(torch.zeros(num_features)))
        self.register_buffer("_variance", _wrap(torch.ones(num_features)))
        self.momentum, self.eps = momentum, epsilon

    def forward(self, x):
        i, v, shape, _ = K.coo_parts(K.to_coo(x._t))
        if self.training:
            mean, var = v.mean(0), v.var(0, unbiased=False)
            with torch.no_grad():
                self._mean._t.mul_(self.momentum).add_(mean.detach().to(self._mean._t.dtype), alpha=1 - self.momentum)
                self._variance._t.mul_(self.momentum).add_(var.detach().to(self._variance._t.dtype),
                                                           alpha=1 - self.momentum)
        else:
            mean, var = self._mean._t, self._variance._t
        y = (v - mean) / torch.sqrt(var + self.eps) * self.weight._t + self.bias._t
        return _wrap(K.make_coo(i, y, shape))


SyncBatchNorm = BatchNorm


class _ConvBase(_nn.Layer):
    _nd = 3
    _subm = False

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", key=None, weight_attr=None, bias_attr=None, data_format=None):
        super().__init__()
        k = [kernel_size] * self._nd if isinstance(kernel_size, int) else list(kernel_size)
        fan_in = in_channels * math.prod(k)
        self.weight = self.create_parameter(k + [in_channels // groups, out_channels], attr=weight_attr,
                                            default_initializer=I.Uniform(-1 / math.sqrt(fan_in), 1 / math.sqrt(fan_in)))
        self.bias = self.create_parameter([out_channels], attr=bias_attr, is_bias=True) if bias_attr is not False \
            else None
        self.stride, self.padding, self.dilation, self.groups = stride, padding, dilation, groups

    def forward(self, x):
        return functional._conv(x, self.weight, self.bias, self.stride, self.padding, self.dilation, self.groups,
                                self._subm, self._nd)


class Conv3D(_ConvBase):
    _nd, _subm = 3, False


class SubmConv3D(_ConvBase):
    _nd, _subm = 3, True


class Conv2D(_ConvBase):
    _nd, _subm = 2, False


class SubmConv2D(_ConvBase):
    _nd, _subm = 2, True


class MaxPool3D(_nn.Layer):
    def __init__(self, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, data_format="NDHWC",
                 name=None):
        super().__init__()
        self.k, self.s, self.p, self.c = kernel_size, stride, padding, ceil_mode

    def forward(self, x):
        return functional.max_pool3d(x, self.k, self.s, self.p, self.c)


functional.subm_conv2d_igemm = functional.subm_conv2d  # implicit-GEMM variants: same math, same entry
functional.subm_conv3d_igemm = functional.subm_conv3d

import sys as _sys  # noqa: E402
# `import paddle.sparse.nn.functional as F` works like in the reference (a namespace object as module)
_sys.modules[__name__ + ".functional"] = functional
__path__ = []  # submodules above are importable by dotted name
