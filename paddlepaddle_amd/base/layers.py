"""paddle.base.layers: the legacy fluid.layers names older static-graph code still calls (reference: the
fluid.layers wrappers that python/paddle/base/ kept re-exporting); each maps onto the modern API."""
from __future__ import annotations

from .. import tensor as _T
from ..nn import functional as _F
from ..static import nn as _snn


def _axis_bcast(x, y, axis):
    """fluid broadcast rule: y's dims align with x's starting at ``axis`` (-1: trailing)."""
    if axis is None or axis == -1 or y.ndim == x.ndim:
        return y
    return y.reshape([1] * axis + list(y.shape) + [1] * (x.ndim - axis - y.ndim))


def elementwise_add(x, y, axis=-1, act=None, name=None):
    return _act(x + _axis_bcast(x, y, axis), act)


def elementwise_sub(x, y, axis=-1, act=None, name=None):
    return _act(x - _axis_bcast(x, y, axis), act)


def elementwise_mul(x, y, axis=-1, act=None, name=None):
    return _act(x * _axis_bcast(x, y, axis), act)


def elementwise_div(x, y, axis=-1, act=None, name=None):
    return _act(x / _axis_bcast(x, y, axis), act)


def _act(x, act):
    return x if act is None else getattr(_F, act)(x)


def fc(input, size, num_flatten_dims=1, param_attr=None, bias_attr=None, act=None, name=None):
    return _snn.fc(input, size, num_flatten_dims, param_attr, bias_attr, act, name)


def mean(x, name=None):
    return _T.mean(x)


def relu(x, name=None):
    return _F.relu(x)


def matmul(x, y, transpose_x=False, transpose_y=False, alpha=1.0, name=None):
    out = _T.matmul(x, y, transpose_x, transpose_y)
    return out if alpha == 1.0 else out * alpha


def data(name, shape, append_batch_size=True, dtype="float32", lod_level=0, type=None, stop_gradient=True):
    from ..static import data as _data
    return _data(name, shape, dtype, lod_level, append_batch_size=append_batch_size)
