"""Activation functions. Reference: python/paddle/nn/functional/activation.py.
softmax / gelu / silu / swiglu route to HIP kernels (``paddlepaddle_amd.ops``) on MI355X."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ...framework.tensor import Tensor, _wrap
from ...tensor._helpers import T, dtype_arg
from ... import ops as _ops


def relu(x, name=None):
    return _wrap(F.relu(T(x)))


def relu_(x, name=None):
    F.relu_(x._t)
    return x


def relu6(x, name=None):
    return _wrap(F.relu6(T(x)))


def elu(x, alpha=1.0, name=None):
    return _wrap(F.elu(T(x), alpha))


def elu_(x, alpha=1.0, name=None):
    F.elu_(x._t, alpha)
    return x


def selu(x, scale=1.0507009873554804934193349852946, alpha=1.6732632423543772848170429916717, name=None):
    t = T(x)
    return _wrap(scale * torch.where(t > 0, t, alpha * (torch.exp(t) - 1)))


def celu(x, alpha=1.0, name=None):
    return _wrap(F.celu(T(x), alpha))


def gelu(x, approximate=False, name=None):
    return _wrap(_ops.gelu(T(x), approximate))


def silu(x, name=None):
    return _wrap(_ops.silu(T(x)))


swish = silu


def sigmoid(x, name=None):
    return _wrap(torch.sigmoid(T(x)))


def hardsigmoid(x, slope=0.1666667, offset=0.5, name=None):
    t = T(x)
    return _wrap(torch.clamp(t * slope + offset, 0.0, 1.0))


def hardswish(x, name=None):
    return _wrap(F.hardswish(T(x)))


def hardtanh(x, min=-1.0, max=1.0, name=None):  # noqa: A002
    return _wrap(F.hardtanh(T(x), min, max))


def hardtanh_(x, min=-1.0, max=1.0, name=None):  # noqa: A002
    F.hardtanh_(x._t, min, max)
    return x


def hardshrink(x, threshold=0.5, name=None):
    return _wrap(F.hardshrink(T(x), threshold))


def softshrink(x, threshold=0.5, name=None):
    return _wrap(F.softshrink(T(x), threshold))


def tanhshrink(x, name=None):
    return _wrap(F.tanhshrink(T(x)))


def leaky_relu(x, negative_slope=0.01, name=None):
    return _wrap(F.leaky_relu(T(x), negative_slope))


def leaky_relu_(x, negative_slope=0.01, name=None):
    F.leaky_relu_(x._t, negative_slope)
    return x


def log_sigmoid(x, name=None):
    return _wrap(F.logsigmoid(T(x)))


def logsigmoid(x, name=None):
    return log_sigmoid(x)


def maxout(x, groups, axis=1, name=None):
    t = T(x)
    shape = list(t.shape)
    c = shape[axis]
    shape[axis:axis + 1] = [c // groups, groups]
    return _wrap(t.reshape(shape).amax(axis + 1))


def mish(x, name=None):
    return _wrap(F.mish(T(x)))


def prelu(x, weight, data_format="NCHW", name=None):
    t, w = T(x), T(weight)
    if data_format == "NHWC" and w.numel() > 1:
        return _wrap(torch.where(t > 0, t, t * w))
    if w.numel() > 1 and t.dim() > 1:
        shape = [1] * t.dim()
        shape[1] = w.numel()
        return _wrap(torch.where(t > 0, t, t * w.reshape(shape)))
    return _wrap(torch.where(t > 0, t, t * w.reshape(-1)[0]))


def rrelu(x, lower=1.0 / 8.0, upper=1.0 / 3.0, training=True, name=None):
    return _wrap(F.rrelu(T(x), lower, upper, training))


def softmax(x, axis=-1, dtype=None, name=None):
    t = T(x)
    if dtype is not None:
        t = t.to(dtype_arg(dtype))
    return _wrap(_ops.softmax(t, axis))


def softmax_(x, axis=-1, dtype=None, name=None):
    x._t = softmax(x, axis, dtype)._t
    return x


def log_softmax(x, axis=-1, dtype=None, name=None):
    t = T(x)
    if dtype is not None:
        t = t.to(dtype_arg(dtype))
    return _wrap(F.log_softmax(t, axis))


def softplus(x, beta=1, threshold=20, name=None):
    return _wrap(F.softplus(T(x), beta, threshold))


def softsign(x, name=None):
    return _wrap(F.softsign(T(x)))


def tanh(x, name=None):
    return _wrap(torch.tanh(T(x)))


def tanh_(x, name=None):
    x._t.tanh_()
    return x


def thresholded_relu(x, threshold=1.0, value=0.0, name=None):
    t = T(x)
    return _wrap(torch.where(t > threshold, t, torch.full_like(t, value)))


def thresholded_relu_(x, threshold=1.0, value=0.0, name=None):
    x._t.copy_(thresholded_relu(x, threshold, value)._t)
    return x


def glu(x, axis=-1, name=None):
    return _wrap(F.glu(T(x), axis))


def gumbel_softmax(x, temperature=1.0, hard=False, axis=-1, name=None):
    return _wrap(F.gumbel_softmax(T(x), tau=temperature, hard=hard, dim=axis))


def swiglu(x, y=None, name=None):
    """Reference: python/paddle/incubate/nn/functional/swiglu.py. HIP kernel on MI355X."""
    return _wrap(_ops.swiglu(T(x), None if y is None else T(y)))
