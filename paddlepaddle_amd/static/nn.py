"""paddle.static.nn: layer-building functions for static programs.
Reference: python/paddle/static/nn/common.py (fc:33, conv2d, batch_norm, layer_norm, embedding...).
Each call creates the parameters (eagerly initialised) and records the compute into the program."""
from __future__ import annotations

import numpy as np

from .. import nn as _nn
from ..nn import functional as F

_ACT = {None: lambda x: x, "relu": F.relu, "sigmoid": F.sigmoid, "tanh": F.tanh, "gelu": F.gelu,
        "softmax": F.softmax, "silu": F.silu, "leaky_relu": F.leaky_relu}


def _act(x, a):
    return _ACT[a](x)


def fc(x, size, num_flatten_dims=1, weight_attr=None, bias_attr=None, activation=None, name=None):
    xs = x if isinstance(x, (list, tuple)) else [x]
    out = None
    for i, xi in enumerate(xs):
        in_f = int(np.prod(xi.shape[num_flatten_dims:]))
        lin = _nn.Linear(in_f, size, weight_attr=weight_attr, bias_attr=bias_attr if i == 0 else False)
        # leading dims from the data (shape-generic: a None batch dim stays dynamic), the rest flattened
        lead = list(xi.shape[1:num_flatten_dims])
        h = xi.reshape([-1] + lead + [in_f]) if xi.ndim != num_flatten_dims + 1 else xi
        y = lin(h)
        out = y if out is None else out + y
    return _act(out, activation)


def conv2d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None, param_attr=None,
           bias_attr=None, use_cudnn=True, act=None, name=None, data_format="NCHW"):
    cin = input.shape[1] if data_format == "NCHW" else input.shape[-1]
    conv = _nn.Conv2D(cin, num_filters, filter_size, stride, padding, dilation, groups or 1,
                      weight_attr=param_attr, bias_attr=bias_attr, data_format=data_format)
    return _act(conv(input), act)


def conv2d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0, stride=1, dilation=1,
                     groups=None, param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None,
                     data_format="NCHW"):
    cin = input.shape[1] if data_format == "NCHW" else input.shape[-1]
    conv = _nn.Conv2DTranspose(cin, num_filters, filter_size, stride, padding, dilation=dilation,
                               groups=groups or 1, weight_attr=param_attr, bias_attr=bias_attr,
                               data_format=data_format)
    return _act(conv(input), act)


def batch_norm(input, act=None, is_test=False, momentum=0.9, epsilon=1e-05, param_attr=None, bias_attr=None,
               data_layout="NCHW", in_place=False, name=None, moving_mean_name=None, moving_variance_name=None,
               do_model_average_for_mean_and_var=True, use_global_stats=False):
    c = input.shape[1] if data_layout == "NCHW" else input.shape[-1]
    bn = _nn.BatchNorm2D(c, momentum=momentum, epsilon=epsilon, weight_attr=param_attr, bias_attr=bias_attr,
                         data_format=data_layout if input.ndim == 4 else "NCL")
    if is_test:
        bn.eval()
    return _act(bn(input), act)


def layer_norm(input, scale=True, shift=True, begin_norm_axis=1, epsilon=1e-05, param_attr=None, bias_attr=None,
               act=None, name=None):
    shape = input.shape[begin_norm_axis:]
    ln = _nn.LayerNorm(shape, epsilon=epsilon, weight_attr=param_attr if scale else False,
                       bias_attr=bias_attr if shift else False)
    return _act(ln(input), act)


def group_norm(input, groups, epsilon=1e-05, param_attr=None, bias_attr=None, act=None, data_layout="NCHW",
               name=None):
    gn = _nn.GroupNorm(groups, input.shape[1], epsilon=epsilon, weight_attr=param_attr, bias_attr=bias_attr)
    return _act(gn(input), act)


def instance_norm(input, epsilon=1e-05, param_attr=None, bias_attr=None, name=None):
    return _nn.InstanceNorm2D(input.shape[1], epsilon=epsilon, weight_attr=param_attr, bias_attr=bias_attr)(input)


def embedding(input, size, is_sparse=False, is_distributed=False, padding_idx=None, param_attr=None,
              dtype="float32"):
    emb = _nn.Embedding(size[0], size[1], padding_idx=padding_idx, weight_attr=param_attr)
    return emb(input)


def prelu(x, mode, param_attr=None, data_format="NCHW", name=None):
    n = 1 if mode == "all" else (x.shape[1] if mode == "channel" else int(np.prod(x.shape[1:])))
    return _nn.PReLU(n, weight_attr=param_attr, data_format=data_format)(x)


def bilinear_tensor_product(x, y, size, act=None, name=None, param_attr=None, bias_attr=None):
    return _act(_nn.Bilinear(x.shape[-1], y.shape[-1], size, weight_attr=param_attr, bias_attr=bias_attr)(x, y), act)


def data_norm(input, *a, **k):
    return F.layer_norm(input, input.shape[1:])


def sequence_softmax(input, use_cudnn=False, name=None):
    return F.softmax(input, axis=-1)
from .control_flow import *  # noqa: F401,F403,E402
