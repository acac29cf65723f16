"""Normalisation. Reference: python/paddle/nn/functional/norm.py, phi layer_norm/rms_norm/batch_norm kernels.
layer_norm / rms_norm run on the HIP kernels in csrc/kernels/norm.hip."""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from ...framework import layout_autotune as _lat
from ...framework.tensor import Tensor, _wrap
from ...tensor._helpers import T
from ... import ops as _ops


def layer_norm(x, normalized_shape, weight=None, bias=None, epsilon=1e-05, name=None):
    t = T(x)
    if isinstance(normalized_shape, int):
        normalized_shape = [normalized_shape]
    ns = list(normalized_shape)
    w, b = T(weight), T(bias)
    if len(ns) == 1:
        return _wrap(_ops.layer_norm(t, w, b, epsilon))
    n = int(np.prod(ns))
    y = _ops.layer_norm(t.reshape(*t.shape[: t.dim() - len(ns)], n), None if w is None else w.reshape(n),
                        None if b is None else b.reshape(n), epsilon)
    return _wrap(y.reshape(t.shape))


def rms_norm(x, normalized_shape=None, weight=None, epsilon=1e-6, name=None):
    t = T(x)
    return _wrap(_ops.rms_norm(t, T(weight), epsilon))


def batch_norm(x, running_mean, running_var, weight=None, bias=None, training=False, momentum=0.9,
               epsilon=1e-05, data_format="NCHW", use_global_stats=None, name=None):
    return fused_bn_act(x, running_mean, running_var, weight, bias, training, momentum, epsilon, data_format,
                        use_global_stats)


def fused_bn_act(x, running_mean, running_var, weight=None, bias=None, training=False, momentum=0.9,
                 epsilon=1e-05, data_format="NCHW", use_global_stats=None, act=None, residual=None, _grad_sink=None):
    """act(batch_norm(x) [+ residual]) — batch_norm with the fused_bn_add_activation epilogue
    (reference: python/paddle/incubate/layers/nn.py:1092). Channels-last bf16 input runs the HIP
    kernels of csrc/kernels/bn.hip (ops.batch_norm_act_nhwc); other layouts / dtypes run torch.
    Running statistics follow the reference: biased batch variance, factor 1 - momentum."""
    t = T(x)
    cl = data_format in ("NHWC", "NLC", "NDHWC")
    if data_format == "NCHW" and _lat.applies(t):
        # layout autotune: the channels-last HIP kernels on the NHWC view (framework/layout_autotune.py)
        r = T(residual)
        y = _ops.batch_norm_act_nhwc(_lat.to_nhwc_view(t), T(weight), T(bias), T(running_mean), T(running_var),
                                     training and not use_global_stats, momentum, epsilon, act,
                                     None if r is None else _lat.to_nhwc_view(r), _grad_sink)
        return _wrap(_lat.to_nchw_view(y))
    use_batch = training and not use_global_stats
    rm, rv = T(running_mean), T(running_var)
    w, b = T(weight), T(bias)
    r = T(residual)
    if cl and t.dim() >= 2:
        return _wrap(_ops.batch_norm_act_nhwc(t, w, b, rm, rv, use_batch, momentum, epsilon, act, r, _grad_sink))
    nd = t.dim()
    if t.dtype in (torch.float16, torch.bfloat16) and w is not None and w.dtype != torch.float32:
        w, b = w.float(), b.float() if b is not None else None
    if use_batch and rm is not None:
        red = [0] + list(range(2, nd))
        with torch.no_grad():
            var, mean = torch.var_mean(t.detach().float(), red, unbiased=False)
            rm.mul_(momentum).add_((1.0 - momentum) * mean.to(rm.dtype))
            rv.mul_(momentum).add_((1.0 - momentum) * var.to(rv.dtype))
        out = F.batch_norm(t, None, None, w, b, True, 0.0, epsilon)
    else:
        out = F.batch_norm(t, rm, rv, w, b, use_batch, 1.0 - momentum, epsilon)
    if r is not None:
        out = out + r
    if act == "relu":
        out = torch.relu(out)
    elif act is not None:
        out = getattr(F, act)(out)
    return _wrap(out)


def instance_norm(x, running_mean=None, running_var=None, weight=None, bias=None, use_input_stats=True,
                  momentum=0.9, eps=1e-05, data_format="NCHW", name=None):
    t = T(x)
    cl = data_format in ("NHWC", "NLC", "NDHWC")
    nd = t.dim()
    if cl:
        t = t.permute(0, nd - 1, *range(1, nd - 1))
    out = F.instance_norm(t, T(running_mean), T(running_var), T(weight), T(bias), use_input_stats,
                          1.0 - momentum, eps)
    if cl:
        out = out.permute(0, *range(2, nd), 1)
    return _wrap(out)


def group_norm(x, num_groups, epsilon=1e-05, weight=None, bias=None, data_format="NCHW", name=None):
    t = T(x)
    cl = data_format in ("NHWC", "NLC", "NDHWC")
    nd = t.dim()
    if cl:
        t = t.permute(0, nd - 1, *range(1, nd - 1))
    out = F.group_norm(t, num_groups, T(weight), T(bias), epsilon)
    if cl:
        out = out.permute(0, *range(2, nd), 1)
    return _wrap(out)


def local_response_norm(x, size, alpha=1e-4, beta=0.75, k=1.0, data_format="NCHW", name=None):
    t = T(x)
    cl = data_format in ("NHWC", "NLC", "NDHWC")
    nd = t.dim()
    if cl:
        t = t.permute(0, nd - 1, *range(1, nd - 1))
    out = F.local_response_norm(t, size, alpha, beta, k)
    if cl:
        out = out.permute(0, *range(2, nd), 1)
    return _wrap(out)


def normalize(x, p=2, axis=1, epsilon=1e-12, name=None):
    return _wrap(F.normalize(T(x), float(p), axis, epsilon))
