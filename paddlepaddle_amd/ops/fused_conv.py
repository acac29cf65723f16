"""Fused convolution units the program passes rewrite to (distributed/passes/conv_passes.py), each ONE traced node:

* ``relu_depthwise_conv2d`` — relu(x) then a depthwise convolution (reference fuse_relu_depthwise_conv_pass /
  depthwise_conv2d ``fuse_relu_before_depthwise_conv``): on the NHWC HIP kernels the ReLU is applied on the
  convolution's loads and its mask in the data gradient (csrc/kernels/dwconv.hip, shape[14]), so relu(x) is never
  written; elsewhere relu + conv.
* ``conv_bn_unit`` — conv (no bias) -> training / inference batch norm (+ residual) (+ relu) (reference fuse_resunit
  pass -> fused resnet_unit, fusion/gpu/resnet_unit_kernel.cu): incubate.operators.resnet_unit.conv_bn_act, i.e.
  the NHWC convolution with the BN statistics in its epilogue and the residual add + ReLU in the BN apply kernel.

Both take and return the layouts of the ops they replace (NCHW logical tensors; ``channels_last`` says the input is
an NHWC tensor whose NCHW view fed the original convolution)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..framework.trace_hook import static_op

__all__ = ["relu_depthwise_conv2d", "conv_bn_unit"]


def _pair(v):
    if isinstance(v, (list, tuple)):
        return (int(v[0]), int(v[1])) if len(v) == 2 else (int(v[0]),) * 2
    return (int(v),) * 2


@static_op
def relu_depthwise_conv2d(x, weight, bias, stride, padding, dilation, groups, channels_last=False):
    """conv2d(relu(x_nchw), weight, bias, stride, padding, dilation, groups) with groups == channels; x is NHWC
    when ``channels_last`` (the result is still the NCHW logical output of the conv it replaces)."""
    from . import dwconv
    st, pd, dl = _pair(stride), _pair(padding), _pair(dilation)
    if channels_last and not isinstance(padding, str) and dwconv.eligible(x, weight, groups):
        w = weight if weight.dtype == x.dtype else weight.to(x.dtype)
        b = None if bias is None else bias.to(x.dtype)

        def fallback(xx, ww):
            return F.conv2d(xx.permute(0, 3, 1, 2), ww, b, st, pd, dl, groups).permute(0, 2, 3, 1)
        y = dwconv.depthwise_conv2d_nhwc(x, w, b, st, pd, dl, fallback, pre_relu=True)
        if y is not None:
            return y.permute(0, 3, 1, 2)
    xc = x.permute(0, 3, 1, 2) if channels_last else x
    return F.conv2d(torch.relu(xc), weight, bias, stride, padding, dilation, groups)


@static_op
def conv_bn_unit(x, weight, stride, padding, dilation, groups, scale, bias, running_mean, running_var,
                 training=True, momentum=0.9, eps=1e-5, act=None, residual=None):
    """act(BN(conv(x)) [+ residual]) with x / residual / the result NHWC (the layout of the batch_norm_act_nhwc
    node it replaces); running statistics updated in place in training."""
    from ..incubate.operators.resnet_unit import conv_bn_act
    st, pd, dl = _pair(stride), _pair(padding), _pair(dilation)
    if st[0] == st[1] and pd[0] == pd[1] and dl[0] == dl[1]:
        return conv_bn_act(x, weight, scale, bias, running_mean, running_var, st[0], pd[0], dl[0], groups, momentum,
                           eps, training, act, residual)
    from .bn import batch_norm_act_nhwc
    y = F.conv2d(x.permute(0, 3, 1, 2), weight.to(x.dtype), None, st, pd, dl, groups).permute(0, 2, 3, 1)
    return batch_norm_act_nhwc(y.contiguous(), scale, bias, running_mean, running_var, training, momentum, eps, act,
                               residual)
