"""paddle.incubate.operators.ResNetUnit / resnet_unit: conv -> BN (-> + shortcut) -> act as one unit.

Reference: python/paddle/incubate/operators/resnet_unit.py:34 (resnet_unit), :158 (ResNetUnit), backed by
paddle/phi/kernels/fusion/gpu/resnet_unit_kernel.cu (cuDNN v8 fused conv-BN graphs). Here the unit runs on the
NHWC hand-written kernels with the conv -> BN statistics fusion always on (ops/_conv_bn.py: the convolution's
epilogue writes the batch-norm partials, the BN skips its statistics pass) and the residual add + relu fused into
the BN apply pass (csrc/kernels/bn.hip)."""
from __future__ import annotations

import torch

from ...framework.tensor import Tensor, _wrap
from ... import nn
from ...nn import initializer as I


def _t(x):
    return x._t if isinstance(x, Tensor) else x


def conv_bn_act(x, w, scale, bias, mean, var, stride, padding, dilation, groups, momentum, eps, training, act,
                residual=None):
    """act(BN(conv(x)) [+ residual]) on torch tensors. x / residual: NHWC; w: [Cout, Cin, KH, KW] (any strides).
    Returns NHWC. Running statistics are updated in place in training."""
    from ...ops import bn as B
    from ...ops import conv as C
    if w.dtype != x.dtype:
        w = w.to(x.dtype)
    if C.eligible_nhwc(x, w, groups) and isinstance(padding, int):
        y = C.conv2d_nhwc(x, w, None, stride, padding, dilation, bn_stats=bool(training))
    else:
        y = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w, None, stride, padding, dilation, groups)
        y = y.permute(0, 2, 3, 1).contiguous()
    return B.batch_norm_act_nhwc(y, scale.reshape(-1), bias.reshape(-1), mean.reshape(-1), var.reshape(-1),
                                 bool(training), float(momentum), float(eps), act if act else None, residual)


def _filter_nchw(f, data_format):
    """[Cout, Cin, KH, KW] view of a unit filter ([Cout, KH, KW, Cin] for NHWC units)."""
    return f.permute(0, 3, 1, 2) if data_format == "NHWC" else f


def resnet_unit(x, filter_x, scale_x, bias_x, mean_x, var_x, z, filter_z, scale_z, bias_z, mean_z, var_z, stride,
                stride_z, padding, dilation, groups, momentum, eps, data_format, fuse_add, has_shortcut,
                use_global_stats, is_test, act):
    """out = act(bn_x(conv_x(x)) + r), r = bn_z(conv_z(z)) (has_shortcut), z (fuse_add) or nothing."""
    if act not in (None, "", "relu", "identity"):
        raise ValueError(f"resnet_unit: unsupported act {act!r} (relu or identity)")
    act = "relu" if act == "relu" else None
    training = not (is_test or use_global_stats)
    xt = _t(x)
    nchw = data_format == "NCHW"
    xn = xt.permute(0, 2, 3, 1).contiguous() if nchw else xt
    res = None
    if has_shortcut:
        if z is None or filter_z is None:
            raise ValueError("resnet_unit: has_shortcut needs z and filter_z")
        zt = _t(z)
        zn = zt.permute(0, 2, 3, 1).contiguous() if nchw else zt
        res = conv_bn_act(zn, _filter_nchw(_t(filter_z), data_format), _t(scale_z), _t(bias_z), _t(mean_z),
                          _t(var_z), stride_z, padding if _t(filter_z).shape[-1] > 1 else 0, dilation, groups,
                          momentum, eps, training, None)
    elif fuse_add:
        if z is None:
            raise ValueError("resnet_unit: fuse_add needs z")
        zt = _t(z)
        res = zt.permute(0, 2, 3, 1).contiguous() if nchw else zt
    out = conv_bn_act(xn, _filter_nchw(_t(filter_x), data_format), _t(scale_x), _t(bias_x), _t(mean_x), _t(var_x),
                      stride, padding, dilation, groups, momentum, eps, training, act,
                      None if res is None else res.to(xn.dtype).contiguous())
    return _wrap(out.permute(0, 3, 1, 2) if nchw else out)


class ResNetUnit(nn.Layer):
    """Reference: incubate/operators/resnet_unit.py:158 (same constructor, parameter shapes and names)."""

    def __init__(self, num_channels_x, num_filters, filter_size, stride=1, momentum=0.9, eps=1e-5, data_format="NHWC",
                 act="relu", fuse_add=False, has_shortcut=False, use_global_stats=False, is_test=False,
                 filter_x_attr=None, scale_x_attr=None, bias_x_attr=None, moving_mean_x_name=None,
                 moving_var_x_name=None, num_channels_z=1, stride_z=1, filter_z_attr=None, scale_z_attr=None,
                 bias_z_attr=None, moving_mean_z_name=None, moving_var_z_name=None):
        super().__init__()
        if data_format not in ("NHWC", "NCHW"):
            raise ValueError(f"conv_format must be one of {{'NHWC', 'NCHW'}}, but got conv_format='{data_format}'")
        self._stride, self._stride_z = stride, stride_z
        self._dilation, self._groups = 1, 1
        self._padding = (filter_size - 1) // 2
        self._momentum, self._eps = momentum, eps
        self._data_format, self._act = data_format, act
        self._fuse_add, self._has_shortcut = fuse_add, has_shortcut
        self._use_global_stats, self._is_test = use_global_stats, is_test
        nhwc = data_format == "NHWC"
        bn_shape = [1, 1, 1, num_filters] if nhwc else [1, num_filters, 1, 1]

        def fshape(cin):
            return [num_filters, filter_size, filter_size, cin] if nhwc else [num_filters, cin, filter_size,
                                                                                filter_size]

        def finit(cin):
            return I.Normal(0.0, (2.0 / (filter_size * filter_size * cin)) ** 0.5)

        def stats(name, value):
            from ...nn.layer.layers import ParamAttr
            p = self.create_parameter(shape=bn_shape, dtype="float32",
                                      attr=ParamAttr(name=name, initializer=I.Constant(value), trainable=False))
            p.stop_gradient = True
            return p

        self.filter_x = self.create_parameter(shape=fshape(num_channels_x), attr=filter_x_attr,
                                              default_initializer=finit(num_channels_x))
        self.scale_x = self.create_parameter(shape=bn_shape, attr=scale_x_attr, dtype="float32",
                                             default_initializer=I.Constant(1.0))
        self.bias_x = self.create_parameter(shape=bn_shape, attr=bias_x_attr, dtype="float32", is_bias=True)
        self.mean_x = stats(moving_mean_x_name, 0.0)
        self.var_x = stats(moving_var_x_name, 1.0)
        if has_shortcut:
            self.filter_z = self.create_parameter(shape=fshape(num_channels_z), attr=filter_z_attr,
                                                  default_initializer=finit(num_channels_z))
            self.scale_z = self.create_parameter(shape=bn_shape, attr=scale_z_attr, dtype="float32",
                                                 default_initializer=I.Constant(1.0))
            self.bias_z = self.create_parameter(shape=bn_shape, attr=bias_z_attr, dtype="float32", is_bias=True)
            self.mean_z = stats(moving_mean_z_name, 0.0)
            self.var_z = stats(moving_var_z_name, 1.0)
        else:
            self.filter_z = self.scale_z = self.bias_z = self.mean_z = self.var_z = None

    def forward(self, x, z=None):
        if self._fuse_add and z is None:
            raise ValueError("z can not be None")
        return resnet_unit(x, self.filter_x, self.scale_x, self.bias_x, self.mean_x, self.var_x, z, self.filter_z,
                           self.scale_z, self.bias_z, self.mean_z, self.var_z, self._stride, self._stride_z,
                           self._padding, self._dilation, self._groups, self._momentum, self._eps, self._data_format,
                           self._fuse_add, self._has_shortcut, self._use_global_stats,
                           self._is_test or not self.training, self._act)

