"""paddle.incubate.xpu.ResNetBasicBlock / resnet_basic_block: the fused ResNet basic block.

Reference: python/paddle/incubate/xpu/resnet_block.py:29 (resnet_basic_block), :327 (ResNetBasicBlock) — an XPU
fused kernel. The same block runs here on the NHWC HIP path: conv1 -> BN1 -> relu -> conv2 -> BN2 (+ shortcut
conv3 -> BN3, or the input) -> relu, with the conv -> BN statistics fusion and the add + relu in the BN apply
(incubate/operators/resnet_unit.py conv_bn_act)."""
from __future__ import annotations

from .. import nn
from ..framework.tensor import _wrap
from ..nn import initializer as I
from .operators.resnet_unit import _filter_nchw, _t, conv_bn_act


def resnet_basic_block(x, filter1, scale1, bias1, mean1, var1, filter2, scale2, bias2, mean2, var2, filter3, scale3,
                       bias3, mean3, var3, stride1, stride2, stride3, padding1, padding2, padding3, dilation1,
                       dilation2, dilation3, groups, momentum, eps, data_format, has_shortcut, use_global_stats=None,
                       training=False, trainable_statistics=False, find_conv_max=True):
    train = bool(training) and not use_global_stats
    nchw = data_format == "NCHW"
    xt = _t(x)
    xn = xt.permute(0, 2, 3, 1).contiguous() if nchw else xt
    h = conv_bn_act(xn, _filter_nchw(_t(filter1), data_format), _t(scale1), _t(bias1), _t(mean1), _t(var1), stride1,
                    padding1, dilation1, groups, momentum, eps, train, "relu")
    if has_shortcut:
        res = conv_bn_act(xn, _filter_nchw(_t(filter3), data_format), _t(scale3), _t(bias3), _t(mean3), _t(var3),
                          stride3, padding3, dilation3, groups, momentum, eps, train, None)
    else:
        res = xn
    out = conv_bn_act(h, _filter_nchw(_t(filter2), data_format), _t(scale2), _t(bias2), _t(mean2), _t(var2), stride2,
                      padding2, dilation2, groups, momentum, eps, train, "relu", res.to(h.dtype).contiguous())
    return _wrap(out.permute(0, 3, 1, 2) if nchw else out)


class ResNetBasicBlock(nn.Layer):
    def __init__(self, num_channels1, num_filter1, filter1_size, num_channels2, num_filter2, filter2_size,
                 num_channels3, num_filter3, filter3_size, stride1=1, stride2=1, stride3=1, act="relu", momentum=0.9,
                 eps=1e-5, data_format="NCHW", has_shortcut=False, use_global_stats=False, is_test=False,
                 filter1_attr=None, scale1_attr=None, bias1_attr=None, moving_mean1_name=None, moving_var1_name=None,
                 filter2_attr=None, scale2_attr=None, bias2_attr=None, moving_mean2_name=None, moving_var2_name=None,
                 filter3_attr=None, scale3_attr=None, bias3_attr=None, moving_mean3_name=None, moving_var3_name=None,
                 padding1=0, padding2=0, padding3=0, dilation1=1, dilation2=1, dilation3=1,
                 trainable_statistics=False, find_conv_max=True):
        super().__init__()
        if act != "relu":
            raise ValueError("ResNetBasicBlock: only act='relu' is supported (as in the reference)")
        self._stride = (stride1, stride2, stride3)
        self._padding = (padding1, padding2, padding3)
        self._dilation = (dilation1, dilation2, dilation3)
        self._groups, self._momentum, self._eps = 1, momentum, eps
        self._data_format, self._has_shortcut = data_format, has_shortcut
        self._use_global_stats, self._is_test = use_global_stats, is_test
        nhwc = data_format == "NHWC"
        from ..nn.layer.layers import ParamAttr

        def branch(i, cin, cout, k, fattr, sattr, battr, mname, vname):
            shape = [cout, k, k, cin] if nhwc else [cout, cin, k, k]
            f = self.create_parameter(shape=shape, attr=fattr,
                                      default_initializer=I.Normal(0.0, (2.0 / (k * k * cin)) ** 0.5))
            bn_shape = [cout]
            s = self.create_parameter(shape=bn_shape, attr=sattr, dtype="float32",
                                      default_initializer=I.Constant(1.0))
            b = self.create_parameter(shape=bn_shape, attr=battr, dtype="float32", is_bias=True)
            m = self.create_parameter(shape=bn_shape, dtype="float32",
                                      attr=ParamAttr(name=mname, initializer=I.Constant(0.0), trainable=False))
            v = self.create_parameter(shape=bn_shape, dtype="float32",
                                      attr=ParamAttr(name=vname, initializer=I.Constant(1.0), trainable=False))
            m.stop_gradient = v.stop_gradient = True
            for n, t in (("filter", f), ("scale", s), ("bias", b), ("mean", m), ("var", v)):
                setattr(self, f"{n}_{i}", t)

        branch(1, num_channels1, num_filter1, filter1_size, filter1_attr, scale1_attr, bias1_attr, moving_mean1_name,
               moving_var1_name)
        branch(2, num_channels2, num_filter2, filter2_size, filter2_attr, scale2_attr, bias2_attr, moving_mean2_name,
               moving_var2_name)
        if has_shortcut:
            branch(3, num_channels3, num_filter3, filter3_size, filter3_attr, scale3_attr, bias3_attr,
                   moving_mean3_name, moving_var3_name)
        else:
            self.filter_3 = self.scale_3 = self.bias_3 = self.mean_3 = self.var_3 = None

    def forward(self, x):
        return resnet_basic_block(x, self.filter_1, self.scale_1, self.bias_1, self.mean_1, self.var_1, self.filter_2,
                                  self.scale_2, self.bias_2, self.mean_2, self.var_2, self.filter_3, self.scale_3,
                                  self.bias_3, self.mean_3, self.var_3, *self._stride, *self._padding,
                                  *self._dilation, self._groups, self._momentum, self._eps, self._data_format,
                                  self._has_shortcut, self._use_global_stats,
                                  self.training and not self._is_test)
