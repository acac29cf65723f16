"""Normalisation layers. Reference: python/paddle/nn/layer/norm.py.
BatchNorm keeps paddle's state names (_mean/_variance) so .pdparams files round-trip."""
from __future__ import annotations

import numpy as np
import torch

from ...framework.tensor import Tensor, _wrap
from .. import functional as F
from .. import initializer as I
from .layers import Layer


class _BatchNormBase(Layer):
    _default_fmt = "NCHW"

    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format=None, use_global_stats=None, name=None):
        super().__init__()
        self._num_features = num_features
        self._momentum, self._epsilon = momentum, epsilon
        self._data_format = data_format or self._default_fmt
        self._use_global_stats = use_global_stats
        if weight_attr is False:
            self.weight = None
        else:
            self.weight = self.create_parameter([num_features], attr=weight_attr, dtype="float32",
                                                default_initializer=I.Constant(1.0))
        if bias_attr is False:
            self.bias = None
        else:
            self.bias = self.create_parameter([num_features], attr=bias_attr, dtype="float32", is_bias=True)
        dev = self.weight._t.device if self.weight is not None else None
        self.register_buffer("_mean", _wrap(torch.zeros(num_features, device=dev)))
        self.register_buffer("_variance", _wrap(torch.ones(num_features, device=dev)))

    def forward(self, x):
        return F.batch_norm(x, self._mean, self._variance, self.weight, self.bias, self.training, self._momentum,
                            self._epsilon, self._data_format, self._use_global_stats)

    def fused_forward(self, x, act=None, residual=None, _grad_sink=None):
        """act(self(x) [+ residual]) in one fused pass where the layer is a plain batch norm
        (fused_bn_add_activation, F.fused_bn_act); layers that override forward (SyncBatchNorm,
        legacy BatchNorm with its own act) compose the ops instead."""
        if type(self).forward is _BatchNormBase.forward:
            return F.fused_bn_act(x, self._mean, self._variance, self.weight, self.bias, self.training,
                                  self._momentum, self._epsilon, self._data_format, self._use_global_stats, act,
                                  residual, _grad_sink)
        y = self(x)
        if residual is not None:
            y = y + residual
        return getattr(F, act)(y) if act else y

    def extra_repr(self):
        return f"num_features={self._num_features}, momentum={self._momentum}, epsilon={self._epsilon}"


class BatchNorm1D(_BatchNormBase):
    _default_fmt = "NCL"

    def forward(self, x):
        fmt = self._data_format
        if x.ndim == 2:
            fmt = "NC"
        return F.batch_norm(x, self._mean, self._variance, self.weight, self.bias, self.training, self._momentum,
                            self._epsilon, fmt if fmt != "NC" else "NCHW", self._use_global_stats)


class BatchNorm2D(_BatchNormBase):
    _default_fmt = "NCHW"


class BatchNorm3D(_BatchNormBase):
    _default_fmt = "NCDHW"


class BatchNorm(_BatchNormBase):
    """Legacy paddle.nn.BatchNorm(num_channels, act=None, ...)."""

    def __init__(self, num_channels, act=None, is_test=False, momentum=0.9, epsilon=1e-05, param_attr=None,
                 bias_attr=None, dtype="float32", data_layout="NCHW", in_place=False, moving_mean_name=None,
                 moving_variance_name=None, do_model_average_for_mean_and_var=True, use_global_stats=False,
                 trainable_statistics=False):
        super().__init__(num_channels, momentum, epsilon, param_attr, bias_attr, data_layout, use_global_stats)
        self._act = act

    def forward(self, x):
        y = super().forward(x)
        if self._act:
            y = getattr(F, self._act)(y)
        return y


class SyncBatchNorm(_BatchNormBase):
    """Cross-rank BN: batch statistics and the backward's gradient statistics are all-reduced over the
    group (RCCL). Channels-last bf16 inputs run the split-phase HIP kernels (ops/bn.py sync_batch_norm).
    Reference: python/paddle/nn/layer/norm.py SyncBatchNorm, phi/kernels/gpu/sync_batch_norm_kernel.cu."""

    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format="NCHW", name=None, process_group=None):
        super().__init__(num_features, momentum, epsilon, weight_attr, bias_attr, data_format)
        self._process_group = process_group

    def forward(self, x):
        from ...distributed import collective as C
        from ...ops.bn import sync_batch_norm
        grp = self._process_group
        if not self.training or not C.is_initialized() or C.get_world_size(grp) == 1:
            return super().forward(x)
        cl = self._data_format in ("NHWC", "NLC", "NDHWC") or x.ndim == 2
        w = self.weight._t if self.weight is not None else None
        b = self.bias._t if self.bias is not None else None
        y = sync_batch_norm(x._t, w, b, self._mean._t, self._variance._t, self._momentum, self._epsilon,
                            channel_last=cl, pg=C._pg(grp))
        return _wrap(y)

    @classmethod
    def convert_sync_batchnorm(cls, layer):
        out = layer
        if isinstance(layer, _BatchNormBase) and not isinstance(layer, SyncBatchNorm):
            out = SyncBatchNorm(layer._num_features, layer._momentum, layer._epsilon, data_format=layer._data_format)
            if layer.weight is not None:
                out.weight = layer.weight
                out.bias = layer.bias
            out._mean = layer._mean
            out._variance = layer._variance
        for name, sub in list(layer._sub_layers.items()):
            out._sub_layers[name] = cls.convert_sync_batchnorm(sub)
        return out


class LayerNorm(Layer):
    def __init__(self, normalized_shape, epsilon=1e-05, weight_attr=None, bias_attr=None, name=None):
        super().__init__()
        if isinstance(normalized_shape, int):
            normalized_shape = [normalized_shape]
        self._normalized_shape = list(normalized_shape)
        self._epsilon = epsilon
        n = int(np.prod(self._normalized_shape))
        self.weight = None if weight_attr is False else self.create_parameter(
            [n], attr=weight_attr, default_initializer=I.Constant(1.0))
        self.bias = None if bias_attr is False else self.create_parameter([n], attr=bias_attr, is_bias=True)

    def forward(self, x):
        return F.layer_norm(x, self._normalized_shape, self.weight, self.bias, self._epsilon)

    def extra_repr(self):
        return f"normalized_shape={self._normalized_shape}, epsilon={self._epsilon}"


class RMSNorm(Layer):
    """RMSNorm (LLaMA). Reference: incubate fused_rms_norm. HIP kernel."""

    def __init__(self, hidden_size, epsilon=1e-6, weight_attr=None, name=None):
        super().__init__()
        self._epsilon = epsilon
        self.weight = self.create_parameter([hidden_size], attr=weight_attr, default_initializer=I.Constant(1.0))

    def forward(self, x):
        return F.rms_norm(x, None, self.weight, self._epsilon)


class GroupNorm(Layer):
    def __init__(self, num_groups, num_channels, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format="NCHW", name=None):
        super().__init__()
        self._num_groups, self._epsilon, self._data_format = num_groups, epsilon, data_format
        self.weight = None if weight_attr is False else self.create_parameter(
            [num_channels], attr=weight_attr, default_initializer=I.Constant(1.0))
        self.bias = None if bias_attr is False else self.create_parameter([num_channels], attr=bias_attr,
                                                                          is_bias=True)

    def forward(self, x):
        return F.group_norm(x, self._num_groups, self._epsilon, self.weight, self.bias, self._data_format)


class _InstanceNormBase(Layer):
    def __init__(self, num_features, epsilon=1e-05, momentum=0.9, weight_attr=None, bias_attr=None,
                 data_format="NCHW", name=None):
        super().__init__()
        self._epsilon, self._data_format = epsilon, data_format
        self.scale = None if weight_attr is False else self.create_parameter(
            [num_features], attr=weight_attr, default_initializer=I.Constant(1.0))
        self.bias = None if bias_attr is False else self.create_parameter([num_features], attr=bias_attr,
                                                                          is_bias=True)

    def forward(self, x):
        return F.instance_norm(x, weight=self.scale, bias=self.bias, eps=self._epsilon, data_format=self._data_format)


class InstanceNorm1D(_InstanceNormBase):
    pass


class InstanceNorm2D(_InstanceNormBase):
    pass


class InstanceNorm3D(_InstanceNormBase):
    pass


class LocalResponseNorm(Layer):
    def __init__(self, size, alpha=0.0001, beta=0.75, k=1.0, data_format="NCHW", name=None):
        super().__init__()
        self.size, self.alpha, self.beta, self.k, self.df = size, alpha, beta, k, data_format

    def forward(self, x):
        return F.local_response_norm(x, self.size, self.alpha, self.beta, self.k, self.df)


class SpectralNorm(Layer):
    def __init__(self, weight_shape, dim=0, power_iters=1, eps=1e-12, dtype="float32"):
        super().__init__()
        self._dim, self._power_iters, self._eps = dim, power_iters, eps
        h = weight_shape[dim]
        w = int(np.prod(weight_shape)) // h
        self.weight_u = self.create_parameter([h], default_initializer=I.Normal(0.0, 1.0))
        self.weight_u.stop_gradient = True
        self.weight_v = self.create_parameter([w], default_initializer=I.Normal(0.0, 1.0))
        self.weight_v.stop_gradient = True

    def forward(self, weight):
        w = weight._t
        perm = [self._dim] + [i for i in range(w.dim()) if i != self._dim]
        mat = w.permute(*perm).reshape(w.shape[self._dim], -1)
        u, v = self.weight_u._t, self.weight_v._t
        with torch.no_grad():
            for _ in range(self._power_iters):
                v.copy_(torch.nn.functional.normalize(mat.T @ u, dim=0, eps=self._eps))
                u.copy_(torch.nn.functional.normalize(mat @ v, dim=0, eps=self._eps))
        sigma = torch.dot(u, mat @ v)
        return _wrap(w / sigma)
