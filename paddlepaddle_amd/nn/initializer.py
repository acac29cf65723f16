"""Parameter initializers. Reference: python/paddle/nn/initializer/*.py."""
from __future__ import annotations

import math

import numpy as np
import torch

from ..framework.tensor import Tensor


def _fans(shape):
    shape = list(shape)
    if len(shape) == 0:
        return 1, 1
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        return shape[0], shape[1]
    # conv weight [out, in, k...] (paddle layout)
    rf = int(np.prod(shape[2:]))
    return shape[1] * rf, shape[0] * rf


class Initializer:
    def __call__(self, param, block=None):
        t = param._t if isinstance(param, Tensor) else param
        with torch.no_grad():
            self._init(t)
        return param

    def _init(self, t):
        raise NotImplementedError

    forward = __call__


class Constant(Initializer):
    def __init__(self, value=0.0, force_cpu=False):
        self.value = value

    def _init(self, t):
        t.fill_(self.value)


ConstantInitializer = Constant


class Normal(Initializer):
    def __init__(self, mean=0.0, std=1.0, name=None):
        self.mean, self.std = mean, std

    def _init(self, t):
        if t.dtype in (torch.bfloat16, torch.float16):
            t.copy_(torch.randn(t.shape, device=t.device, dtype=torch.float32) * self.std + self.mean)
        else:
            t.normal_(self.mean, self.std)


class NormalInitializer(Normal):
    """Legacy name (reference nn/initializer/normal.py NormalInitializer): (loc, scale, seed)."""

    def __init__(self, loc=0.0, scale=1.0, seed=0):
        super().__init__(loc, scale)


class TruncatedNormal(Initializer):
    def __init__(self, mean=0.0, std=1.0, a=-2.0, b=2.0, name=None):
        self.mean, self.std, self.a, self.b = mean, std, a, b

    def _init(self, t):
        tmp = torch.empty(t.shape, device=t.device, dtype=torch.float32)
        torch.nn.init.trunc_normal_(tmp, self.mean, self.std, self.mean + self.a * self.std,
                                    self.mean + self.b * self.std)
        t.copy_(tmp)


class TruncatedNormalInitializer(TruncatedNormal):
    """Legacy name: (loc, scale, seed, a, b) — truncation at a / b standard deviations."""

    def __init__(self, loc=0.0, scale=1.0, seed=0, a=-2.0, b=2.0):
        super().__init__(loc, scale, a, b)


class Uniform(Initializer):
    def __init__(self, low=-1.0, high=1.0, name=None):
        self.low, self.high = low, high

    def _init(self, t):
        tmp = torch.empty(t.shape, device=t.device, dtype=torch.float32).uniform_(self.low, self.high)
        t.copy_(tmp)


class UniformInitializer(Uniform):
    """Legacy name (reference uniform.py UniformInitializer): (low, high, seed, diag_num, diag_step, diag_val);
    with diag_num > 0 the flat elements i * diag_step + i (i < diag_num) are set to diag_val afterwards."""

    def __init__(self, low=-1.0, high=1.0, seed=0, diag_num=0, diag_step=0, diag_val=1.0):
        super().__init__(low, high)
        self.diag_num, self.diag_step, self.diag_val = int(diag_num), int(diag_step), float(diag_val)

    def _init(self, t):
        super()._init(t)
        if self.diag_num > 0:
            idx = torch.arange(self.diag_num, device=t.device) * (self.diag_step + 1)
            t.view(-1).index_fill_(0, idx, self.diag_val)


class XavierNormal(Initializer):
    def __init__(self, fan_in=None, fan_out=None, gain=1.0, name=None):
        self.fan_in, self.fan_out, self.gain = fan_in, fan_out, gain

    def _init(self, t):
        fi, fo = _fans(t.shape)
        fi = self.fan_in or fi
        fo = self.fan_out or fo
        std = self.gain * math.sqrt(2.0 / (fi + fo))
        Normal(0.0, std)._init(t)


class XavierUniform(Initializer):
    def __init__(self, fan_in=None, fan_out=None, gain=1.0, name=None):
        self.fan_in, self.fan_out, self.gain = fan_in, fan_out, gain

    def _init(self, t):
        fi, fo = _fans(t.shape)
        fi = self.fan_in or fi
        fo = self.fan_out or fo
        lim = self.gain * math.sqrt(6.0 / (fi + fo))
        Uniform(-lim, lim)._init(t)


class XavierInitializer(Initializer):
    """Legacy name (reference xavier.py XavierInitializer): (uniform, fan_in, fan_out, seed)."""

    def __init__(self, uniform=True, fan_in=None, fan_out=None, seed=0, gain=1.0):
        self._impl = (XavierUniform if uniform else XavierNormal)(fan_in, fan_out, gain)

    def _init(self, t):
        self._impl._init(t)


def calculate_gain(nonlinearity, param=None):
    nl = nonlinearity.lower()
    if nl in ("sigmoid", "linear", "conv1d", "conv2d", "conv3d", "conv1d_transpose", "conv2d_transpose",
              "conv3d_transpose"):
        return 1.0
    if nl == "tanh":
        return 5.0 / 3
    if nl == "relu":
        return math.sqrt(2.0)
    if nl == "leaky_relu":
        p = 0.01 if param is None else param
        return math.sqrt(2.0 / (1 + p ** 2))
    if nl == "selu":
        return 3.0 / 4
    raise ValueError(f"unsupported nonlinearity {nonlinearity}")


class KaimingNormal(Initializer):
    def __init__(self, fan_in=None, negative_slope=0.0, nonlinearity="relu", name=None):
        self.fan_in, self.slope, self.nl = fan_in, negative_slope, nonlinearity

    def _init(self, t):
        fi = self.fan_in or _fans(t.shape)[0]
        gain = calculate_gain(self.nl, self.slope)
        Normal(0.0, gain / math.sqrt(fi))._init(t)


class KaimingUniform(Initializer):
    def __init__(self, fan_in=None, negative_slope=0.0, nonlinearity="relu", name=None):
        self.fan_in, self.slope, self.nl = fan_in, negative_slope, nonlinearity

    def _init(self, t):
        fi = self.fan_in or _fans(t.shape)[0]
        gain = calculate_gain(self.nl, self.slope)
        lim = gain * math.sqrt(3.0 / fi)
        Uniform(-lim, lim)._init(t)


class MSRAInitializer(Initializer):
    """Legacy name (reference kaiming.py MSRAInitializer): (uniform, fan_in, seed, negative_slope,
    nonlinearity); uniform by default like the reference."""

    def __init__(self, uniform=True, fan_in=None, seed=0, negative_slope=0, nonlinearity="relu"):
        self._impl = (KaimingUniform if uniform else KaimingNormal)(fan_in, negative_slope, nonlinearity)

    def _init(self, t):
        self._impl._init(t)


class Assign(Initializer):
    def __init__(self, value, name=None):
        self.value = value

    def _init(self, t):
        v = self.value._t if isinstance(self.value, Tensor) else torch.as_tensor(np.asarray(self.value))
        if v.numel() == t.numel():
            t.copy_(v.reshape(t.shape).to(t.dtype))
        else:  # the reference's assign_value_ gives the parameter the value's shape
            with torch.no_grad():
                t.data = v.detach().to(device=t.device, dtype=t.dtype).clone()


NumpyArrayInitializer = Assign


class Orthogonal(Initializer):
    def __init__(self, gain=1.0, name=None):
        self.gain = gain

    def _init(self, t):
        tmp = torch.empty(t.shape, dtype=torch.float32, device=t.device)
        torch.nn.init.orthogonal_(tmp, self.gain)
        t.copy_(tmp)


class Dirac(Initializer):
    def __init__(self, groups=1, name=None):
        self.groups = groups

    def _init(self, t):
        torch.nn.init.dirac_(t, self.groups)


class Bilinear(Initializer):
    def _init(self, t):
        shape = t.shape
        f = math.ceil(shape[3] / 2)
        c = (2 * f - 1 - f % 2) / (2.0 * f)
        w = torch.zeros(shape, dtype=torch.float32)
        for i in range(int(np.prod(shape))):
            x = i % shape[3]
            y = (i // shape[3]) % shape[2]
            w.view(-1)[i] = (1 - abs(x / f - c)) * (1 - abs(y / f - c))
        t.copy_(w)


_global_weight_init = None
_global_bias_init = None


def set_global_initializer(weight_init, bias_init=None):
    global _global_weight_init, _global_bias_init
    _global_weight_init, _global_bias_init = weight_init, bias_init
