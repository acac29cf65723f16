"""Activation layers. Reference: python/paddle/nn/layer/activation.py."""
from __future__ import annotations

from .. import functional as F
from .. import initializer as I
from .layers import Layer


def _simple(name, fn, params=()):
    def __init__(self, *args, name=None, **kwargs):
        Layer.__init__(self)
        vals = dict(zip(params, args))
        for k, default in params_defaults.items():
            setattr(self, "_" + k, kwargs.get(k, vals.get(k, default)))

    params_defaults = dict(params)
    params = [p for p, _ in params]

    def forward(self, x):
        kw = {k: getattr(self, "_" + k) for k in params}
        return fn(x, **kw)

    def extra_repr(self):
        return ", ".join(f"{k}={getattr(self, '_' + k)}" for k in params)

    return type(name, (Layer,), {"__init__": __init__, "forward": forward, "extra_repr": extra_repr})


ReLU = _simple("ReLU", F.relu)
ReLU6 = _simple("ReLU6", F.relu6)
ELU = _simple("ELU", F.elu, (("alpha", 1.0),))
SELU = _simple("SELU", F.selu, (("scale", 1.0507009873554804934193349852946), ("alpha", 1.6732632423543772848170429916717)))
CELU = _simple("CELU", F.celu, (("alpha", 1.0),))
GELU = _simple("GELU", F.gelu, (("approximate", False),))
Silu = _simple("Silu", F.silu)
Swish = _simple("Swish", F.silu)
Sigmoid = _simple("Sigmoid", F.sigmoid)
Hardsigmoid = _simple("Hardsigmoid", F.hardsigmoid)
Hardswish = _simple("Hardswish", F.hardswish)
Hardtanh = _simple("Hardtanh", F.hardtanh, (("min", -1.0), ("max", 1.0)))
Hardshrink = _simple("Hardshrink", F.hardshrink, (("threshold", 0.5),))
Softshrink = _simple("Softshrink", F.softshrink, (("threshold", 0.5),))
Tanhshrink = _simple("Tanhshrink", F.tanhshrink)
LeakyReLU = _simple("LeakyReLU", F.leaky_relu, (("negative_slope", 0.01),))
LogSigmoid = _simple("LogSigmoid", F.log_sigmoid)
Mish = _simple("Mish", F.mish)
Softmax = _simple("Softmax", F.softmax, (("axis", -1),))
LogSoftmax = _simple("LogSoftmax", F.log_softmax, (("axis", -1),))
Softplus = _simple("Softplus", F.softplus, (("beta", 1), ("threshold", 20)))
Softsign = _simple("Softsign", F.softsign)
Tanh = _simple("Tanh", F.tanh)
ThresholdedReLU = _simple("ThresholdedReLU", F.thresholded_relu, (("threshold", 1.0), ("value", 0.0)))
Maxout = _simple("Maxout", F.maxout, (("groups", 2), ("axis", 1)))
GLU = _simple("GLU", F.glu, (("axis", -1),))
RReLU = _simple("RReLU", F.rrelu, (("lower", 1.0 / 8.0), ("upper", 1.0 / 3.0)))


class Softmax2D(Layer):
    def __init__(self, name=None):
        super().__init__()

    def forward(self, x):
        return F.softmax(x, axis=-3)


class PReLU(Layer):
    def __init__(self, num_parameters=1, init=0.25, weight_attr=None, data_format="NCHW", name=None):
        super().__init__()
        self._data_format = data_format
        self.weight = self.create_parameter([num_parameters], attr=weight_attr,
                                            default_initializer=I.Constant(init))

    def forward(self, x):
        return F.prelu(x, self.weight, self._data_format)
