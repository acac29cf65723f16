"""paddle.quantization: QAT / PTQ with configurable quanters and observers, int8 and fp8 (OCP e4m3).

Reference: python/paddle/quantization/ (config.py QuantConfig, factory.py quanter/ObserverFactory,
base_quanter.py, base_observer.py, qat.py QAT, ptq.py PTQ, quanters/abs_max.py
FakeQuanterWithAbsMaxObserver, observers/abs_max.py AbsmaxObserver, observers/groupwise.py,
wrapper.py ObserveWrapper).

gfx950 has native OCP fp8 (e4m3fn / e5m2, not the fnuz variants of gfx942), so the fp8 quanter
rounds through the real fp8 dtype; int8 uses symmetric rounding. Fake quantisation uses a
straight-through estimator so QAT trains through the rounding."""
from __future__ import annotations

import copy

import torch

from .. import nn
from ..framework.tensor import Tensor, _wrap


# ------------------------------------------------------------------------------ primitives
class _STE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scale, qmax, fp8):
        s = scale.clamp_min(1e-12)
        if fp8 is not None:
            y = (x / s * qmax).clamp(-qmax, qmax).to(fp8).to(x.dtype) * s / qmax
        else:
            y = torch.round(x / s * qmax).clamp(-qmax, qmax) * s / qmax
        return y

    @staticmethod
    def backward(ctx, g):
        return g, None, None, None


def _fp8_of(bits):
    return {"e4m3": torch.float8_e4m3fn, "e5m2": torch.float8_e5m2}.get(bits)


def _qmax(bit_length):
    if isinstance(bit_length, str):
        return {"e4m3": 448.0, "e5m2": 57344.0}[bit_length]
    return float(2 ** (bit_length - 1) - 1)


def fake_quant(x, scale, bit_length=8):
    return _STE.apply(x, scale, _qmax(bit_length), _fp8_of(bit_length))


# ------------------------------------------------------------------------------ base classes
class BaseObserver(nn.Layer):
    def __init__(self):
        super().__init__()

    def forward(self, x):
        self._observe(x._t.detach())
        return x

    def _observe(self, t):
        raise NotImplementedError

    def cal_thresholds(self):
        pass

    def scales(self):
        raise NotImplementedError

    def zero_points(self):
        return None

    def bit_length(self):
        return self._bits

    def quant_axis(self):
        return -1


class BaseQuanter(BaseObserver):
    pass


class _Factory:
    """quanter/observer factory: holds the class + kwargs, instantiated per layer."""

    def __init__(self, cls, **kwargs):
        self.cls, self.kwargs = cls, kwargs

    def _instance(self, layer=None):
        return self.cls(**self.kwargs)

    def __repr__(self):
        return f"{self.cls.__name__}Factory({self.kwargs})"


def quanter(class_name):
    """Decorator registering a quanter class; the decorated name becomes a factory."""
    def deco(cls):
        def factory(**kwargs):
            return _Factory(cls, **kwargs)
        factory._cls = cls
        factory.__name__ = class_name
        return factory
    return deco


# ------------------------------------------------------------------------------ observers / quanters
class _AbsmaxObserverImpl(BaseObserver):
    def __init__(self, quant_bits=8):
        super().__init__()
        self._bits = quant_bits
        self.register_buffer("_absmax", _wrap(torch.zeros(())))

    def _observe(self, t):
        m = t.abs().max().float().to(self._absmax._t.device)
        self._absmax._t.copy_(torch.maximum(self._absmax._t, m))

    def scales(self):
        return self._absmax


class _GroupWiseObserverImpl(BaseObserver):
    def __init__(self, quant_bits=4, group_size=128):
        super().__init__()
        self._bits, self.group_size = quant_bits, group_size
        self._scales = None

    def _observe(self, t):
        g = t.reshape(-1, self.group_size).abs().amax(-1).float()
        self._scales = g if self._scales is None else torch.maximum(self._scales, g)

    def scales(self):
        return _wrap(self._scales)


class _FakeQuanterWithAbsMaxObserverImpl(BaseQuanter):
    def __init__(self, moving_rate=0.9, bit_length=8, dtype="float32", name=None):
        super().__init__()
        self._bits = bit_length
        self.moving_rate = moving_rate
        self.register_buffer("_scale", _wrap(torch.zeros(())))
        self.register_buffer("_state", _wrap(torch.zeros(())))
        self.register_buffer("_accum", _wrap(torch.zeros(())))

    def forward(self, x):
        t = x._t
        if self.training:
            with torch.no_grad():
                m = t.detach().abs().max().float().to(self._scale._t.device)
                self._state._t.mul_(self.moving_rate).add_(1.0)
                self._accum._t.mul_(self.moving_rate).add_(m)
                self._scale._t.copy_(self._accum._t / self._state._t)
        scale = self._scale._t.to(t.device, t.dtype if t.is_floating_point() else torch.float32)
        return _wrap(fake_quant(t, scale, self._bits))

    def scales(self):
        return self._scale


class _FakeQuanterChannelWiseAbsMaxImpl(BaseQuanter):
    def __init__(self, bit_length=8, quant_axis=-1, dtype="float32", name=None):
        super().__init__()
        self._bits, self._axis = bit_length, quant_axis
        self._scale = None

    def forward(self, x):
        t = x._t
        ax = self._axis % t.dim()
        dims = [d for d in range(t.dim()) if d != ax]
        s = t.detach().abs().amax(dim=dims, keepdim=True).float()
        self._scale = s
        return _wrap(fake_quant(t, s.to(t.dtype), self._bits))

    def scales(self):
        return _wrap(self._scale)

    def quant_axis(self):
        return self._axis


AbsmaxObserver = quanter("AbsmaxObserver")(_AbsmaxObserverImpl)
GroupWiseWeightObserver = quanter("GroupWiseWeightObserver")(_GroupWiseObserverImpl)
FakeQuanterWithAbsMaxObserver = quanter("FakeQuanterWithAbsMaxObserver")(_FakeQuanterWithAbsMaxObserverImpl)
FakeQuanterChannelWiseAbsMaxObserver = quanter("FakeQuanterChannelWiseAbsMaxObserver")(
    _FakeQuanterChannelWiseAbsMaxImpl)


class observers:  # paddle.quantization.observers namespace
    AbsmaxObserver = AbsmaxObserver
    GroupWiseWeightObserver = GroupWiseWeightObserver


class quanters:  # paddle.quantization.quanters namespace
    FakeQuanterWithAbsMaxObserver = FakeQuanterWithAbsMaxObserver
    FakeQuanterChannelWiseAbsMaxObserver = FakeQuanterChannelWiseAbsMaxObserver


# ------------------------------------------------------------------------------ config
class QuantConfig:
    def __init__(self, activation=None, weight=None):
        self._global = (activation, weight)
        self._by_layer = {}
        self._by_name = {}
        self._by_type = {}
        self._qat_layer_mapping = {nn.Linear: QuantedLinear, nn.Conv2D: QuantedConv2D}

    def add_layer_config(self, layer, activation=None, weight=None):
        for l in (layer if isinstance(layer, (list, tuple)) else [layer]):
            self._by_layer[id(l)] = (activation, weight)

    def add_name_config(self, layer_name, activation=None, weight=None):
        for n in (layer_name if isinstance(layer_name, (list, tuple)) else [layer_name]):
            self._by_name[n] = (activation, weight)

    def add_type_config(self, layer_type, activation=None, weight=None):
        for t in (layer_type if isinstance(layer_type, (list, tuple)) else [layer_type]):
            self._by_type[t] = (activation, weight)

    def add_qat_layer_mapping(self, source, target):
        self._qat_layer_mapping[source] = target

    def _config_for(self, name, layer):
        if id(layer) in self._by_layer:
            return self._by_layer[id(layer)]
        if name in self._by_name:
            return self._by_name[name]
        for t, c in self._by_type.items():
            if isinstance(layer, t):
                return c
        return self._global

    def __repr__(self):
        return f"QuantConfig(global={self._global})"


def _make(f):
    if f is None:
        return None
    if isinstance(f, _Factory):
        return f._instance()
    if isinstance(f, type):
        return f()
    return copy.deepcopy(f)


class QuantedLinear(nn.Layer):
    def __init__(self, layer, q_config):
        super().__init__()
        self.weight = layer.weight
        self.bias = layer.bias
        act, wq = q_config
        self.activation_quanter = _make(act)
        self.weight_quanter = _make(wq)

    def forward(self, x):
        if self.activation_quanter is not None:
            x = self.activation_quanter(x)
        w = self.weight_quanter(self.weight) if self.weight_quanter is not None else self.weight
        return nn.functional.linear(x, w, self.bias)


class QuantedConv2D(nn.Layer):
    def __init__(self, layer, q_config):
        super().__init__()
        self._conv = layer
        act, wq = q_config
        self.activation_quanter = _make(act)
        self.weight_quanter = _make(wq)

    def forward(self, x):
        if self.activation_quanter is not None:
            x = self.activation_quanter(x)
        w = self._conv.weight
        if self.weight_quanter is not None:
            qw = self.weight_quanter(w)
            saved = w._t
            w._t = qw._t
            try:
                return self._conv(x)
            finally:
                w._t = saved
        return self._conv(x)


class ObserveWrapper(nn.Layer):
    def __init__(self, observer, observed, observe_input=True):
        super().__init__()
        self._observer = observer
        self._observed = observed
        self._observe_input = observe_input

    def forward(self, *inputs, **kw):
        if self._observe_input:
            self._observer(inputs[0])
            return self._observed(*inputs, **kw)
        out = self._observed(*inputs, **kw)
        self._observer(out)
        return out


def _replace(model, config, mapping, inplace):
    m = model if inplace else copy.deepcopy(model)
    for name, sub in list(m.named_sublayers()):
        cfg = config._config_for(name, sub)
        if cfg == (None, None):
            continue
        for src, dst in mapping.items():
            if type(sub) is src:
                parent = m
                parts = name.split(".")
                for p in parts[:-1]:
                    parent = getattr(parent, p) if not p.isdigit() else parent[int(p)]
                new = dst(sub, cfg)
                if parts[-1].isdigit():
                    parent[int(parts[-1])] = new
                else:
                    setattr(parent, parts[-1], new)
                break
    return m


class QAT:
    def __init__(self, config):
        self._config = config

    def quantize(self, model, inplace=False):
        return _replace(model, self._config, self._config._qat_layer_mapping, inplace)

    def convert(self, model, inplace=False, remain_weight=False):
        """Freeze: weights are replaced by their quantised-dequantised values; quanters become
        fixed-scale (eval) fake quant nodes."""
        m = model if inplace else copy.deepcopy(model)
        m.eval()
        with torch.no_grad():
            for _, sub in m.named_sublayers(include_self=True):
                if not isinstance(sub, (QuantedLinear, QuantedConv2D)):
                    continue
                w = sub.weight if isinstance(sub, QuantedLinear) else sub._conv.weight
                q = sub.weight_quanter
                if q is not None and not remain_weight:
                    if isinstance(q, BaseQuanter):
                        w._t.copy_(q(w)._t)
                    else:  # observer: quantise with the observed range
                        q(w)
                        w._t.copy_(fake_quant(w._t, q.scales()._t.to(w._t.dtype), q.bit_length()))
                    sub.weight_quanter = None
                a = sub.activation_quanter
                if a is not None and not isinstance(a, BaseQuanter):
                    sub.activation_quanter = _FixedQuant(a.scales()._t.clone(), a.bit_length())
        return m


class _FixedQuant(nn.Layer):
    """Inference-time activation quant-dequant with a calibrated scale."""

    def __init__(self, scale, bits):
        super().__init__()
        self.register_buffer("scale", _wrap(scale))
        self.bits = bits

    def forward(self, x):
        t = x._t
        return _wrap(fake_quant(t, self.scale._t.to(t.device, t.dtype), self.bits))


class PTQ(QAT):
    """Observers record activation / weight ranges on calibration batches; convert() bakes scales."""

    def quantize(self, model, inplace=False):
        return _replace(model, self._config, self._config._qat_layer_mapping, inplace)

    def convert(self, model, inplace=False, remain_weight=False):
        m = super().convert(model, inplace, remain_weight)
        return m


import sys as _sys  # noqa: E402
# `from paddle.quantization.quanters import ...` / `.observers import ...` work like the reference packages
_sys.modules[__name__ + ".quanters"] = quanters
_sys.modules[__name__ + ".observers"] = observers
