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
import inspect

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
    """quanter/observer factory: holds the layer class + its arguments, instantiated per layer
    (reference factory.py QuanterFactory / ObserverFactory). Printing lists every argument with the
    defaults filled in, `name` first, as the reference's factories do."""

    def __init__(self, cls, display, args=(), kwargs=None):
        self.cls, self._display = cls, display
        # the layer being quantized is the instance's first argument (reference observer / quanter layers), not a
        # factory argument
        params = inspect.signature(cls.__init__).parameters
        self._takes_layer = "layer" in params
        sig = [p for p in params.values() if p.name not in ("self", "layer")]
        bound = {p.name: p.default for p in sig if p.default is not inspect.Parameter.empty}
        for p, v in zip(sig, args):
            bound[p.name] = v
        bound.update(kwargs or {})
        order = (["name"] if "name" in bound else []) + [p.name for p in sig if p.name != "name"]
        self.kwargs = {k: bound[k] for k in order if k in bound}

    def _instance(self, layer=None):
        return self.cls(layer, **self.kwargs) if self._takes_layer else self.cls(**self.kwargs)

    def __str__(self):
        return f"{self._display}(" + ",".join(f"{k}={v}" for k, v in self.kwargs.items()) + ")"

    __repr__ = __str__


def quanter(class_name):
    """Decorator registering a quanter class; the decorated name becomes a factory."""
    def deco(cls):
        def factory(*args, **kwargs):
            return _Factory(cls, class_name, args, kwargs)
        factory._cls = cls
        factory.__name__ = class_name
        return factory
    return deco


# ------------------------------------------------------------------------------ observers / quanters
class AbsmaxObserverLayer(BaseObserver):
    def __init__(self, layer=None, quant_bits=8):
        super().__init__()
        object.__setattr__(self, "_layer", layer)  # a reference, not a sublayer (no parameter re-registration)
        self._bits = quant_bits
        self.register_buffer("_absmax", _wrap(torch.zeros(())))

    def _observe(self, t):
        m = t.abs().max().float().to(self._absmax._t.device)
        self._absmax._t.copy_(torch.maximum(self._absmax._t, m))

    def scales(self):
        return self._absmax


class GroupWiseWeightObserverLayer(BaseObserver):
    def __init__(self, layer=None, quant_bits=8, group_size=128):
        super().__init__()
        object.__setattr__(self, "_layer", layer)  # a reference, not a sublayer (no parameter re-registration)
        self._bits, self.group_size = quant_bits, group_size
        self._scales = None

    def _observe(self, t):
        g = t.reshape(-1, self.group_size).abs().amax(-1).float()
        self._scales = g if self._scales is None else torch.maximum(self._scales, g)

    def scales(self):
        return _wrap(self._scales)


class FakeQuanterWithAbsMaxObserverLayer(BaseQuanter):
    def __init__(self, layer=None, name=None, moving_rate=0.9, bit_length=8, dtype="float32"):
        super().__init__()
        object.__setattr__(self, "_layer", layer)  # a reference, not a sublayer (no parameter re-registration)
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


class FakeQuanterChannelWiseAbsMaxObserverLayer(BaseQuanter):
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


AbsmaxObserver = quanter("AbsmaxObserver")(AbsmaxObserverLayer)
GroupWiseWeightObserver = quanter("GroupWiseWeightObserver")(GroupWiseWeightObserverLayer)


def FakeQuanterWithAbsMaxObserver(moving_rate=0.9, bit_length=8, dtype="float32", name=None):
    """factory; positional order is the reference's (moving_rate, bit_length, dtype, name)"""
    return _Factory(FakeQuanterWithAbsMaxObserverLayer, "FakeQuanterWithAbsMaxObserver",
                    kwargs=dict(name=name, moving_rate=moving_rate, bit_length=bit_length, dtype=dtype))


FakeQuanterWithAbsMaxObserver._cls = FakeQuanterWithAbsMaxObserverLayer
FakeQuanterChannelWiseAbsMaxObserver = quanter("FakeQuanterChannelWiseAbsMaxObserver")(
    FakeQuanterChannelWiseAbsMaxObserverLayer)


class observers:  # paddle.quantization.observers namespace
    AbsmaxObserver = AbsmaxObserver
    GroupWiseWeightObserver = GroupWiseWeightObserver


class quanters:  # paddle.quantization.quanters namespace
    FakeQuanterWithAbsMaxObserver = FakeQuanterWithAbsMaxObserver
    FakeQuanterChannelWiseAbsMaxObserver = FakeQuanterChannelWiseAbsMaxObserver


# ------------------------------------------------------------------------------ config
class SingleLayerConfig:
    """activation + weight quanter factories of one layer (reference config.py SingleLayerConfig)."""

    def __init__(self, activation=None, weight=None):
        self._activation, self._weight = activation, weight

    @property
    def activation(self):
        return self._activation

    @property
    def weight(self):
        return self._weight

    def __str__(self):
        return f"activation: {self._activation}\nweight: {self._weight}"


_DEFAULT_LEAVES = (nn.ReLU, nn.AvgPool2D)


class QuantConfig:
    """Maps every sublayer of a model to a SingleLayerConfig (reference config.py QuantConfig).

    Precedence when `_specify` walks the model: global config < parent's config < config by layer
    type < config by layer full name (`add_layer_config` keys by `layer.full_name()`, so it survives
    the deep copy QAT/PTQ make of a non-inplace model)."""

    def __init__(self, activation=None, weight=None):
        self._global_config = None if activation is None and weight is None else \
            SingleLayerConfig(activation, weight)
        self._layer2config = {}
        self._prefix2config = {}
        self._type2config = {}
        self._model = None
        self._qat_layer_mapping = {nn.Linear: QuantedLinear, nn.Conv2D: QuantedConv2D}
        self._customized_qat_layer_mapping = {}
        self._customized_leaves = []

    # ------------------------------------------------------------------ configuration
    def add_layer_config(self, layer, activation=None, weight=None):
        for l in (layer if isinstance(layer, (list, tuple)) else [layer]):
            self.add_name_config(l.full_name(), activation=activation, weight=weight)

    def add_name_config(self, layer_name, activation=None, weight=None):
        for n in (layer_name if isinstance(layer_name, (list, tuple)) else [layer_name]):
            self._prefix2config[n] = SingleLayerConfig(activation, weight)

    def add_type_config(self, layer_type, activation=None, weight=None):
        for t in (layer_type if isinstance(layer_type, (list, tuple)) else [layer_type]):
            if not (isinstance(t, type) and issubclass(t, nn.Layer)):
                raise TypeError("add_type_config expects subclasses of paddle.nn.Layer")
            self._type2config[t] = SingleLayerConfig(activation, weight)

    def add_qat_layer_mapping(self, source, target):
        if not (isinstance(source, type) and isinstance(target, type) and issubclass(target, nn.Layer)):
            raise TypeError("add_qat_layer_mapping expects two Layer classes")
        self._qat_layer_mapping[source] = target
        self._customized_qat_layer_mapping[source] = target

    def add_customized_leaf(self, layer_type):
        self._customized_leaves.append(layer_type)

    @property
    def customized_leaves(self):
        return self._customized_leaves

    @property
    def qat_layer_mappings(self):
        return self._qat_layer_mapping

    @property
    def default_qat_layer_mapping(self):
        return {nn.Linear: QuantedLinear, nn.Conv2D: QuantedConv2D}

    @property
    def global_config(self):
        return self._global_config

    # ------------------------------------------------------------------ resolution
    def _specify(self, model):
        self._model = model
        self._specify_helper(model)
        return self

    def _specify_helper(self, model):
        for child in model.children():
            cfg = self._layer2config.get(model, self._global_config)
            cfg = self._type2config.get(type(child), cfg)
            cfg = self._prefix2config.get(child.full_name(), cfg)
            if cfg is not None:
                self._layer2config[child] = cfg
            self._specify_helper(child)
        return self

    def _get_config_by_layer(self, layer):
        return self._layer2config.get(layer)

    def _is_quantifiable(self, layer):
        return layer in self._layer2config

    def _is_leaf(self, layer):
        return (type(layer) in _DEFAULT_LEAVES or not layer._sub_layers
                or type(layer) in self._customized_leaves)

    def _has_observer_config(self, layer):
        cfg = self._get_config_by_layer(layer)
        return cfg is not None and cfg.activation is not None

    def _need_observe(self, layer):
        return self._is_leaf(layer) and self._has_observer_config(layer)

    def _get_qat_layer(self, layer):
        target = self._customized_qat_layer_mapping.get(type(layer), self._qat_layer_mapping.get(type(layer)))
        return target(layer, self._get_config_by_layer(layer))

    def _get_observe_wrapper(self, layer):
        return ObserveWrapper(_make(self._get_config_by_layer(layer).activation, layer), layer)

    # ------------------------------------------------------------------ printing
    def details(self):
        return str(self) if self._model is None else self._details_helper(self._model)

    def _details_helper(self, layer):
        lines = []
        for name, sub in layer.named_children():
            if sub in self._layer2config:
                body = self._details_helper(sub).replace("\n", "\n  ")
                cfg = str(self._layer2config[sub]).replace("\n", "\n  ")
                lines.append(f"({name}): {body}, {cfg}")
        out = layer.__class__.__name__ + "("
        if lines:
            out += "\n  " + "\n  ".join(lines) + "\n"
        return out + ")"

    def __str__(self):
        out = f"Global config:\n{self._global_config}\n"
        if self._type2config:
            out += f"Layer type config:\n{self._type2config}\n"
        if self._prefix2config:
            out += f"Layer prefix config: \n{self._prefix2config}\n"
        return out

    __repr__ = __str__


def _make(f, layer=None):
    if f is None:
        return None
    if isinstance(f, _Factory):
        return f._instance(layer)
    if isinstance(f, type):
        return f()
    return copy.deepcopy(f)


class QuantedLinear(nn.Layer):
    """Linear whose weight (and input activation) go through fake quant (reference nn/quant/qat/linear.py)."""

    def __init__(self, layer, q_config):
        super().__init__()
        self.weight = layer.weight
        self.bias = layer.bias
        self.weight_quanter = _make(q_config.weight, layer)
        self.activation_quanter = _make(q_config.activation, layer)

    def forward(self, x):
        if self.activation_quanter is not None:
            x = self.activation_quanter(x)
        w = self.weight_quanter(self.weight) if self.weight_quanter is not None else self.weight
        return nn.functional.linear(x, w, self.bias)


class QuantedConv2D(nn.Layer):
    """Conv2D with fake-quantised weight / input (reference nn/quant/qat/conv.py); the conv's parameters
    and geometry move here so the quantised weight feeds the same conv kernel."""

    def __init__(self, layer, q_config):
        super().__init__()
        self.weight, self.bias = layer.weight, layer.bias
        self._stride, self._padding, self._dilation = layer._stride, layer._padding, layer._dilation
        self._groups, self._data_format = layer._groups, layer._data_format
        self._padding_mode = layer._padding_mode
        self.weight_quanter = _make(q_config.weight, layer)
        self.activation_quanter = _make(q_config.activation, layer)

    def forward(self, x):
        if self.activation_quanter is not None:
            x = self.activation_quanter(x)
        w = self.weight_quanter(self.weight) if self.weight_quanter is not None else self.weight
        p = self._padding
        if self._padding_mode != "zeros":
            pads = [p] * 4 if isinstance(p, int) else list(p)
            x = nn.functional.pad(x, pads, mode=self._padding_mode, data_format=self._data_format)
            p = 0
        return nn.functional.conv2d(x, w, self.bias, self._stride, p, self._dilation, self._groups,
                                    self._data_format)


class ObserveWrapper(nn.Layer):
    """Puts an observer / quanter in front of (or behind) a leaf layer (reference quantization/wrapper.py)."""

    def __init__(self, observer, observed, observe_input=True):
        super().__init__()
        self._observer = observer
        self._observed = observed
        self._observe_input = observe_input

    def forward(self, *inputs, **kw):
        if self._observe_input:
            return self._observed(self._observer(*inputs), **kw)
        return self._observer(self._observed(*inputs, **kw))


class _Quantization:
    """Shared QAT / PTQ passes (reference quantization/quantize.py Quantization)."""

    def __init__(self, config):
        self._config = copy.deepcopy(config)

    def _convert_to_quant_layers(self, model):
        cfg = self._config
        for name, child in list(model.named_children()):
            if cfg._is_quantifiable(child) and type(child) in cfg.qat_layer_mappings:
                model._sub_layers[name] = cfg._get_qat_layer(child)
            else:
                self._convert_to_quant_layers(child)

    def _insert_activation_observers(self, model):
        cfg = self._config
        quanted = set(cfg._qat_layer_mapping.values()) | set(cfg._customized_qat_layer_mapping.values())
        for name, child in list(model.named_children()):
            if cfg._need_observe(child):
                model._sub_layers[name] = cfg._get_observe_wrapper(child)
            elif type(child) not in quanted:
                self._insert_activation_observers(child)

    def _prepare(self, model, inplace):
        m = model if inplace else copy.deepcopy(model)
        self._config._specify(m)
        self._convert_to_quant_layers(m)
        self._insert_activation_observers(m)
        return m

    def convert(self, model, inplace=False, remain_weight=False):
        """Freeze: weights are replaced by their quantised-dequantised values (unless remain_weight);
        activation observers / quanters become fixed-scale quant-dequant nodes."""
        m = model if inplace else copy.deepcopy(model)
        m.eval()
        with torch.no_grad():
            for sub in m.sublayers(include_self=True):
                if isinstance(sub, (QuantedLinear, QuantedConv2D)):
                    q = sub.weight_quanter
                    if q is not None and not remain_weight:
                        w = sub.weight
                        if isinstance(q, BaseQuanter):
                            w._t.copy_(q(w)._t)
                        else:  # observer: quantise with the observed range
                            q(w)
                            w._t.copy_(fake_quant(w._t, q.scales()._t.to(w._t.dtype), q.bit_length()))
                        sub.weight_quanter = None
                    a = sub.activation_quanter
                    if a is not None and not isinstance(a, BaseQuanter):
                        sub.activation_quanter = _FixedQuant(a.scales()._t.clone(), a.bit_length())
                elif isinstance(sub, ObserveWrapper):
                    o = sub._observer
                    if isinstance(o, BaseObserver) and not isinstance(o, BaseQuanter) and o.scales() is not None:
                        sub._observer = _FixedQuant(o.scales()._t.clone(), o.bit_length())
        return m

    def _details(self):
        return self._config.details()

    def __str__(self):
        return self._details()

    __repr__ = __str__


class QAT(_Quantization):
    """Quantization-aware training: fake quanters on weights + activations, trained through an STE
    (reference quantization/qat.py)."""

    def quantize(self, model, inplace=False):
        if not model.training:
            raise ValueError("QAT works on training models: call model.train() first")
        return self._prepare(model, inplace)


class _FixedQuant(nn.Layer):
    """Inference-time activation quant-dequant with a calibrated scale."""

    def __init__(self, scale, bits):
        super().__init__()
        self.register_buffer("scale", _wrap(scale))
        self.bits = bits

    def forward(self, x):
        t = x._t
        return _wrap(fake_quant(t, self.scale._t.to(t.device, t.dtype), self.bits))


class PTQ(_Quantization):
    """Post-training quantization: observers record activation / weight ranges on calibration batches;
    convert() bakes the scales (reference quantization/ptq.py)."""

    def quantize(self, model, inplace=False):
        m = self._prepare(model, inplace)
        m.eval()
        return m


import sys as _sys  # noqa: E402
# `from paddle.quantization.quanters import ...` / `.observers import ...` work like the reference packages
_sys.modules[__name__ + ".quanters"] = quanters
_sys.modules[__name__ + ".observers"] = observers
