"""paddle.quantization.imperative: the dygraph QAT / PTQ API of PaddleSlim-era models.

Reference: python/paddle/quantization/imperative/qat.py:52 (ImperativeQuantAware), ptq.py:42 (ImperativePTQ),
ptq_config.py (PTQConfig, default_ptq_config), ptq_quantizer.py (Absmax / PerChannelAbsmax / Hist / KL
quantizers), ptq_registry.py, fuse_utils.py (conv + BN folding).

QAT runs on the fake-quant layers of paddle.quantization (QuantedConv2D / QuantedLinear, straight-through
estimator); PTQ records ranges with forward hooks on the quantizable layers and, on save, replaces them by
quant-dequant layers with the calibrated thresholds (KL: minimum Kullback-Leibler divergence between the
activation histogram and its quantised version; Hist: a percentile of |x|)."""
from __future__ import annotations

import copy
import math

import numpy as np
import torch

from ... import nn
from ...framework.tensor import Tensor, _wrap
from .. import (QAT, BaseQuanter, FakeQuanterChannelWiseAbsMaxObserver, FakeQuanterWithAbsMaxObserver,
                QuantConfig, QuantedConv2D, QuantedLinear, _FixedQuant, _STE, _qmax, fake_quant, quanter)
from . import fuse_utils  # noqa: F401

__all__ = ["ImperativeQuantAware", "ImperativePTQ", "PTQConfig", "default_ptq_config", "AbsmaxQuantizer",
           "PerChannelAbsmaxQuantizer", "HistQuantizer", "KLQuantizer", "PTQRegistry"]


# ------------------------------------------------------------------ QAT
class AbsMaxWeightQuanterLayer(BaseQuanter):
    """Per-tensor abs-max fake quant of the current weight every step (weight_quantize_type='abs_max')."""

    def __init__(self, layer=None, bit_length=8):
        super().__init__()
        self._bits = bit_length
        self._scale = None

    def forward(self, x):
        t = x._t
        s = t.detach().abs().max().clamp_min(1e-8)
        self._scale = s
        return _wrap(_STE.apply(t, s, _qmax(self._bits), None))

    def scales(self):
        return None if self._scale is None else _wrap(self._scale)

    def bit_length(self):
        return self._bits


AbsMaxWeightQuanter = quanter("AbsMaxWeightQuanter")(AbsMaxWeightQuanterLayer)

_TYPES = {"Conv2D": nn.Conv2D, "Linear": nn.Linear}


class ImperativeQuantAware:
    def __init__(self, quantizable_layer_type=("Conv2D", "Linear", "Conv2DTranspose"),
                 weight_quantize_type="abs_max", activation_quantize_type="moving_average_abs_max", weight_bits=8,
                 activation_bits=8, moving_rate=0.9, fuse_conv_bn=False, weight_preprocess_layer=None,
                 act_preprocess_layer=None, weight_quantize_layer=None, act_quantize_layer=None, onnx_format=False):
        if weight_quantize_type not in ("abs_max", "channel_wise_abs_max"):
            raise ValueError(f"unsupported weight_quantize_type {weight_quantize_type}")
        if activation_quantize_type not in ("moving_average_abs_max", "abs_max"):
            raise ValueError(f"unsupported activation_quantize_type {activation_quantize_type}")
        self._types = [_TYPES[t] if isinstance(t, str) else t for t in quantizable_layer_type
                       if not isinstance(t, str) or t in _TYPES]
        self._fuse_conv_bn = fuse_conv_bn
        if weight_quantize_layer is not None:
            w = weight_quantize_layer
        elif weight_quantize_type == "abs_max":
            w = AbsMaxWeightQuanter(bit_length=weight_bits)
        else:
            w = FakeQuanterChannelWiseAbsMaxObserver(bit_length=weight_bits, quant_axis=0)
        a = act_quantize_layer if act_quantize_layer is not None else FakeQuanterWithAbsMaxObserver(
            moving_rate=moving_rate if activation_quantize_type == "moving_average_abs_max" else 0.0,
            bit_length=activation_bits)
        self._config = QuantConfig(activation=None, weight=None)
        for t in self._types:
            self._config.add_type_config(t, activation=a, weight=w)
        self._qat = QAT(self._config)

    def quantize(self, model):
        """Replaces the quantizable layers of ``model`` in place by fake-quant layers."""
        if self._fuse_conv_bn:
            fuse_utils.fuse_conv_bn(model)
        model.train()
        return self._qat.quantize(model, inplace=True)

    def save_quantized_model(self, layer, path, input_spec=None, **config):
        from ... import jit
        frozen = self._qat.convert(layer, inplace=False)
        frozen.eval()
        jit.save(frozen, path, input_spec=input_spec, **config)


# ------------------------------------------------------------------ PTQ quantizers
def _abs_max(t):
    return float(t.detach().abs().max()) if t.numel() else 0.0


class BaseQuantizer:
    def __init__(self, quant_bits=8):
        self.quant_bits = quant_bits
        self.abs_max_vals = []
        self.thresholds = []

    def sample_data(self, layer, tensors):
        raise NotImplementedError

    def cal_thresholds(self):
        raise NotImplementedError


class AbsmaxQuantizer(BaseQuantizer):
    def sample_data(self, layer, tensors):
        vals = [_abs_max(t) for t in tensors]
        self.abs_max_vals = vals if not self.abs_max_vals else [max(a, b) for a, b in zip(self.abs_max_vals, vals)]

    def cal_thresholds(self):
        self.thresholds = list(self.abs_max_vals)


class PerChannelAbsmaxQuantizer(BaseQuantizer):
    """Per output channel (conv weights: axis 0, linear weights [in, out]: axis 1)."""

    def sample_data(self, layer, tensors):
        axis = 1 if isinstance(layer, nn.Linear) else 0
        vals = []
        for t in tensors:
            d = t.detach().abs()
            red = [i for i in range(d.dim()) if i != axis]
            vals.append(d.amax(dim=red).float().cpu().numpy() if red else d.float().cpu().numpy())
        self.abs_max_vals = vals if not self.abs_max_vals else [np.maximum(a, b) for a, b in
                                                               zip(self.abs_max_vals, vals)]

    def cal_thresholds(self):
        self.thresholds = list(self.abs_max_vals)


class BaseHistQuantizer(BaseQuantizer):
    """|x| histograms over [0, running max]; a larger batch max re-bins the old counts into the wider range
    (each old bin's count spread uniformly over the part of the new bins it covers)."""

    def __init__(self, quant_bits=8, bins=1024, upsample_bins=64):
        super().__init__(quant_bits)
        self.bins = bins
        self.upsample_bins = upsample_bins
        self.hists = []

    def _hist(self, t, hi):
        a = t.detach().abs().float().reshape(-1).cpu().numpy()
        return np.histogram(a, bins=self.bins, range=(0.0, hi))[0].astype(np.float64)

    def _rebin(self, hist, old_max, new_max):
        edges = np.linspace(0.0, old_max, self.bins + 1)
        new_w = new_max / self.bins
        out = np.zeros(self.bins)
        for i in range(self.bins):
            if hist[i] == 0:
                continue
            lo, hi = edges[i], edges[i + 1]
            j0, j1 = int(lo // new_w), min(self.bins - 1, int(hi // new_w))
            for j in range(j0, j1 + 1):
                ov = min(hi, (j + 1) * new_w) - max(lo, j * new_w)
                if ov > 0:
                    out[j] += hist[i] * ov / (hi - lo)
        return out

    def sample_data(self, layer, tensors):
        if not self.hists:
            self.abs_max_vals = [_abs_max(t) for t in tensors]
            self.hists = [None if m == 0.0 else self._hist(t, m) for t, m in zip(tensors, self.abs_max_vals)]
            return
        for i, t in enumerate(tensors):
            m = _abs_max(t)
            if m == 0.0:
                continue
            old = self.abs_max_vals[i]
            if self.hists[i] is None or old == 0.0:
                self.abs_max_vals[i], self.hists[i] = m, self._hist(t, m)
            elif m <= old:
                self.hists[i] = self.hists[i] + self._hist(t, old)
            else:
                self.hists[i] = self._rebin(self.hists[i], old, m) + self._hist(t, m)
                self.abs_max_vals[i] = m


class HistQuantizer(BaseHistQuantizer):
    def __init__(self, quant_bits=8, bins=1024, upsample_bins=64, hist_percent=0.99999):
        super().__init__(quant_bits, bins, upsample_bins)
        self.hist_percent = hist_percent

    def cal_thresholds(self):
        self.thresholds = []
        for m, h in zip(self.abs_max_vals, self.hists):
            if h is None:
                self.thresholds.append(m)
                continue
            c = np.cumsum(h / h.sum())
            idx = int(np.argmax(c >= self.hist_percent))
            self.thresholds.append((idx + 0.5) * m / self.bins)


def _kl_threshold(hist, bin_width, bits):
    """Threshold minimising KL(P || Q): P = the histogram clipped at bin i (outliers folded into the last bin),
    Q = the clipped histogram quantised to 2^(bits-1) - 1 levels and expanded back over the non-zero bins of
    each level; candidates i run from half the histogram range to its end."""
    levels = 2 ** (bits - 1) - 1
    n = hist.shape[0]
    if n <= levels:
        return n * bin_width
    best, best_i = float("inf"), n
    total = hist.sum()
    # like the reference search (static/quantization/cal_kl_threshold.py), candidates start at half the range
    for i in range(max(levels, (n - 1) // 2), n + 1):
        p = hist[:i].astype(np.float64).copy()
        p[i - 1] += hist[i:].sum()
        nz = p > 0
        # quantise: merge i bins into `levels` groups
        edges = np.linspace(0, i, levels + 1)
        q = np.zeros(i)
        for k in range(levels):
            a, b = int(math.floor(edges[k])), max(int(math.floor(edges[k + 1])), int(math.floor(edges[k])) + 1)
            b = min(b, i)
            seg = hist[a:b]  # the candidate quantisation sees the clipped range only (no outlier mass)
            cnt = np.count_nonzero(seg)
            if cnt:
                q[a:b] = np.where(seg > 0, seg.sum() / cnt, 0.0)
        ps, qs = p / total, q / max(q.sum(), 1e-30)
        m = nz & (qs > 0)
        if not np.all(qs[nz] > 0):
            kl = float("inf")
        else:
            kl = float(np.sum(ps[m] * np.log(ps[m] / qs[m])))
        if kl < best:
            best, best_i = kl, i
    return (best_i + 0.5) * bin_width


class KLQuantizer(BaseHistQuantizer):
    def cal_thresholds(self):
        self.thresholds = []
        for m, h in zip(self.abs_max_vals, self.hists):
            self.thresholds.append(m if h is None else _kl_threshold(h, m / self.bins, self.quant_bits))


SUPPORT_ACT_QUANTIZERS = [AbsmaxQuantizer, HistQuantizer, KLQuantizer]
SUPPORT_WT_QUANTIZERS = [AbsmaxQuantizer, PerChannelAbsmaxQuantizer]


class PTQConfig:
    def __init__(self, activation_quantizer, weight_quantizer):
        if type(activation_quantizer) not in SUPPORT_ACT_QUANTIZERS:
            raise TypeError(f"activation quantizer must be one of {SUPPORT_ACT_QUANTIZERS}")
        if type(weight_quantizer) not in SUPPORT_WT_QUANTIZERS:
            raise TypeError(f"weight quantizer must be one of {SUPPORT_WT_QUANTIZERS}")
        self.in_act_quantizer = copy.deepcopy(activation_quantizer)
        self.out_act_quantizer = copy.deepcopy(activation_quantizer)
        self.wt_quantizer = copy.deepcopy(weight_quantizer)
        self.quant_hook_handle = None
        self.is_skip = False


default_ptq_config = PTQConfig(KLQuantizer(), PerChannelAbsmaxQuantizer())


class PTQRegistry:
    """Quantizable layer types (reference ptq_registry.py): their weight attribute names."""
    _registry = {nn.Conv2D: ["weight"], nn.Linear: ["weight"]}

    @classmethod
    def is_supported_layer(cls, layer):
        return type(layer) in cls._registry or isinstance(layer, tuple(cls._registry))

    @classmethod
    def layer_info(cls, layer):
        return cls._registry.get(type(layer), ["weight"])


class _PTQLinear(nn.Layer):
    def __init__(self, layer, in_scale, w, bits):
        super().__init__()
        self.weight, self.bias = w, layer.bias
        self._in = _FixedQuant(in_scale, bits)

    def forward(self, x):
        return nn.functional.linear(self._in(x), self.weight, self.bias)


class _PTQConv2D(nn.Layer):
    def __init__(self, layer, in_scale, w, bits):
        super().__init__()
        self.weight, self.bias = w, layer.bias
        self._layer = layer
        self._in = _FixedQuant(in_scale, bits)

    def forward(self, x):
        L = self._layer
        return nn.functional.conv2d(self._in(x), self.weight, self.bias, L._stride, L._padding, L._dilation,
                                    L._groups, L._data_format)


class ImperativePTQ:
    def __init__(self, quant_config=default_ptq_config):
        self._cfg = quant_config

    def quantize(self, model, inplace=False, fuse=False, fuse_list=None):
        m = model if inplace else copy.deepcopy(model)
        if fuse:
            fuse_utils.fuse_layers(m, fuse_list, inplace=True) if fuse_list else fuse_utils.fuse_conv_bn(m)
        for _, sub in m.named_sublayers():
            if not PTQRegistry.is_supported_layer(sub):
                continue
            cfg = copy.deepcopy(self._cfg)
            sub._quant_config = cfg

            def hook(layer, inputs, outputs, cfg=cfg):
                ins = tuple(i._t for i in inputs if isinstance(i, Tensor))
                outs = outputs if isinstance(outputs, (list, tuple)) else (outputs,)
                cfg.in_act_quantizer.sample_data(layer, ins)
                cfg.out_act_quantizer.sample_data(layer, tuple(o._t for o in outs if isinstance(o, Tensor)))
            cfg.quant_hook_handle = sub.register_forward_post_hook(hook)
        return m

    def _convert(self, model):
        for name, sub in list(model.named_children()):
            cfg = getattr(sub, "_quant_config", None)
            if cfg is None:
                self._convert(sub)
                continue
            if cfg.quant_hook_handle is not None:
                cfg.quant_hook_handle.remove()
            cfg.in_act_quantizer.cal_thresholds()
            wq = cfg.wt_quantizer
            wq.sample_data(sub, (sub.weight._t,))
            wq.cal_thresholds()
            bits = cfg.wt_quantizer.quant_bits
            thr = wq.thresholds[0]
            w = sub.weight._t.detach()
            if isinstance(thr, np.ndarray):
                axis = 1 if isinstance(sub, nn.Linear) else 0
                shape = [1] * w.dim()
                shape[axis] = -1
                s = torch.as_tensor(thr, dtype=w.dtype, device=w.device).reshape(shape)
            else:
                s = torch.tensor(float(thr), dtype=w.dtype, device=w.device)
            with torch.no_grad():
                sub.weight._t.copy_(fake_quant(w, s.clamp_min(1e-8), bits))
            in_thr = torch.tensor(float(cfg.in_act_quantizer.thresholds[0]) or 1e-8)
            act_bits = cfg.in_act_quantizer.quant_bits
            cls = _PTQLinear if isinstance(sub, nn.Linear) else _PTQConv2D
            model._sub_layers[name] = cls(sub, in_thr, sub.weight, act_bits)
        return model

    def save_quantized_model(self, model, path, input_spec=None, **config):
        from ... import jit
        m = self._convert(model)
        m.eval()
        jit.save(m, path, input_spec=input_spec, **config)
        return m


_ = (QuantedConv2D, QuantedLinear)
