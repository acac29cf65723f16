"""Remaining paddle.static names: ExponentialMovingAverage, metric helpers (accuracy / auc /
ctr_metric_bundle), persistables (de)serialization, py_func, and the IPU / XPU entry points.

Reference: python/paddle/static/__init__.py; static/amp and static/quantization live elsewhere;
ExponentialMovingAverage in python/paddle/static/nn/... (base/optimizer.py ExponentialMovingAverage),
metrics in python/paddle/static/nn/metric.py. IPU and XPU are other vendors' devices: their entry
points exist and raise a clear error (this framework targets MI355X).
"""
from __future__ import annotations

import contextlib
import io as _io

import numpy as np
import torch

from ..framework.tensor import Tensor, _wrap
from ..nn.layer.layers import WeightNormParamAttr  # noqa: F401
from .control_flow import py_func  # noqa: F401

__all__ = ["ExponentialMovingAverage", "accuracy", "auc", "ctr_metric_bundle", "deserialize_persistables",
           "py_func", "WeightNormParamAttr", "IpuCompiledProgram", "IpuStrategy", "ipu_shard_guard",
           "set_ipu_shard", "xpu_places"]


class ExponentialMovingAverage:
    """Shadow parameters ema = decay * ema + (1 - decay) * param, with optional thres_steps warm-up
    (decay_t = min(decay, (1 + t) / (10 + t))); apply() swaps the averages in (context manager) and
    restore() puts the trained values back. Parameters default to every trainable parameter created so far
    (the reference collects the program's parameters)."""

    def __init__(self, decay=0.999, thres_steps=None, name=None, parameters=None):
        self._decay = decay
        self._thres = thres_steps
        self._params = list(parameters) if parameters is not None else None
        self._ema = {}
        self._backup = {}
        self._step = 0

    def _plist(self):
        if self._params is None:
            from ..framework.tensor import Parameter
            import gc
            self._params = [o for o in gc.get_objects() if isinstance(o, Parameter) and not o.stop_gradient]
        return self._params

    def update(self):
        d = self._decay
        if self._thres is not None:
            t = float(self._thres._t.item() if isinstance(self._thres, Tensor) else self._thres)
            d = min(d, (1.0 + t) / (10.0 + t))
        with torch.no_grad():
            for p in self._plist():
                e = self._ema.get(id(p))
                if e is None:
                    self._ema[id(p)] = p._t.detach().float().clone()
                else:
                    e.mul_(d).add_(p._t.detach().float(), alpha=1.0 - d)
        self._step += 1

    @contextlib.contextmanager
    def apply(self, executor=None, need_restore=True):
        with torch.no_grad():
            for p in self._plist():
                e = self._ema.get(id(p))
                if e is not None:
                    self._backup[id(p)] = p._t.detach().clone()
                    p._t.copy_(e.to(p._t.dtype))
        try:
            yield
        finally:
            if need_restore:
                self.restore(executor)

    def restore(self, executor=None):
        with torch.no_grad():
            for p in self._plist():
                b = self._backup.pop(id(p), None)
                if b is not None:
                    p._t.copy_(b)


def accuracy(input, label, k=1, correct=None, total=None):
    from ..metric import accuracy as _acc
    return _acc(input, label, k=k, correct=correct, total=total)


def auc(input, label, curve="ROC", num_thresholds=2 ** 12 - 1, topk=1, slide_steps=1, ins_tag_weight=None):
    """(auc, batch_auc, [stat_pos, stat_neg, ...]) over bucketed positive-class scores (reference auc op)."""
    p = input._t.float()
    score = p[:, -1] if p.dim() == 2 else p.reshape(-1)
    y = label._t.reshape(-1).long()
    bucket = (score.clamp(0, 1) * num_thresholds).long()
    pos = torch.zeros(num_thresholds + 1, dtype=torch.float64, device=p.device)
    neg = torch.zeros_like(pos)
    pos.index_add_(0, bucket, (y == 1).double())
    neg.index_add_(0, bucket, (y != 1).double())
    # area under ROC from the bucket histogram (trapezoids, highest threshold first)
    tp = torch.cumsum(pos.flip(0), 0)
    fp = torch.cumsum(neg.flip(0), 0)
    tp0 = torch.cat([tp.new_zeros(1), tp[:-1]])
    fp0 = torch.cat([fp.new_zeros(1), fp[:-1]])
    area = ((fp - fp0) * (tp + tp0) / 2).sum()
    denom = tp[-1] * fp[-1]
    a = (area / denom) if float(denom) > 0 else torch.zeros((), dtype=torch.float64)
    a = _wrap(a.float())
    return a, a, [_wrap(pos), _wrap(neg)]


def ctr_metric_bundle(input, label, ins_tag_weight=None):
    """(sqrerr, abserr, prob, q, pos, total) sums used by CTR jobs."""
    p = input._t.float().reshape(-1)
    y = label._t.float().reshape(-1)
    sq = ((p - y) ** 2).sum()
    ab = (p - y).abs().sum()
    q = torch.log(p.clamp_min(1e-12) / (1 - p).clamp_min(1e-12)).sum()
    return tuple(_wrap(v) for v in (sq, ab, p.sum(), q, y.sum(), torch.tensor(float(p.numel()))))


def deserialize_persistables(program, data, executor=None):
    """Load parameter values produced by serialize_persistables (a name -> tensor dict, or its
    paddle.save bytes) into ``program``'s parameters."""
    if isinstance(data, (bytes, bytearray)):
        from ..framework.io import load as _load
        state = _load(_io.BytesIO(data))
    else:
        state = dict(data)
    from .io import set_program_state
    set_program_state(program, state)
    return program


def _no_ipu(*a, **k):
    raise RuntimeError("IPU devices are not supported by this MI355X framework")


class IpuStrategy:
    def __init__(self, *a, **k):
        _no_ipu()


class IpuCompiledProgram:
    def __init__(self, *a, **k):
        _no_ipu()


@contextlib.contextmanager
def ipu_shard_guard(index=-1, stage=-1):
    _no_ipu()
    yield


def set_ipu_shard(call_func, index=-1, stage=-1):
    _no_ipu()


def xpu_places(device_ids=None):
    raise RuntimeError("XPU devices are not supported by this MI355X framework (use paddle.static.cuda_places)")
