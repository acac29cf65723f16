"""Uniform on [low, high). Reference: python/paddle/distribution/uniform.py."""
from __future__ import annotations

import torch

from ..framework.tensor import _wrap
from .distribution import Distribution, _bshape, _ft, _t


class Uniform(Distribution):
    has_rsample = True

    def __init__(self, low, high, name=None):
        lo, hi = _ft(low), _ft(high)
        dt = torch.float64 if torch.float64 in (lo.dtype, hi.dtype) else lo.dtype
        self._low, self._high = lo.to(dt), hi.to(dt).to(lo.device)
        self.low, self.high = _wrap(self._low), _wrap(self._high)
        self.name = name or "Uniform"
        super().__init__(_bshape(self._low, self._high))

    @property
    def mean(self):
        return _wrap(((self._low + self._high) / 2).expand(self.batch_shape))

    @property
    def variance(self):
        return _wrap(((self._high - self._low) ** 2 / 12).expand(self.batch_shape))

    def rsample(self, shape=()):
        u = torch.rand(self._extend_shape(shape), dtype=self._low.dtype, device=self._low.device)
        return _wrap(self._low + (self._high - self._low) * u)

    def sample(self, shape=(), seed=0):
        return super().sample(shape)

    def log_prob(self, value):
        v = _t(value, self._low.dtype, self._low)
        inside = (v >= self._low) & (v < self._high)
        lp = -torch.log(self._high - self._low)
        return _wrap(torch.where(inside, lp, torch.full_like(lp, float("-inf")) if lp.dim() else
                                 torch.tensor(float("-inf"), dtype=lp.dtype, device=lp.device)))

    def prob(self, value):
        v = _t(value, self._low.dtype, self._low)
        inside = ((v >= self._low) & (v < self._high)).to(self._low.dtype)
        return _wrap(inside / (self._high - self._low))

    def probs(self, value):
        return self.prob(value)

    def entropy(self):
        return _wrap(torch.log(self._high - self._low).expand(self.batch_shape))

    def cdf(self, value):
        v = _t(value, self._low.dtype, self._low)
        return _wrap(((v - self._low) / (self._high - self._low)).clamp(0, 1))

    def icdf(self, value):
        v = _t(value, self._low.dtype, self._low)
        return _wrap(self._low + v * (self._high - self._low))
