"""Normal. Reference: python/paddle/distribution/normal.py."""
from __future__ import annotations

import math

import torch

from ..framework.tensor import _wrap
from .distribution import Distribution, _bshape, _ft, _shape, _t


class Normal(Distribution):
    has_rsample = True

    def __init__(self, loc, scale, name=None):
        l, s = _ft(loc), _ft(scale)
        dt = torch.float64 if torch.float64 in (l.dtype, s.dtype) else l.dtype
        self._loc, self._scale = l.to(dt), s.to(dt).to(l.device)
        self.loc, self.scale = _wrap(self._loc), _wrap(self._scale)
        self.name = name or "Normal"
        super().__init__(_bshape(self._loc, self._scale))

    @property
    def mean(self):
        return _wrap(self._loc.expand(self.batch_shape))

    @property
    def variance(self):
        return _wrap(self._scale.pow(2).expand(self.batch_shape))

    def rsample(self, shape=()):
        sh = self._extend_shape(shape)
        z = torch.randn(sh, dtype=self._loc.dtype, device=self._loc.device)
        return _wrap(self._loc + self._scale * z)

    def sample(self, shape=(), seed=0):
        return super().sample(shape)

    def log_prob(self, value):
        v = _t(value, self._loc.dtype, self._loc)
        var = self._scale.pow(2)
        return _wrap(-((v - self._loc) ** 2) / (2 * var) - torch.log(self._scale) - 0.5 * math.log(2 * math.pi))

    def entropy(self):
        return _wrap((0.5 + 0.5 * math.log(2 * math.pi) + torch.log(self._scale)).expand(self.batch_shape))

    def cdf(self, value):
        v = _t(value, self._loc.dtype, self._loc)
        return _wrap(0.5 * (1 + torch.erf((v - self._loc) / (self._scale * math.sqrt(2)))))

    def icdf(self, value):
        v = _t(value, self._loc.dtype, self._loc)
        return _wrap(self._loc + self._scale * math.sqrt(2) * torch.erfinv(2 * v - 1))

    def probs(self, value):
        return self.prob(value)

    def kl_divergence(self, other):
        from .kl import kl_divergence
        return kl_divergence(self, other)
