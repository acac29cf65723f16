"""Laplace(loc, scale). Reference: python/paddle/distribution/laplace.py."""
from __future__ import annotations

import math

import torch

from ..framework.tensor import _wrap
from .distribution import Distribution, _bshape, _ft, _t


class Laplace(Distribution):
    has_rsample = True

    def __init__(self, loc, scale):
        l, s = _ft(loc), _ft(scale)
        shape = _bshape(l, s)
        self._loc, self._scale = l.expand(shape), s.to(l.dtype).to(l.device).expand(shape)
        self.loc, self.scale = _wrap(self._loc), _wrap(self._scale)
        super().__init__(shape)

    @property
    def mean(self):
        return _wrap(self._loc)

    @property
    def variance(self):
        return _wrap(2 * self._scale.pow(2))

    @property
    def stddev(self):
        return _wrap(math.sqrt(2) * self._scale)

    def rsample(self, shape=()):
        sh = self._extend_shape(shape)
        eps = torch.finfo(self._loc.dtype).eps
        u = torch.rand(sh, dtype=self._loc.dtype, device=self._loc.device) * (2 - 2 * eps) - (1 - eps)
        return _wrap(self._loc - self._scale * torch.sign(u) * torch.log1p(-u.abs()))

    def log_prob(self, value):
        v = _t(value, self._loc.dtype, self._loc)
        return _wrap(-torch.log(2 * self._scale) - (v - self._loc).abs() / self._scale)

    def entropy(self):
        return _wrap(1 + torch.log(2 * self._scale))

    def cdf(self, value):
        v = _t(value, self._loc.dtype, self._loc)
        z = (v - self._loc) / self._scale
        return _wrap(0.5 - 0.5 * torch.sign(z) * torch.expm1(-z.abs()))

    def icdf(self, value):
        v = _t(value, self._loc.dtype, self._loc)
        t = v - 0.5
        return _wrap(self._loc - self._scale * torch.sign(t) * torch.log1p(-2 * t.abs()))
