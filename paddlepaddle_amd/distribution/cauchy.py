"""Cauchy(loc, scale). Reference: python/paddle/distribution/cauchy.py."""
from __future__ import annotations

import math

import torch

from ..framework.tensor import _wrap
from .distribution import Distribution, _bshape, _ft, _t


class Cauchy(Distribution):
    has_rsample = True

    def __init__(self, loc, scale, name=None):
        l, s = _ft(loc), _ft(scale)
        shape = _bshape(l, s)
        self._loc, self._scale = l.expand(shape), s.to(l.dtype).to(l.device).expand(shape)
        self.loc, self.scale = _wrap(self._loc), _wrap(self._scale)
        self.name = name or "Cauchy"
        super().__init__(shape)

    @property
    def mean(self):
        raise ValueError("Cauchy distribution has no mean.")

    @property
    def variance(self):
        raise ValueError("Cauchy distribution has no variance.")

    @property
    def stddev(self):
        raise ValueError("Cauchy distribution has no stddev.")

    def rsample(self, shape=()):
        u = torch.rand(self._extend_shape(shape), dtype=self._loc.dtype, device=self._loc.device)
        return _wrap(self._loc + self._scale * torch.tan(math.pi * (u - 0.5)))

    def log_prob(self, value):
        v = _t(value, self._loc.dtype, self._loc)
        z = (v - self._loc) / self._scale
        return _wrap(-math.log(math.pi) - torch.log(self._scale) - torch.log1p(z * z))

    def entropy(self):
        return _wrap(math.log(4 * math.pi) + torch.log(self._scale))

    def cdf(self, value):
        v = _t(value, self._loc.dtype, self._loc)
        return _wrap(torch.atan((v - self._loc) / self._scale) / math.pi + 0.5)

    def icdf(self, value):
        v = _t(value, self._loc.dtype, self._loc)
        return _wrap(self._loc + self._scale * torch.tan(math.pi * (v - 0.5)))

    def kl_divergence(self, other):
        from .kl import kl_divergence
        return kl_divergence(self, other)
