"""Gumbel(loc, scale). Reference: python/paddle/distribution/gumbel.py."""
from __future__ import annotations

import math

import torch

from ..framework.tensor import _wrap
from .distribution import Distribution, _bshape, _ft, _t

_EULER = 0.57721566490153286060


class Gumbel(Distribution):
    has_rsample = True

    def __init__(self, loc, scale):
        l, s = _ft(loc), _ft(scale)
        shape = _bshape(l, s)
        self._loc, self._scale = l.expand(shape), s.to(l.dtype).to(l.device).expand(shape)
        self.loc, self.scale = _wrap(self._loc), _wrap(self._scale)
        super().__init__(shape)

    @property
    def mean(self):
        return _wrap(self._loc + self._scale * _EULER)

    @property
    def variance(self):
        return _wrap(self._scale.pow(2) * math.pi ** 2 / 6)

    @property
    def stddev(self):
        return _wrap(self._scale * math.pi / math.sqrt(6))

    def rsample(self, shape=()):
        tiny = torch.finfo(self._loc.dtype).tiny
        u = torch.rand(self._extend_shape(shape), dtype=self._loc.dtype, device=self._loc.device)
        u = u.clamp(tiny, 1 - torch.finfo(self._loc.dtype).eps)
        return _wrap(self._loc - self._scale * torch.log(-torch.log(u)))

    def log_prob(self, value):
        v = _t(value, self._loc.dtype, self._loc)
        z = (v - self._loc) / self._scale
        return _wrap(-(z + torch.exp(-z)) - torch.log(self._scale))

    def entropy(self):
        return _wrap(torch.log(self._scale) + 1 + _EULER)

    def cdf(self, value):
        v = _t(value, self._loc.dtype, self._loc)
        return _wrap(torch.exp(-torch.exp(-(v - self._loc) / self._scale)))

    def icdf(self, value):
        v = _t(value, self._loc.dtype, self._loc)
        return _wrap(self._loc - self._scale * torch.log(-torch.log(v)))
