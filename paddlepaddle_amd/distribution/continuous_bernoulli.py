"""Continuous Bernoulli(probs) on [0, 1] (Loaiza-Ganem & Cunningham 2019). Reference:
python/paddle/distribution/continuous_bernoulli.py (Taylor expansion of the normaliser inside ``lims``)."""
from __future__ import annotations

import math

import torch

from ..framework.tensor import _wrap
from .distribution import Distribution, _eps, _ft, _t


class ContinuousBernoulli(Distribution):
    has_rsample = True

    def __init__(self, probs, lims=(0.499, 0.501)):
        p = _ft(probs)
        eps = _eps(p)
        self._p = p.clamp(eps, 1 - eps)
        self.probs = _wrap(self._p)
        self._lims = lims
        super().__init__(tuple(p.shape))

    def _outside(self):
        return (self._p <= self._lims[0]) | (self._p >= self._lims[1])

    def _cut(self):
        return torch.where(self._outside(), self._p, torch.full_like(self._p, self._lims[0]))

    def _log_norm(self):
        # log C(p), C(p) = 2 atanh(1 - 2p) / (1 - 2p); near p = 1/2 its Taylor series
        p = self._cut()
        val = torch.log(torch.abs(torch.log1p(-p) - torch.log(p))) - torch.log(torch.abs(1 - 2 * p))
        x = (self._p - 0.5) ** 2
        taylor = math.log(2.0) + (4.0 / 3.0 + 104.0 / 45.0 * x) * x
        return torch.where(self._outside(), val, taylor)

    @property
    def mean(self):
        p = self._cut()
        m = p / (2 * p - 1) + 1 / (torch.log1p(-p) - torch.log(p))
        x = self._p - 0.5
        taylor = 0.5 + (1.0 / 3.0 + 16.0 / 45.0 * x ** 2) * x
        return _wrap(torch.where(self._outside(), m, taylor))

    @property
    def variance(self):
        p = self._cut()
        v = p * (p - 1) / (1 - 2 * p) ** 2 + 1 / (torch.log1p(-p) - torch.log(p)) ** 2
        x = (self._p - 0.5) ** 2
        taylor = 1.0 / 12.0 - (1.0 / 15.0 - 128.0 / 945.0 * x) * x
        return _wrap(torch.where(self._outside(), v, taylor))

    def rsample(self, shape=()):
        u = torch.rand(self._extend_shape(shape), dtype=self._p.dtype, device=self._p.device)
        return self.icdf(_wrap(u))

    def log_prob(self, value):
        v = _t(value, self._p.dtype, self._p)
        return _wrap(v * torch.log(self._p) + (1 - v) * torch.log1p(-self._p) + self._log_norm())

    def prob(self, value):
        return _wrap(self.log_prob(value)._t.exp())

    def cdf(self, value):
        v = _t(value, self._p.dtype, self._p)
        p = self._cut()
        c = (p.pow(v) * (1 - p).pow(1 - v) + p - 1) / (2 * p - 1)
        out = torch.where(self._outside(), c, v)
        return _wrap(torch.where(v <= 0, torch.zeros_like(out), torch.where(v >= 1, torch.ones_like(out), out)))

    def icdf(self, value):
        v = _t(value, self._p.dtype, self._p)
        p = self._cut()
        x = (torch.log1p(-p + v * (2 * p - 1)) - torch.log1p(-p)) / (torch.log(p) - torch.log1p(-p))
        return _wrap(torch.where(self._outside(), x, v))

    def entropy(self):
        p = self._p
        m = self.mean._t
        return _wrap(-(m * torch.log(p) + (1 - m) * torch.log1p(-p)) - self._log_norm())
