"""Poisson(rate). Reference: python/paddle/distribution/poisson.py (entropy and KL summed over a
rate + 30 sqrt(rate) bounded support)."""
from __future__ import annotations

import torch

from ..framework.tensor import _wrap
from .distribution import Distribution, _eps, _ft, _t


class Poisson(Distribution):
    def __init__(self, rate):
        r = _ft(rate)
        self._rate = r
        self.rate = _wrap(r)
        self.dtype = r.dtype
        super().__init__(tuple(r.shape))

    @property
    def mean(self):
        return _wrap(self._rate)

    @property
    def variance(self):
        return _wrap(self._rate)

    def sample(self, shape=()):
        sh = self._extend_shape(shape)
        with torch.no_grad():
            return _wrap(torch.poisson(self._rate.expand(sh)))

    def _support(self, rate):
        m = float(rate.max().item())
        s = m ** 0.5 if m >= 1 else 1.0
        upper = int(max(rate.max().item() + 30 * s, 1))
        return torch.arange(0, upper, dtype=self.dtype, device=rate.device)

    def log_prob(self, value):
        v = _t(value, self.dtype, self._rate)
        eps = _eps(self._rate)
        return _wrap(torch.nan_to_num(-self._rate + v * torch.log(self._rate) - torch.lgamma(v + 1), neginf=-eps))

    def entropy(self):
        vals = self._support(self._rate).reshape((-1,) + (1,) * len(self.batch_shape))
        lp = self.log_prob(vals)._t
        ent = -(lp.exp() * lp).sum(0)
        return _wrap(ent * (self._rate != 0).to(self.dtype))

    def kl_divergence(self, other):
        vals = self._support(torch.maximum(self._rate, other._rate)).reshape((-1,) + (1,) * len(self.batch_shape))
        a, b = self.log_prob(vals)._t, other.log_prob(vals)._t
        return _wrap((a.exp() * (a - b)).sum(0))
