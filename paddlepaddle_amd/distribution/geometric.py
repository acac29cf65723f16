"""Geometric(probs): number of failures before the first success, support {0, 1, 2, ...}.
Reference: python/paddle/distribution/geometric.py (its entropy / kl_divergence formulas are kept)."""
from __future__ import annotations

import numbers

import torch

from ..framework.tensor import Tensor, _wrap
from .distribution import Distribution, _ft, _t


class Geometric(Distribution):
    has_rsample = True

    def __init__(self, probs):
        p = _ft(probs)
        self._p = p
        self.probs = _wrap(p)
        super().__init__(tuple(p.shape))

    @property
    def mean(self):
        return _wrap(1.0 / self._p - 1.0)

    @property
    def variance(self):
        return _wrap((1.0 / self._p - 1.0) / self._p)

    def _k(self, k):
        if not isinstance(k, (numbers.Integral, Tensor, torch.Tensor)):
            raise TypeError(f"Expected type of k is number.Real|Tensor, but got {type(k)}")
        return _t(k, self._p.dtype, self._p)

    def pmf(self, k):
        kk = self._k(k)
        return _wrap(torch.pow(1.0 - self._p, kk) * self._p)

    def log_pmf(self, k):
        kk = self._k(k)
        return _wrap(kk * torch.log1p(-self._p) + torch.log(self._p))

    def log_prob(self, value):
        return self.log_pmf(value if not isinstance(value, float) else torch.tensor(value))

    def prob(self, value):
        return self.pmf(value if not isinstance(value, float) else torch.tensor(value))

    def rsample(self, shape=()):
        tiny = torch.finfo(self._p.dtype).tiny
        u = torch.rand(self._extend_shape(shape), dtype=self._p.dtype, device=self._p.device).clamp(tiny, 1)
        return _wrap(torch.floor(torch.log(u) / torch.log1p(-self._p)))

    def entropy(self):
        p = self._p
        return _wrap(-((1.0 - p) * torch.log(1.0 - p) + p * torch.log(p)) / p)

    def cdf(self, k):
        kk = self._k(k)
        return _wrap(1.0 - torch.pow(1.0 - self._p, kk + 1))

    def kl_divergence(self, other):
        if not isinstance(other, Geometric):
            raise TypeError(f"Exacted type of other is geometric.Geometric, but got {type(other)}")
        p, q = self._p, other._p
        return _wrap(p * torch.log(p / q) + (1.0 - p) * torch.log((1.0 - p) / (1.0 - q)))
