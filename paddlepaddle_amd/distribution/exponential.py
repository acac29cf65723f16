"""Exponential. Reference: python/paddle/distribution/exponential.py."""
from __future__ import annotations

import torch

from ..framework.tensor import _wrap
from .distribution import ExponentialFamily, _ft, _t


class Exponential(ExponentialFamily):
    has_rsample = True

    def __init__(self, rate):
        self._rate = _ft(rate)
        self.rate = _wrap(self._rate)
        super().__init__(tuple(self._rate.shape))

    @property
    def mean(self):
        return _wrap(self._rate.reciprocal())

    @property
    def variance(self):
        return _wrap(self._rate.pow(-2))

    def rsample(self, shape=()):
        u = torch.rand(self._extend_shape(shape), dtype=self._rate.dtype, device=self._rate.device)
        u = u.clamp_min(torch.finfo(u.dtype).tiny)
        return _wrap(-torch.log(u) / self._rate)

    def log_prob(self, value):
        v = _t(value, self._rate.dtype, self._rate)
        lp = torch.log(self._rate) - self._rate * v
        return _wrap(torch.where(v >= 0, lp, torch.full_like(lp, float("-inf"))))

    def entropy(self):
        return _wrap(1.0 - torch.log(self._rate))

    def cdf(self, value):
        v = _t(value, self._rate.dtype, self._rate)
        return _wrap(-torch.expm1(-self._rate * v))

    def icdf(self, value):
        v = _t(value, self._rate.dtype, self._rate)
        return _wrap(-torch.log1p(-v) / self._rate)

    @property
    def _natural_parameters(self):
        return (-self._rate,)

    def _log_normalizer(self, x):
        return -torch.log(-x)

    @property
    def _mean_carrier_measure(self):
        return 0.0
