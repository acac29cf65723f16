"""Gamma(concentration, rate). Reference: python/paddle/distribution/gamma.py."""
from __future__ import annotations

import torch

from ..framework.tensor import _wrap
from .distribution import ExponentialFamily, _bshape, _ft, _t


class Gamma(ExponentialFamily):
    has_rsample = True

    def __init__(self, concentration, rate):
        c, r = _ft(concentration), _ft(rate)
        shape = _bshape(c, r)
        self._conc, self._rate = c.expand(shape), r.to(c.dtype).to(c.device).expand(shape)
        self.concentration, self.rate = _wrap(self._conc), _wrap(self._rate)
        super().__init__(shape)

    @property
    def mean(self):
        return _wrap(self._conc / self._rate)

    @property
    def variance(self):
        return _wrap(self._conc / self._rate.pow(2))

    def rsample(self, shape=()):
        sh = self._extend_shape(shape)
        g = torch._standard_gamma(self._conc.expand(sh))  # implicit-reparameterisation gradient
        return _wrap((g / self._rate).clamp_min(torch.finfo(g.dtype).tiny))

    def log_prob(self, value):
        v = _t(value, self._conc.dtype, self._conc)
        return _wrap(self._conc * torch.log(self._rate) + (self._conc - 1) * torch.log(v) - self._rate * v
                     - torch.lgamma(self._conc))

    def entropy(self):
        c = self._conc
        return _wrap(c - torch.log(self._rate) + torch.lgamma(c) + (1 - c) * torch.digamma(c))

    @property
    def _natural_parameters(self):
        return (self._conc - 1, -self._rate)

    def _log_normalizer(self, x, y):
        return torch.lgamma(x + 1) + (x + 1) * torch.log(-y.reciprocal())

    @property
    def _mean_carrier_measure(self):
        return 0.0
