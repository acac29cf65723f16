"""Beta(alpha, beta) on (0, 1). Reference: python/paddle/distribution/beta.py."""
from __future__ import annotations

import torch

from ..framework.tensor import _wrap
from .distribution import ExponentialFamily, _bshape, _ft, _t


class Beta(ExponentialFamily):
    has_rsample = True

    def __init__(self, alpha, beta):
        a, b = _ft(alpha), _ft(beta)
        shape = _bshape(a, b)
        self._a, self._b = a.expand(shape), b.to(a.dtype).to(a.device).expand(shape)
        self.alpha, self.beta = _wrap(self._a), _wrap(self._b)
        super().__init__(shape)

    @property
    def mean(self):
        return _wrap(self._a / (self._a + self._b))

    @property
    def variance(self):
        s = self._a + self._b
        return _wrap(self._a * self._b / (s.pow(2) * (s + 1)))

    def rsample(self, shape=()):
        sh = self._extend_shape(shape)
        x = torch._standard_gamma(self._a.expand(sh))
        y = torch._standard_gamma(self._b.expand(sh))
        return _wrap(x / (x + y))

    def _lbeta(self):
        return torch.lgamma(self._a) + torch.lgamma(self._b) - torch.lgamma(self._a + self._b)

    def log_prob(self, value):
        v = _t(value, self._a.dtype, self._a)
        return _wrap((self._a - 1) * torch.log(v) + (self._b - 1) * torch.log1p(-v) - self._lbeta())

    def entropy(self):
        a, b = self._a, self._b
        s = a + b
        return _wrap(self._lbeta() - (a - 1) * torch.digamma(a) - (b - 1) * torch.digamma(b)
                     + (s - 2) * torch.digamma(s))

    @property
    def _natural_parameters(self):
        return (self._a, self._b)

    def _log_normalizer(self, x, y):
        return torch.lgamma(x) + torch.lgamma(y) - torch.lgamma(x + y)

    @property
    def _mean_carrier_measure(self):
        return 0.0
