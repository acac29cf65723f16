"""Dirichlet(concentration) over the simplex. Reference: python/paddle/distribution/dirichlet.py."""
from __future__ import annotations

import torch

from ..framework.tensor import _wrap
from .distribution import ExponentialFamily, _ft, _t


class Dirichlet(ExponentialFamily):
    has_rsample = True

    def __init__(self, concentration):
        c = _ft(concentration)
        if c.dim() < 1:
            raise ValueError("`concentration` of Dirichlet should have at least one dimension")
        self._c = c
        self.concentration = _wrap(c)
        super().__init__(tuple(c.shape[:-1]), tuple(c.shape[-1:]))

    @property
    def mean(self):
        return _wrap(self._c / self._c.sum(-1, keepdim=True))

    @property
    def variance(self):
        s = self._c.sum(-1, keepdim=True)
        return _wrap(self._c * (s - self._c) / (s.pow(2) * (s + 1)))

    def rsample(self, shape=()):
        sh = self._extend_shape(shape)
        g = torch._standard_gamma(self._c.expand(sh))
        return _wrap(g / g.sum(-1, keepdim=True))

    def log_prob(self, value):
        v = _t(value, self._c.dtype, self._c)
        return _wrap(((self._c - 1) * torch.log(v)).sum(-1) + torch.lgamma(self._c.sum(-1))
                     - torch.lgamma(self._c).sum(-1))

    def entropy(self):
        c = self._c
        k = c.shape[-1]
        s = c.sum(-1)
        return _wrap(torch.lgamma(c).sum(-1) - torch.lgamma(s) + (s - k) * torch.digamma(s)
                     - ((c - 1) * torch.digamma(c)).sum(-1))

    @property
    def _natural_parameters(self):
        return (self._c,)

    def _log_normalizer(self, x):
        return torch.lgamma(x).sum(-1) - torch.lgamma(x.sum(-1))

    @property
    def _mean_carrier_measure(self):
        return 0.0
