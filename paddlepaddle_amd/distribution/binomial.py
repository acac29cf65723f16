"""Binomial(total_count, probs). Reference: python/paddle/distribution/binomial.py (entropy and KL by
summing over the enumerated support 0..n)."""
from __future__ import annotations

import torch

from ..framework.tensor import _wrap
from .distribution import Distribution, _bshape, _eps, _ft, _t


class Binomial(Distribution):
    def __init__(self, total_count, probs):
        n, p = _t(total_count), _ft(probs)
        shape = _bshape(n, p)
        self.dtype = p.dtype
        self._n = n.to(p.dtype).expand(shape)
        self._p = p.expand(shape)
        self.total_count, self.probs = _wrap(self._n.to(torch.int64) if not _t(total_count).is_floating_point()
                                             else self._n), _wrap(self._p)
        super().__init__(shape)

    @property
    def mean(self):
        return _wrap(self._n * self._p)

    @property
    def variance(self):
        return _wrap(self._n * self._p * (1 - self._p))

    def sample(self, shape=()):
        sh = self._extend_shape(shape)
        with torch.no_grad():
            return _wrap(torch.binomial(self._n.expand(sh).float(), self._p.expand(sh).float()).to(self.dtype))

    def _support(self):
        vals = torch.arange(int(self._n.max().item()) + 1, dtype=self.dtype, device=self._p.device)
        return vals.reshape((-1,) + (1,) * len(self.batch_shape))

    def log_prob(self, value):
        v = _t(value, self.dtype, self._p)
        eps = _eps(self._p)
        p = self._p.clamp(eps, 1 - eps)
        lp = (torch.lgamma(self._n + 1) - torch.lgamma(self._n - v + 1) - torch.lgamma(v + 1)
              + v * torch.log(p) + (self._n - v) * torch.log1p(-p))
        return _wrap(torch.nan_to_num(lp, neginf=-eps))

    def entropy(self):
        lp = self.log_prob(self._support())._t
        return _wrap(-(lp.exp() * lp).sum(0))

    def kl_divergence(self, other):
        s = self._support()
        a, b = self.log_prob(s)._t, other.log_prob(s)._t
        return _wrap((a.exp() * (a - b)).sum(0))
