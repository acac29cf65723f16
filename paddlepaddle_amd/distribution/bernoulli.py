"""Bernoulli(probs). Reference: python/paddle/distribution/bernoulli.py."""
from __future__ import annotations

import torch

from ..framework.tensor import _wrap
from .distribution import ExponentialFamily, _eps, _ft, _t


class Bernoulli(ExponentialFamily):
    def __init__(self, probs, name=None):
        p = _ft(probs)
        self._p = p
        self.probs = _wrap(p)
        eps = _eps(p)
        pc = p.clamp(eps, 1 - eps)
        self._logits = torch.log(pc) - torch.log1p(-pc)
        self.logits = _wrap(self._logits)
        self.name = name or "Bernoulli"
        super().__init__(tuple(p.shape))

    @property
    def mean(self):
        return _wrap(self._p)

    @property
    def variance(self):
        return _wrap(self._p * (1 - self._p))

    def sample(self, shape=()):
        sh = self._extend_shape(shape)
        with torch.no_grad():
            return _wrap(torch.bernoulli(self._p.expand(sh)))

    def rsample(self, shape=(), temperature=1.0):
        """Relaxed (logistic-noise) sample in logit space; apply a sigmoid to map it into (0, 1)."""
        sh = self._extend_shape(shape)
        tiny = torch.finfo(self._p.dtype).tiny
        u = torch.rand(sh, dtype=self._p.dtype, device=self._p.device).clamp(tiny, 1 - _eps(self._p))
        return _wrap((self._logits + torch.log(u) - torch.log1p(-u)) / float(temperature))

    def log_prob(self, value):
        v = _t(value, self._p.dtype, self._p)
        return _wrap(-torch.nn.functional.binary_cross_entropy_with_logits(
            self._logits.expand(torch.broadcast_shapes(v.shape, self._logits.shape)),
            v.expand(torch.broadcast_shapes(v.shape, self._logits.shape)), reduction="none"))

    def prob(self, value):
        return _wrap(self.log_prob(value)._t.exp())

    def cdf(self, value):
        v = _t(value, self._p.dtype, self._p)
        out = torch.where(v < 0, torch.zeros_like(v), torch.where(v < 1, (1 - self._p).expand_as(v), torch.ones_like(v)))
        return _wrap(out)

    def entropy(self):
        return _wrap(torch.nn.functional.binary_cross_entropy_with_logits(self._logits, self._p, reduction="none"))

    @property
    def _natural_parameters(self):
        return (self._logits,)

    def _log_normalizer(self, x):
        return torch.nn.functional.softplus(x)

    @property
    def _mean_carrier_measure(self):
        return 0.0
