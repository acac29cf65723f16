"""LogNormal(loc, scale) = exp(Normal(loc, scale)). Reference: python/paddle/distribution/lognormal.py."""
from __future__ import annotations

import math

import torch

from ..framework.tensor import _wrap
from .normal import Normal
from .transform import ExpTransform
from .transformed_distribution import TransformedDistribution


class LogNormal(TransformedDistribution):
    has_rsample = True

    def __init__(self, loc, scale):
        self._base_normal = Normal(loc, scale)
        self.loc, self.scale = self._base_normal.loc, self._base_normal.scale
        super().__init__(self._base_normal, [ExpTransform()])

    @property
    def mean(self):
        n = self._base_normal
        return _wrap(torch.exp(n._loc + n._scale.pow(2) / 2).expand(self.batch_shape))

    @property
    def variance(self):
        n = self._base_normal
        s2 = n._scale.pow(2)
        return _wrap((torch.expm1(s2) * torch.exp(2 * n._loc + s2)).expand(self.batch_shape))

    def entropy(self):
        return _wrap(self._base_normal.entropy()._t + self._base_normal._loc.expand(self.batch_shape))

    def probs(self, value):
        return self.prob(value)

    def kl_divergence(self, other):
        from .kl import kl_divergence
        return kl_divergence(self, other)
