"""Categorical over the last axis of ``logits``. Reference: python/paddle/distribution/categorical.py —
probs() / log_prob() normalise ``logits`` as non-negative weights (logits / sum), while entropy() and
kl_divergence() use softmax(logits); both behaviours are kept."""
from __future__ import annotations

import numpy as np
import torch

from ..framework.tensor import _wrap
from .distribution import Distribution, _shape, _t


class Categorical(Distribution):
    def __init__(self, logits, name=None):
        lg = _t(logits)
        if not lg.is_floating_point():
            lg = lg.float()
        self._logits = lg
        self.logits = _wrap(lg)
        self._prob = lg / lg.sum(-1, keepdim=True)
        self.name = name or "Categorical"
        super().__init__(tuple(lg.shape[:-1]))

    def sample(self, shape=()):
        shape = list(_shape(shape))
        n = int(np.prod(shape)) if shape else 1
        lg = self._logits.reshape(-1, self._logits.shape[-1])
        p = torch.softmax(lg, -1)
        with torch.no_grad():
            idx = torch.multinomial(p, n, replacement=True)  # [B, n]
        idx = idx.t().reshape(shape + list(self._logits.shape[:-1]))
        return _wrap(idx)

    def probs(self, value):
        v = _t(value).long()
        p = self._prob
        if p.dim() == 1:
            return _wrap(p[v.reshape(-1)].reshape(v.shape))
        if v.dim() == 1:
            idx = v.reshape([1] * (p.dim() - 1) + [-1]).expand(list(p.shape[:-1]) + [v.shape[0]])
            return _wrap(torch.gather(p, -1, idx))
        return _wrap(torch.gather(p, -1, v))

    def prob(self, value):
        return self.probs(value)

    def log_prob(self, value):
        return _wrap(torch.log(self.probs(value)._t))

    def entropy(self):
        lg = self._logits - self._logits.max(-1, keepdim=True).values
        e = lg.exp()
        z = e.sum(-1, keepdim=True)
        p = e / z
        return _wrap(-(p * (lg - torch.log(z))).sum(-1))

    def kl_divergence(self, other):
        a = self._logits - self._logits.max(-1, keepdim=True).values
        b = other._logits - other._logits.max(-1, keepdim=True).values
        za, zb = a.exp().sum(-1, keepdim=True), b.exp().sum(-1, keepdim=True)
        p = a.exp() / za
        return _wrap((p * (a - torch.log(za) - b + torch.log(zb))).sum(-1, keepdim=True))
