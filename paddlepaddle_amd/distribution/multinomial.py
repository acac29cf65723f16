"""Multinomial(total_count, probs). Reference: python/paddle/distribution/multinomial.py (entropy through
the binomial marginals)."""
from __future__ import annotations

import numpy as np
import torch

from ..framework.tensor import _wrap
from .distribution import Distribution, _ft, _shape, _t


class Multinomial(Distribution):
    def __init__(self, total_count, probs):
        if not isinstance(total_count, int) or total_count < 1:
            raise ValueError("input parameter total_count must be int type and greater than 0")
        p = _ft(probs)
        if p.dim() < 1:
            raise ValueError("probs parameter shoule not be none and over one dimension")
        self.total_count = total_count
        self._p = p / p.sum(-1, keepdim=True)
        self.probs = _wrap(self._p)
        super().__init__(tuple(p.shape[:-1]), tuple(p.shape[-1:]))

    @property
    def mean(self):
        return _wrap(self._p * self.total_count)

    @property
    def variance(self):
        return _wrap(self.total_count * self._p * (1 - self._p))

    def prob(self, value):
        return _wrap(self.log_prob(value)._t.exp())

    def log_prob(self, value):
        v = _t(value, self._p.dtype, self._p)
        logits = torch.log(self._p.clamp_min(torch.finfo(self._p.dtype).tiny))
        return _wrap(torch.lgamma(v.sum(-1) + 1) - torch.lgamma(v + 1).sum(-1) + (v * logits).sum(-1))

    def sample(self, shape=()):
        shape = list(_shape(shape))
        n = int(np.prod(shape)) if shape else 1
        k = self._p.shape[-1]
        flat = self._p.reshape(-1, k)
        with torch.no_grad():
            idx = torch.multinomial(flat, self.total_count * n, replacement=True)  # [B, n * total]
            idx = idx.reshape(flat.shape[0], n, self.total_count)
            counts = torch.nn.functional.one_hot(idx, k).sum(-2).to(self._p.dtype)  # [B, n, k]
        counts = counts.permute(1, 0, 2).reshape(shape + list(self._p.shape))
        return _wrap(counts)

    def entropy(self):
        n = self.total_count
        p = self._p
        s = torch.arange(n + 1, dtype=p.dtype, device=p.device).reshape((-1,) + (1,) * p.dim())
        eps = torch.finfo(p.dtype).eps
        pc = p.clamp(eps, 1 - eps)
        log_binom = (torch.lgamma(torch.tensor(n + 1.0, dtype=p.dtype)) - torch.lgamma(n - s + 1) - torch.lgamma(s + 1)
                     + s * torch.log(pc) + (n - s) * torch.log1p(-pc))
        e_lgamma = (log_binom.exp() * torch.lgamma(s + 1)).sum(0)
        return _wrap(-torch.lgamma(torch.tensor(n + 1.0, dtype=p.dtype)) - n * (p * torch.log(pc)).sum(-1)
                     + e_lgamma.sum(-1))
