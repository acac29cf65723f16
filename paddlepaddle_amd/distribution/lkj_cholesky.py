"""LKJ distribution over Cholesky factors of correlation matrices (Lewandowski, Kurowicka, Joe 2009).
Reference: python/paddle/distribution/lkj_cholesky.py (onion and C-vine samplers)."""
from __future__ import annotations

import math

import numpy as np
import torch

from ..framework.tensor import _wrap
from .distribution import Distribution, _ft, _shape, _t


def _mvlgamma(a, p):
    j = torch.arange(p, dtype=a.dtype, device=a.device)
    return p * (p - 1) / 4 * math.log(math.pi) + torch.lgamma(a.unsqueeze(-1) - j / 2).sum(-1)


class LKJCholesky(Distribution):
    def __init__(self, dim=2, concentration=1.0, sample_method="onion"):
        if dim < 2:
            raise ValueError(f"Expected dim to be an integer greater than or equal to 2. Found dim={dim}.")
        self.dim = dim
        c = _ft(concentration)
        self._c = c
        self.concentration = _wrap(c)
        self.sample_method = sample_method
        super().__init__(tuple(c.shape), (dim, dim))
        # beta parameters of the onion method, per row i = 1..dim-1
        marg = c + 0.5 * (dim - 2)
        offset = torch.arange(dim - 1, dtype=c.dtype, device=c.device)
        self._b1 = 0.5 * (offset + 1)
        self._b0 = marg.unsqueeze(-1) - 0.5 * offset

    def _onion(self, sh):
        d = self.dim
        from .beta import Beta
        y = Beta(self._b1.expand(sh + (d - 1,)), self._b0.expand(sh + (d - 1,))).sample()._t.unsqueeze(-1)
        u = torch.randn(sh + (d, d), dtype=self._c.dtype, device=self._c.device).tril(-1)
        u_hyper = u / u.norm(dim=-1, keepdim=True).clamp_min(torch.finfo(u.dtype).tiny)
        u_hyper[..., 0, :].fill_(0.0)
        w = torch.sqrt(y) * u_hyper[..., 1:, :]
        w = torch.cat([torch.zeros_like(w[..., :1, :]), w], -2)
        diag = torch.sqrt((1 - w.pow(2).sum(-1)).clamp_min(torch.finfo(u.dtype).tiny))
        return w + torch.diag_embed(diag)

    def _cvine(self, sh):
        d = self.dim
        from .beta import Beta
        conc = self._c.expand(sh)
        # partial correlations: Beta(eta + (d - 1 - k) / 2, same) rescaled to (-1, 1)
        rows = []
        L = torch.zeros(sh + (d, d), dtype=self._c.dtype, device=self._c.device)
        L[..., 0, 0] = 1.0
        for i in range(1, d):
            z = torch.ones(sh, dtype=self._c.dtype, device=self._c.device)
            for j in range(i):
                a = conc + 0.5 * (d - 1 - j - 1)
                r = 2 * Beta(a, a).sample()._t - 1
                L[..., i, j] = r * torch.sqrt(z)
                z = z * (1 - r * r)
            L[..., i, i] = torch.sqrt(z)
        return L

    def sample(self, shape=()):
        sh = tuple(_shape(shape)) + self.batch_shape
        with torch.no_grad():
            out = self._onion(sh) if self.sample_method == "onion" else self._cvine(sh)
        return _wrap(out)

    def log_prob(self, value):
        L = _t(value, self._c.dtype, self._c)
        d = self.dim
        diag = torch.diagonal(L, dim1=-2, dim2=-1)[..., 1:]
        order = torch.arange(2, d + 1, dtype=self._c.dtype, device=self._c.device)
        powers = 2 * (self._c.unsqueeze(-1) - 1) + d - order
        unnorm = (powers * torch.log(diag)).sum(-1)
        dm1 = d - 1
        alpha = self._c + 0.5 * dm1
        log_norm = 0.5 * dm1 * math.log(math.pi) + _mvlgamma(alpha - 0.5, dm1) - dm1 * torch.lgamma(alpha)
        return _wrap(unnorm - log_norm)
