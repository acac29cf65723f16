"""MultivariateNormal(loc, covariance | precision | scale_tril). Reference:
python/paddle/distribution/multivariate_normal.py. Everything is evaluated through the Cholesky factor L."""
from __future__ import annotations

import math

import torch

from ..framework.tensor import _wrap
from .distribution import Distribution, _ft, _t


class MultivariateNormal(Distribution):
    has_rsample = True

    def __init__(self, loc, covariance_matrix=None, precision_matrix=None, scale_tril=None):
        l = _ft(loc)
        given = [m is not None for m in (covariance_matrix, precision_matrix, scale_tril)]
        if sum(given) != 1:
            raise ValueError("Exactly one of covariance_matrix or precision_matrix or scale_tril may be specified.")
        if scale_tril is not None:
            L = _ft(scale_tril)
        elif covariance_matrix is not None:
            L = torch.linalg.cholesky(_ft(covariance_matrix))
        else:
            P = _ft(precision_matrix)
            # L = chol(P^-1) through the flipped Cholesky of P (no explicit inverse)
            Lf = torch.linalg.cholesky(torch.flip(P, (-2, -1)))
            Linv = torch.transpose(torch.flip(Lf, (-2, -1)), -2, -1)
            L = torch.linalg.solve_triangular(Linv, torch.eye(P.shape[-1], dtype=P.dtype, device=P.device),
                                              upper=False)
        batch = torch.broadcast_shapes(l.shape[:-1], L.shape[:-2])
        self._loc = l.expand(batch + l.shape[-1:])
        self._L = L.to(l.dtype).expand(batch + L.shape[-2:])
        self.loc = _wrap(self._loc)
        self.scale_tril = _wrap(self._L)
        super().__init__(tuple(batch), tuple(l.shape[-1:]))

    @property
    def covariance_matrix(self):
        return _wrap(self._L @ self._L.transpose(-2, -1))

    @property
    def precision_matrix(self):
        return _wrap(torch.cholesky_inverse(self._L))

    @property
    def mean(self):
        return _wrap(self._loc)

    @property
    def variance(self):
        return _wrap(self._L.pow(2).sum(-1))

    def rsample(self, shape=()):
        sh = self._extend_shape(shape)
        z = torch.randn(sh, dtype=self._loc.dtype, device=self._loc.device)
        return _wrap(self._loc + (self._L @ z.unsqueeze(-1)).squeeze(-1))

    def log_prob(self, value):
        v = _t(value, self._loc.dtype, self._loc)
        diff = v - self._loc
        L = self._L.expand(torch.broadcast_shapes(diff.shape[:-1], self._L.shape[:-2]) + self._L.shape[-2:])
        sol = torch.linalg.solve_triangular(L, diff.expand(L.shape[:-1]).unsqueeze(-1), upper=False).squeeze(-1)
        k = self._loc.shape[-1]
        half_logdet = torch.log(torch.diagonal(self._L, dim1=-2, dim2=-1)).sum(-1)
        return _wrap(-0.5 * (k * math.log(2 * math.pi) + sol.pow(2).sum(-1)) - half_logdet)

    def entropy(self):
        k = self._loc.shape[-1]
        half_logdet = torch.log(torch.diagonal(self._L, dim1=-2, dim2=-1)).sum(-1)
        return _wrap(0.5 * k * (1.0 + math.log(2 * math.pi)) + half_logdet)

    def kl_divergence(self, other):
        from .kl import kl_divergence
        return kl_divergence(self, other)
