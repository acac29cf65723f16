"""Student's t(df, loc, scale). Reference: python/paddle/distribution/student_t.py."""
from __future__ import annotations

import math

import torch

from ..framework.tensor import _wrap
from .distribution import Distribution, _bshape, _ft, _t


class StudentT(Distribution):
    has_rsample = True

    def __init__(self, df, loc, scale, name=None):
        d, l, s = _ft(df), _ft(loc), _ft(scale)
        shape = _bshape(d, l, s)
        dt = l.dtype
        self._df, self._loc, self._scale = (d.to(dt).expand(shape), l.expand(shape),
                                            s.to(dt).to(l.device).expand(shape))
        self.df, self.loc, self.scale = _wrap(self._df), _wrap(self._loc), _wrap(self._scale)
        self.name = name or "StudentT"
        super().__init__(shape)

    @property
    def mean(self):
        return _wrap(torch.where(self._df > 1, self._loc, torch.full_like(self._loc, float("nan"))))

    @property
    def variance(self):
        d = self._df
        v = self._scale.pow(2) * d / (d - 2)
        v = torch.where(d > 2, v, torch.where(d > 1, torch.full_like(v, float("inf")), torch.full_like(v, float("nan"))))
        return _wrap(v)

    def rsample(self, shape=()):
        sh = self._extend_shape(shape)
        z = torch.randn(sh, dtype=self._loc.dtype, device=self._loc.device)
        g = torch._standard_gamma((0.5 * self._df).expand(sh)) * 2  # chi2(df)
        return _wrap(self._loc + self._scale * z * torch.rsqrt(g / self._df))

    def log_prob(self, value):
        v = _t(value, self._loc.dtype, self._loc)
        d = self._df
        y = (v - self._loc) / self._scale
        return _wrap(torch.lgamma(0.5 * (d + 1)) - torch.lgamma(0.5 * d) - 0.5 * torch.log(d * math.pi)
                     - torch.log(self._scale) - 0.5 * (d + 1) * torch.log1p(y * y / d))

    def entropy(self):
        d = self._df
        lbeta = torch.lgamma(0.5 * d) + math.lgamma(0.5) - torch.lgamma(0.5 * (d + 1))
        return _wrap(torch.log(self._scale) + 0.5 * (d + 1) * (torch.digamma(0.5 * (d + 1)) - torch.digamma(0.5 * d))
                     + 0.5 * torch.log(d) + lbeta)
