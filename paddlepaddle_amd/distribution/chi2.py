"""Chi-squared = Gamma(df / 2, 1 / 2). Reference: python/paddle/distribution/chi2.py."""
from __future__ import annotations

import torch

from ..framework.tensor import _wrap
from .distribution import _ft
from .gamma import Gamma


class Chi2(Gamma):
    def __init__(self, df):
        d = _ft(df)
        self._df = d
        self.df = _wrap(d)
        super().__init__(0.5 * d, torch.full_like(d, 0.5))
