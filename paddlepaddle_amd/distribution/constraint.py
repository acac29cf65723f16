"""Support constraints. Reference: python/paddle/distribution/constraint.py."""
from __future__ import annotations

import torch

from ..framework.tensor import _wrap
from .distribution import _t


class Constraint:
    def __call__(self, value):
        raise NotImplementedError


class Real(Constraint):
    def __call__(self, value):
        v = _t(value)
        return _wrap(v == v)


class Range(Constraint):
    def __init__(self, lower, upper):
        self._lower, self._upper = lower, upper

    def __call__(self, value):
        v = _t(value)
        return _wrap((self._lower <= v) & (v <= self._upper))


class Positive(Constraint):
    def __call__(self, value):
        return _wrap(_t(value) >= 0.0)


class Simplex(Constraint):
    def __call__(self, value):
        v = _t(value)
        return _wrap(torch.all(v >= 0, -1) & ((v.sum(-1) - 1).abs() < 1e-6))


real = Real()
positive = Positive()
simplex = Simplex()
