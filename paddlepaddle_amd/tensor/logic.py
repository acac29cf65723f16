"""Comparison / logical ops. Reference: python/paddle/tensor/logic.py."""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor, _wrap
from ._helpers import T

_g = globals()


def _make_cmp(name, fn):
    def op(x, y, name=None):
        return _wrap(fn(T(x), T(y)))
    op.__name__ = name
    _g[name] = op

    def op_(x, y, name=None):
        x._t = fn(x._t, T(y)).to(x._t.dtype)
        return x
    _g[name + "_"] = op_


for _n, _f in {"equal": torch.eq, "not_equal": torch.ne, "less_than": torch.lt, "less_equal": torch.le,
               "greater_than": torch.gt, "greater_equal": torch.ge}.items():
    _make_cmp(_n, _f)
less = _g["less_than"]
less_ = _g["less_than_"]
greater = _g["greater_than"]


def equal_all(x, y, name=None):
    a, b = T(x), T(y)
    return _wrap(torch.tensor(a.shape == b.shape and bool(torch.equal(a, b)), device=a.device))


def is_empty(x, name=None):
    return _wrap(torch.tensor(T(x).numel() == 0))


def isin(x, test_x, assume_unique=False, invert=False, name=None):
    return _wrap(torch.isin(T(x), T(test_x), assume_unique=assume_unique, invert=invert))


def is_tensor(x):
    return isinstance(x, Tensor)
