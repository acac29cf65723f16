"""Statistics. Reference: python/paddle/tensor/stat.py."""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor, _wrap
from ._helpers import T, axis_arg


def std(x, axis=None, unbiased=True, keepdim=False, name=None):
    ax = axis_arg(axis)
    t = T(x)
    return _wrap(torch.std(t, dim=ax, correction=1 if unbiased else 0, keepdim=keepdim))


def var(x, axis=None, unbiased=True, keepdim=False, name=None):
    ax = axis_arg(axis)
    return _wrap(torch.var(T(x), dim=ax, correction=1 if unbiased else 0, keepdim=keepdim))


def median(x, axis=None, keepdim=False, mode="avg", name=None):
    t = T(x)
    if axis is None:
        t = t.flatten()
        ax = 0
    else:
        ax = axis
    if mode == "min":
        v, i = torch.median(t, ax, keepdim)
        return (_wrap(v), _wrap(i)) if axis is not None else _wrap(v)
    n = t.shape[ax]
    s = torch.sort(t, ax).values
    if n % 2 == 1:
        r = s.narrow(ax, n // 2, 1)
    else:
        r = (s.narrow(ax, n // 2 - 1, 1) + s.narrow(ax, n // 2, 1)) / 2
    if not keepdim or axis is None:
        r = r.squeeze(ax)
    if keepdim and axis is None:
        r = r.reshape([1] * T(x).dim())
    return _wrap(r)


def nanmedian(x, axis=None, keepdim=False, mode="avg", name=None):
    t = T(x)
    if axis is None:
        return _wrap(torch.nanmedian(t))
    v, i = torch.nanmedian(t, axis, keepdim)
    return _wrap(v)


def quantile(x, q, axis=None, keepdim=False, interpolation="linear", name=None):
    t = T(x)
    qq = torch.as_tensor(q, dtype=t.dtype, device=t.device)
    return _wrap(torch.quantile(t, qq, dim=axis, keepdim=keepdim, interpolation=interpolation))


def nanquantile(x, q, axis=None, keepdim=False, interpolation="linear", name=None):
    t = T(x)
    qq = torch.as_tensor(q, dtype=t.dtype, device=t.device)
    return _wrap(torch.nanquantile(t, qq, dim=axis, keepdim=keepdim, interpolation=interpolation))


def numel(x, name=None):
    return _wrap(torch.tensor(T(x).numel(), dtype=torch.int64))
