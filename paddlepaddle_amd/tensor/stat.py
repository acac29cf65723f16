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


def _median_impl(x, axis, keepdim, mode, ignore_nan):
    """Shared body of median / nanmedian. Reference: python/paddle/tensor/stat.py median, nanmedian.

    ``axis``: None (all elements), an int, or a list/tuple of ints (those axes are reduced together).
    mode 'avg': mean of the two middle values when the (valid) count is even; 'min': the lower one, and with
    an int axis also its index. median propagates NaN (a slice holding one is NaN); nanmedian skips NaNs
    (an all-NaN slice is NaN)."""
    t = T(x)
    nd = t.dim()
    if axis is None:
        axes = list(range(nd))
    elif isinstance(axis, (list, tuple)):
        axes = sorted(a % max(nd, 1) for a in axis)
    else:
        axes = [axis % max(nd, 1)]
    keep = [d for d in range(nd) if d not in axes]
    work = t.permute(*keep, *axes).reshape(*[t.shape[d] for d in keep], -1) if nd else t.reshape(1)
    if not (work.is_floating_point()):
        work_f = work.to(torch.float32 if mode == "avg" else work.dtype)
    else:
        work_f = work
    s, idx = torch.sort(work_f, dim=-1, stable=True)  # NaN sorts last
    n = work.shape[-1]
    if work_f.is_floating_point():
        isnan = torch.isnan(work_f)
        nvalid = (~isnan).sum(-1, keepdim=True) if ignore_nan else torch.full_like(s[..., :1], n, dtype=torch.int64)
        anynan = isnan.any(-1, keepdim=True)
    else:
        nvalid = torch.full(s.shape[:-1] + (1,), n, dtype=torch.int64, device=s.device)
        anynan = None
    lo = ((nvalid - 1).clamp(min=0)) // 2
    hi = nvalid // 2
    v_lo = torch.gather(s, -1, lo)
    if mode == "avg":
        v = (v_lo + torch.gather(s, -1, hi.clamp(max=n - 1))) / 2 if n else v_lo
        out_dtype = torch.float64 if t.dtype == torch.float64 else (t.dtype if t.is_floating_point() else torch.float32)
        v = v.to(out_dtype)
        i = None
    else:
        v = v_lo
        i = torch.gather(idx, -1, lo)
    nan_mask = None
    if anynan is not None:
        nan_mask = (nvalid == 0) if ignore_nan else anynan
        if bool(nan_mask.any()):
            v = torch.where(nan_mask, torch.full_like(v, float("nan")), v)
            if i is not None and not ignore_nan:
                first_nan = torch.argmax(isnan.to(torch.int8), -1, keepdim=True)
                i = torch.where(nan_mask, first_nan, i)
    v = v.squeeze(-1)
    if i is not None:
        i = i.squeeze(-1)
    if keepdim:
        shape = [1 if d in axes else t.shape[d] for d in range(nd)]
        v = v.reshape(shape)
        if i is not None:
            i = i.reshape(shape)
    if mode == "min" and axis is not None and not isinstance(axis, (list, tuple)):
        return _wrap(v), _wrap(i)
    return _wrap(v)


def median(x, axis=None, keepdim=False, mode="avg", name=None):
    """paddle.median (NaN-propagating). Reference: python/paddle/tensor/stat.py median."""
    return _median_impl(x, axis, keepdim, mode, ignore_nan=False)


def nanmedian(x, axis=None, keepdim=False, mode="avg", name=None):
    """paddle.nanmedian (NaN-skipping). Reference: python/paddle/tensor/stat.py nanmedian."""
    return _median_impl(x, axis, keepdim, mode, ignore_nan=True)


def _quantile_impl(fn, x, q, axis, keepdim, interpolation):
    t = T(x)
    scalar_q = not isinstance(q, (list, tuple)) and not (isinstance(q, Tensor) and q._t.dim() > 0)
    qq = torch.as_tensor(q._t if isinstance(q, Tensor) else q, dtype=t.dtype, device=t.device)
    if isinstance(axis, (list, tuple)):
        nd = t.dim()
        axes = sorted(a % nd for a in axis)
        keep = [d for d in range(nd) if d not in axes]
        w = t.permute(*keep, *axes).reshape(*[t.shape[d] for d in keep], -1)
        r = fn(w, qq, dim=-1, keepdim=True, interpolation=interpolation)
        if keepdim:
            shape = ([r.shape[0]] if not scalar_q else []) + [1 if d in axes else t.shape[d] for d in range(nd)]
            r = r.reshape(shape)
        else:
            r = r.squeeze(-1)
        return _wrap(r)
    return _wrap(fn(t, qq, dim=axis, keepdim=keepdim, interpolation=interpolation))


def quantile(x, q, axis=None, keepdim=False, interpolation="linear", name=None):
    """paddle.quantile; ``axis`` may be a list of axes. Reference: python/paddle/tensor/stat.py quantile."""
    return _quantile_impl(torch.quantile, x, q, axis, keepdim, interpolation)


def nanquantile(x, q, axis=None, keepdim=False, interpolation="linear", name=None):
    """paddle.nanquantile; ``axis`` may be a list of axes. Reference: python/paddle/tensor/stat.py nanquantile."""
    return _quantile_impl(torch.nanquantile, x, q, axis, keepdim, interpolation)


def numel(x, name=None):
    return _wrap(torch.tensor(T(x).numel(), dtype=torch.int64))
