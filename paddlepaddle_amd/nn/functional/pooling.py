"""Pooling. Reference: python/paddle/nn/functional/pooling.py (MIOpen/ATen pooling kernels on HIP)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ...framework import layout_autotune as _lat
from ...framework.tensor import _wrap
from ...tensor._helpers import T


def _cf(t, data_format):
    nd = t.dim()
    if data_format in ("NHWC", "NLC", "NDHWC"):
        return t.permute(0, nd - 1, *range(1, nd - 1)), True
    return t, False


def _back(t, cl):
    if cl:
        nd = t.dim()
        return t.permute(0, *range(2, nd), 1)
    return t


def _pad_arg(padding, n, data_format=None):
    """Spatial padding as "same", an int / per-dim tuple (symmetric), or ("asym", [before0, after0, ...]).
    Accepts paddle's forms: int, [p] * n, [before0, after0, ...] and the nested per-axis pairs
    ([[0, 0], [0, 0], [ph0, ph1], [pw0, pw1]] NCHW, [[0, 0], [ph0, ph1], [pw0, pw1], [0, 0]] NHWC)."""
    if isinstance(padding, str):
        return 0 if padding.upper() == "VALID" else "same"
    if isinstance(padding, (list, tuple)) and padding and isinstance(padding[0], (list, tuple)):
        cl = data_format in ("NHWC", "NLC", "NDHWC")
        pairs = padding[1:1 + n] if cl else padding[2:2 + n]
        flat = [int(a) for pr in pairs for a in pr]
    elif isinstance(padding, (list, tuple)) and len(padding) == 2 * n:
        flat = [int(a) for a in padding]
    else:
        return padding
    if all(flat[2 * i] == flat[2 * i + 1] for i in range(n)):
        return tuple(flat[2 * i] for i in range(n))
    return ("asym", flat)


def _explicit_pad(t, flat, value):
    """Pad the trailing spatial dims of a channels-first tensor ([before0, after0, before1, ...] in dim order)."""
    n = len(flat) // 2
    spec = []
    for i in reversed(range(n)):
        spec += [flat[2 * i], flat[2 * i + 1]]
    return F.pad(t, spec, value=value)


def _scalar(v):
    """The single value of an int / uniform list (None otherwise). Paddle's nested padding form
    ([[0, 0], [ph, ph], [pw, pw], [0, 0]] for NHWC) is read through its spatial pairs."""
    if isinstance(v, (list, tuple)):
        if any(isinstance(e, (list, tuple)) for e in v):
            if len(v) != 4 or list(v[0]) != [0, 0] or list(v[3]) != [0, 0]:
                return None
            v = [int(a) for pair in v[1:3] for a in pair]
        return v[0] if len(v) and len(set(v)) == 1 else None
    return v


def _maxpool(n, x, kernel_size, stride, padding, return_mask, ceil_mode, data_format):
    if n == 2 and data_format == "NCHW" and not return_mask and _lat.applies(T(x)) \
            and not isinstance(padding, str) and _scalar(padding) is not None:
        y = _maxpool(2, _wrap(_lat.to_nhwc_view(T(x))), kernel_size, stride, padding, False, ceil_mode, "NHWC")
        return _wrap(_lat.to_nchw_view(T(y)))
    if n == 2 and data_format == "NHWC" and not isinstance(padding, str):
        # channels-last HIP kernel (ops/pool.py): first-max mask kept as uint8, gather backward
        from ...ops import pool as _pool
        xt = T(x)
        k, s, p = _scalar(kernel_size), _scalar(stride if stride is not None else kernel_size), _scalar(padding)
        if k is not None and s is not None and p is not None and _pool.maxpool2d_nhwc_supported(
                xt, k, s, p, ceil_mode=ceil_mode, return_mask=return_mask):
            return _wrap(_pool.maxpool2d_nhwc(xt, k, s, p))
    t, cl = _cf(T(x), data_format)
    fn = {1: F.max_pool1d, 2: F.max_pool2d, 3: F.max_pool3d}[n]
    pad = _pad_arg(padding, n, data_format)
    if isinstance(pad, tuple) and pad and pad[0] == "asym":
        t, pad = _explicit_pad(t, pad[1], float("-inf")), 0
    if pad == "same":
        pad = tuple(k // 2 for k in ((kernel_size,) * n if isinstance(kernel_size, int) else kernel_size))
    r = fn(t, kernel_size, stride, pad, 1, ceil_mode, return_mask)
    if return_mask:
        return _wrap(_back(r[0], cl)), _wrap(_back(r[1], cl))
    return _wrap(_back(r, cl))


def max_pool1d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, name=None):
    return _maxpool(1, x, kernel_size, stride, padding, return_mask, ceil_mode, "NCL")


def max_pool2d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, data_format="NCHW",
               name=None):
    return _maxpool(2, x, kernel_size, stride, padding, return_mask, ceil_mode, data_format)


def max_pool3d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, data_format="NCDHW",
               name=None):
    return _maxpool(3, x, kernel_size, stride, padding, return_mask, ceil_mode, data_format)


def _avgpool(n, x, kernel_size, stride, padding, ceil_mode, exclusive, divisor_override, data_format):
    t, cl = _cf(T(x), data_format)
    pad = _pad_arg(padding, n, data_format)
    if isinstance(pad, tuple) and pad and pad[0] == "asym":
        if exclusive:
            # average over the real elements of each window: window sums of the zero-padded input divided by
            # the window counts of a zero-padded ones map (both pooled with the same divisor, which cancels)
            tp = _explicit_pad(t, pad[1], 0.0)
            ones = _explicit_pad(torch.ones_like(t[:, :1]), pad[1], 0.0)
            fn = {1: F.avg_pool1d, 2: F.avg_pool2d, 3: F.avg_pool3d}[n]
            s_ = fn(tp, kernel_size, stride, 0, ceil_mode, True)
            c_ = fn(ones, kernel_size, stride, 0, ceil_mode, True)
            return _wrap(_back(s_ / c_.clamp_min(1e-12), cl))
        t, pad = _explicit_pad(t, pad[1], 0.0), 0
    if pad == "same":
        pad = tuple(k // 2 for k in ((kernel_size,) * n if isinstance(kernel_size, int) else kernel_size))
    if n == 1:
        r = F.avg_pool1d(t, kernel_size, stride, pad, ceil_mode, not exclusive)
    elif n == 2:
        r = F.avg_pool2d(t, kernel_size, stride, pad, ceil_mode, not exclusive, divisor_override)
    else:
        r = F.avg_pool3d(t, kernel_size, stride, pad, ceil_mode, not exclusive, divisor_override)
    return _wrap(_back(r, cl))


def avg_pool1d(x, kernel_size, stride=None, padding=0, exclusive=True, ceil_mode=False, name=None):
    return _avgpool(1, x, kernel_size, stride, padding, ceil_mode, exclusive, None, "NCL")


def avg_pool2d(x, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True, divisor_override=None,
               data_format="NCHW", name=None):
    return _avgpool(2, x, kernel_size, stride, padding, ceil_mode, exclusive, divisor_override, data_format)


def avg_pool3d(x, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True, divisor_override=None,
               data_format="NCDHW", name=None):
    return _avgpool(3, x, kernel_size, stride, padding, ceil_mode, exclusive, divisor_override, data_format)


def adaptive_avg_pool1d(x, output_size, name=None):
    return _wrap(F.adaptive_avg_pool1d(T(x), output_size))


def adaptive_avg_pool2d(x, output_size, data_format="NCHW", name=None):
    t, cl = _cf(T(x), data_format)
    if output_size == 1 or output_size == [1, 1] or output_size == (1, 1):
        r = t.mean((2, 3), keepdim=True)
    else:
        r = F.adaptive_avg_pool2d(t, output_size)
    return _wrap(_back(r, cl))


def adaptive_avg_pool3d(x, output_size, data_format="NCDHW", name=None):
    t, cl = _cf(T(x), data_format)
    return _wrap(_back(F.adaptive_avg_pool3d(t, output_size), cl))


def adaptive_max_pool1d(x, output_size, return_mask=False, name=None):
    r = F.adaptive_max_pool1d(T(x), output_size, return_mask)
    return (_wrap(r[0]), _wrap(r[1])) if return_mask else _wrap(r)


def adaptive_max_pool2d(x, output_size, return_mask=False, name=None):
    r = F.adaptive_max_pool2d(T(x), output_size, return_mask)
    return (_wrap(r[0]), _wrap(r[1])) if return_mask else _wrap(r)


def adaptive_max_pool3d(x, output_size, return_mask=False, name=None):
    r = F.adaptive_max_pool3d(T(x), output_size, return_mask)
    return (_wrap(r[0]), _wrap(r[1])) if return_mask else _wrap(r)


def lp_pool1d(x, norm_type, kernel_size, stride=None, padding=0, ceil_mode=False, data_format="NCL", name=None):
    return _wrap(F.lp_pool1d(T(x), norm_type, kernel_size, stride, ceil_mode))


def lp_pool2d(x, norm_type, kernel_size, stride=None, padding=0, ceil_mode=False, data_format="NCHW", name=None):
    t, cl = _cf(T(x), data_format)
    return _wrap(_back(F.lp_pool2d(t, norm_type, kernel_size, stride, ceil_mode), cl))


def max_unpool1d(x, indices, kernel_size, stride=None, padding=0, data_format="NCL", output_size=None, name=None):
    return _wrap(F.max_unpool1d(T(x), T(indices), kernel_size, stride, padding, output_size))


def max_unpool2d(x, indices, kernel_size, stride=None, padding=0, data_format="NCHW", output_size=None,
                 name=None):
    return _wrap(F.max_unpool2d(T(x), T(indices), kernel_size, stride, padding, output_size))


def max_unpool3d(x, indices, kernel_size, stride=None, padding=0, data_format="NCDHW", output_size=None,
                 name=None):
    return _wrap(F.max_unpool3d(T(x), T(indices), kernel_size, stride, padding, output_size))
