"""Shape / layout / indexing manipulation ops. Reference: python/paddle/tensor/manipulation.py."""
from __future__ import annotations

import numpy as _np
np = _np
import torch

from ..framework.tensor import Tensor, _wrap
from ._helpers import T, TT, axis_arg, dtype_arg, shape_arg


def _reshape_shape(t, shape):
    shape = list(shape_arg(shape))
    for i, s in enumerate(shape):
        if s == 0 and i < t.dim():
            shape[i] = t.shape[i]
    return shape


def reshape(x, shape, name=None):
    t = T(x)
    return _wrap(t.reshape(_reshape_shape(t, shape)))


def reshape_(x, shape, name=None):
    x._t = x._t.reshape(_reshape_shape(x._t, shape))
    return x


def view(x, shape_or_dtype, name=None):
    t = T(x)
    if isinstance(shape_or_dtype, (list, tuple, Tensor)):
        return _wrap(t.view(_reshape_shape(t, shape_or_dtype)))
    return _wrap(t.view(dtype_arg(shape_or_dtype)))


def view_as(x, other, name=None):
    return _wrap(T(x).view_as(T(other)))


def flatten(x, start_axis=0, stop_axis=-1, name=None):
    t = T(x)
    if t.dim() == 0:
        return _wrap(t.reshape(1))
    return _wrap(torch.flatten(t, start_axis, stop_axis))


def flatten_(x, start_axis=0, stop_axis=-1, name=None):
    x._t = flatten(x, start_axis, stop_axis)._t
    return x


def unflatten(x, axis, shape, name=None):
    return _wrap(torch.unflatten(T(x), axis, shape_arg(shape)))


def squeeze(x, axis=None, name=None):
    t = T(x)
    ax = axis_arg(axis)
    if ax is None:
        return _wrap(t.squeeze())
    if isinstance(ax, int):
        ax = (ax,)
    ax = tuple(a for a in ax if t.dim() > 0 and t.shape[a] == 1)
    return _wrap(t.squeeze(ax) if ax else t)


def squeeze_(x, axis=None, name=None):
    x._t = squeeze(x, axis)._t
    return x


def unsqueeze(x, axis, name=None):
    t = T(x)
    ax = axis_arg(axis)
    if isinstance(ax, int):
        return _wrap(t.unsqueeze(ax))
    for a in ax:
        t = t.unsqueeze(a)
    return _wrap(t)


def unsqueeze_(x, axis, name=None):
    x._t = unsqueeze(x, axis)._t
    return x


def transpose(x, perm, name=None):
    return _wrap(T(x).permute(*[int(p) for p in perm]))


def transpose_(x, perm, name=None):
    x._t = x._t.permute(*perm).contiguous()
    return x


def t(input, name=None):
    tt = T(input)
    return _wrap(tt.t() if tt.dim() == 2 else tt)


def t_(input, name=None):
    input._t = t(input)._t
    return input


def matrix_transpose(x, name=None):
    return _wrap(T(x).transpose(-1, -2))


def moveaxis(x, source, destination, name=None):
    return _wrap(torch.movedim(T(x), source, destination))


def swapaxes(x, axis0, axis1, name=None):
    return _wrap(torch.swapaxes(T(x), axis0, axis1))


swapdims = swapaxes


def concat(x, axis=0, name=None):
    if isinstance(axis, Tensor):
        axis = int(axis._t.item())
    ts = [T(v) for v in x]
    if len(ts) > 1:
        d = ts[0].dtype
        for v in ts[1:]:
            d = torch.promote_types(d, v.dtype)
        ts = [v.to(d) for v in ts]
    return _wrap(torch.cat(ts, axis))


def stack(x, axis=0, name=None):
    return _wrap(torch.stack([T(v) for v in x], axis))


def hstack(x, name=None):
    return _wrap(torch.hstack([T(v) for v in x]))


def vstack(x, name=None):
    return _wrap(torch.vstack([T(v) for v in x]))


row_stack = vstack


def dstack(x, name=None):
    return _wrap(torch.dstack([T(v) for v in x]))


def column_stack(x, name=None):
    return _wrap(torch.column_stack([T(v) for v in x]))


def split(x, num_or_sections, axis=0, name=None):
    t = T(x)
    if isinstance(axis, Tensor):
        axis = int(axis._t.item())
    n = t.shape[axis]
    if isinstance(num_or_sections, int):
        if n % num_or_sections != 0:
            raise ValueError(f"split: dim {n} is not divisible by {num_or_sections}")
        sizes = [n // num_or_sections] * num_or_sections
    else:
        sizes = [int(s._t.item()) if isinstance(s, Tensor) else int(s) for s in num_or_sections]
        if -1 in sizes:
            known = sum(s for s in sizes if s != -1)
            sizes[sizes.index(-1)] = n - known
    return [_wrap(v) for v in torch.split(t, sizes, axis)]


def tensor_split(x, num_or_indices, axis=0, name=None):
    return [_wrap(v) for v in torch.tensor_split(T(x), num_or_indices, axis)]


def hsplit(x, num_or_indices, name=None):
    return [_wrap(v) for v in torch.hsplit(T(x), num_or_indices)]


def vsplit(x, num_or_indices, name=None):
    return [_wrap(v) for v in torch.vsplit(T(x), num_or_indices)]


def dsplit(x, num_or_indices, name=None):
    return [_wrap(v) for v in torch.dsplit(T(x), num_or_indices)]


def chunk(x, chunks, axis=0, name=None):
    return split(x, chunks, axis)


def unbind(input, axis=0):
    return [_wrap(v) for v in torch.unbind(T(input), axis)]


def unstack(x, axis=0, num=None):
    return unbind(x, axis)


def tile(x, repeat_times, name=None):
    return _wrap(T(x).repeat(*shape_arg(repeat_times)) if len(shape_arg(repeat_times)) >= T(x).dim()
                 else torch.tile(T(x), shape_arg(repeat_times)))


def expand(x, shape, name=None):
    return _wrap(T(x).expand(*shape_arg(shape)))


def expand_as(x, y, name=None):
    return _wrap(T(x).expand_as(T(y)))


def broadcast_to(x, shape, name=None):
    return _wrap(T(x).broadcast_to(shape_arg(shape)))


def broadcast_tensors(input, name=None):
    return [_wrap(v) for v in torch.broadcast_tensors(*[T(v) for v in input])]


def flip(x, axis, name=None):
    ax = axis_arg(axis)
    if isinstance(ax, int):
        ax = (ax,)
    return _wrap(torch.flip(T(x), ax))


reverse = flip


def roll(x, shifts, axis=None, name=None):
    s = shape_arg(shifts) if not isinstance(shifts, int) else shifts
    return _wrap(torch.roll(T(x), s, axis_arg(axis)))


def rot90(x, k=1, axes=[0, 1], name=None):
    return _wrap(torch.rot90(T(x), k, list(axes)))


def repeat_interleave(x, repeats, axis=None, name=None):
    r = T(repeats) if isinstance(repeats, Tensor) else repeats
    return _wrap(torch.repeat_interleave(T(x), r, axis))


def gather(x, index, axis=None, name=None):
    t = T(x)
    i = T(index)
    if axis is None:
        axis = 0
    if isinstance(axis, Tensor):
        axis = int(axis._t.item())
    if i.dim() == 0:
        return _wrap(t.select(axis, int(i.item())))
    return _wrap(torch.index_select(t, axis, i.reshape(-1).long()))


def gather_nd(x, index, name=None):
    t = T(x)
    i = T(index).long()
    k = i.shape[-1]
    idx = tuple(i[..., j] for j in range(k))
    return _wrap(t[idx])


def index_select(x, index, axis=0, name=None):
    return _wrap(torch.index_select(T(x), axis, T(index).reshape(-1).long()))


def index_sample(x, index, name=None):
    return _wrap(torch.gather(T(x), 1, T(index).long()))


def index_add(x, index, axis, value, name=None):
    return _wrap(torch.index_add(T(x), axis, T(index).long(), T(value)))


def index_add_(x, index, axis, value, name=None):
    x._t.index_add_(axis, T(index).long(), T(value))
    return x


def index_fill(x, index, axis, value, name=None):
    v = value._t.item() if isinstance(value, Tensor) else value
    return _wrap(torch.index_fill(T(x), axis, T(index).long(), v))


def index_fill_(x, index, axis, value, name=None):
    v = value._t.item() if isinstance(value, Tensor) else value
    x._t.index_fill_(axis, T(index).long(), v)
    return x


def index_put(x, indices, value, accumulate=False, name=None):
    return _wrap(torch.index_put(T(x), tuple(T(i) for i in indices), T(value), accumulate))


def index_put_(x, indices, value, accumulate=False, name=None):
    x._t.index_put_(tuple(T(i) for i in indices), TT(value, x._t), accumulate)
    return x


def take_along_axis(arr, indices, axis, broadcast=True):
    t, i = T(arr), T(indices).long()
    if broadcast:
        shape = list(t.shape)
        shape[axis] = i.shape[axis]
        bshape = list(torch.broadcast_shapes(tuple(i.shape), tuple(shape)))
        i = i.expand(bshape)
        tshape = list(bshape)
        tshape[axis] = t.shape[axis]
        t = t.expand(tshape)
    return _wrap(torch.gather(t, axis, i))


def put_along_axis(arr, indices, values, axis, reduce="assign", include_self=True, broadcast=True):
    t, i = T(arr), T(indices).long()
    v = TT(values, t).to(t.dtype)
    if broadcast and i.dim() == t.dim():
        # paddle broadcasts indices against arr on every axis but `axis` (put_along_axis docstring:
        # indices [[0]] on a [2, 3] arr with axis=0 writes the whole first row)
        shape = [i.shape[d] if d == axis % t.dim() else t.shape[d] for d in range(t.dim())]
        if list(i.shape) != shape:
            i = i.expand(shape)
    if v.dim() == 0 or v.shape != i.shape:
        v = v.expand_as(i) if v.dim() <= i.dim() else v
    if reduce == "assign":
        return _wrap(t.scatter(axis, i, v))
    red = {"add": "sum", "mul": "prod", "multiply": "prod", "mean": "mean", "amax": "amax", "amin": "amin"}[reduce]
    return _wrap(t.scatter_reduce(axis, i, v, red, include_self=include_self))


def put_along_axis_(arr, indices, values, axis, reduce="assign", include_self=True, broadcast=True):
    arr._t.copy_(put_along_axis(arr, indices, values, axis, reduce, include_self, broadcast)._t)
    return arr


def scatter(x, index, updates, overwrite=True, name=None):
    t = T(x)
    i = T(index).reshape(-1).long()
    u = T(updates)
    if overwrite:
        out = t.clone()
        out[i] = u
        return _wrap(out)
    out = t.clone()
    out[i] = 0
    return _wrap(out.index_add(0, i, u))


def scatter_(x, index, updates, overwrite=True, name=None):
    r = scatter(x, index, updates, overwrite)
    x._t.data.copy_(r._t)
    return x


def scatter_nd_add(x, index, updates, name=None):
    t = T(x)
    i = T(index).long()
    k = i.shape[-1]
    idx = tuple(i[..., j].reshape(-1) for j in range(k))
    u = T(updates).reshape((-1,) + tuple(t.shape[k:]))
    return _wrap(t.index_put(idx, u, accumulate=True))


def scatter_nd(index, updates, shape, name=None):
    z = torch.zeros(shape_arg(shape), dtype=T(updates).dtype, device=T(updates).device)
    return scatter_nd_add(_wrap(z), index, updates)


def masked_select(x, mask, name=None):
    return _wrap(torch.masked_select(T(x), T(mask)))


def masked_fill(x, mask, value, name=None):
    v = T(value)
    return _wrap(torch.masked_fill(T(x), T(mask), v))


def masked_fill_(x, mask, value, name=None):
    x._t.masked_fill_(T(mask), T(value))
    return x


def masked_scatter(x, mask, value, name=None):
    return _wrap(torch.masked_scatter(T(x), T(mask), T(value)))


def masked_scatter_(x, mask, value, name=None):
    x._t.masked_scatter_(T(mask), T(value))
    return x


def slice(input, axes, starts, ends):  # noqa: A001
    t = T(input)
    idx = [builtins_slice(None)] * t.dim()
    for a, s, e in zip(axes, starts, ends):
        s = int(s._t.item()) if isinstance(s, Tensor) else int(s)
        e = int(e._t.item()) if isinstance(e, Tensor) else int(e)
        n = t.shape[a]
        s = max(s + n, 0) if s < 0 else min(s, n)
        e = max(e + n, 0) if e < 0 else min(e, n)
        idx[a] = builtins_slice(s, e)
    return _wrap(t[tuple(idx)])


import builtins as _b  # noqa: E402

builtins_slice = _b.slice


def strided_slice(x, axes, starts, ends, strides, name=None):
    t = T(x)
    for a, s, e, st in zip(axes, starts, ends, strides):
        s, e, st = int(s), int(e), int(st)
        n = t.shape[a]
        if st > 0:
            s = max(s + n, 0) if s < 0 else min(s, n)
            e = max(e + n, 0) if e < 0 else min(e, n)
            idx = torch.arange(s, e, st, device=t.device)
        else:
            s = s + n if s < 0 else min(s, n - 1)
            e = e + n if e < -1 or (e < 0 and e != -n - 1) else e
            idx = torch.arange(s, e, st, device=t.device)
            idx = idx[(idx >= 0) & (idx < n)]
        t = t.index_select(a, idx)
    return _wrap(t)


def crop(x, shape=None, offsets=None, name=None):
    t = T(x)
    shape = shape_arg(shape) if shape is not None else t.shape
    offsets = shape_arg(offsets) if offsets is not None else [0] * t.dim()
    idx = tuple(_b.slice(o, o + (s if s != -1 else t.shape[i] - o)) for i, (o, s) in enumerate(zip(offsets, shape)))
    return _wrap(t[idx])


def unique(x, return_index=False, return_inverse=False, return_counts=False, axis=None, dtype="int64", name=None):
    t = T(x)
    out, inv, cnt = torch.unique(t, sorted=True, return_inverse=True, return_counts=True, dim=axis)
    res = [_wrap(out)]
    if return_index:
        flat_inv = inv if axis is None else inv
        src = t.flatten() if axis is None else None
        n = flat_inv.numel()
        perm = torch.arange(n, device=t.device)
        first = torch.full((out.shape[0] if axis is not None else out.numel(),), n, dtype=torch.long, device=t.device)
        first = first.scatter_reduce(0, flat_inv.flatten(), perm, "amin")
        res.append(_wrap(first.to(dtype_arg(dtype))))
    if return_inverse:
        res.append(_wrap(inv.to(dtype_arg(dtype))))
    if return_counts:
        res.append(_wrap(cnt.to(dtype_arg(dtype))))
    return res[0] if len(res) == 1 else tuple(res)


def unique_consecutive(x, return_inverse=False, return_counts=False, axis=None, dtype="int64", name=None):
    out, inv, cnt = torch.unique_consecutive(T(x), return_inverse=True, return_counts=True, dim=axis)
    res = [_wrap(out)]
    if return_inverse:
        res.append(_wrap(inv.to(dtype_arg(dtype))))
    if return_counts:
        res.append(_wrap(cnt.to(dtype_arg(dtype))))
    return res[0] if len(res) == 1 else tuple(res)


def cast(x, dtype):
    return x.astype(dtype)


def cast_(x, dtype):
    x._t = x._t.to(dtype_arg(dtype))
    return x


def shard_index(input, index_num, nshards, shard_id, ignore_value=-1):
    t = T(input)
    size = (index_num + nshards - 1) // nshards
    lo = shard_id * size
    in_shard = (t >= lo) & (t < lo + size)
    return _wrap(torch.where(in_shard, t - lo, torch.full_like(t, ignore_value)))


def unfold(x, axis, size, step, name=None):
    return _wrap(T(x).unfold(axis, size, step))


def as_strided(x, shape, stride, offset=0, name=None):
    return _wrap(torch.as_strided(T(x), shape_arg(shape), tuple(stride), offset))


def select_scatter(x, values, axis, index, name=None):
    return _wrap(torch.select_scatter(T(x), T(values), axis, index))


def slice_scatter(x, value, axes, starts, ends, strides, name=None):
    t = T(x).clone()
    idx = [_b.slice(None)] * t.dim()
    for a, s, e, st in zip(axes, starts, ends, strides):
        idx[a] = _b.slice(s, e, st)
    t[tuple(idx)] = T(value)
    return _wrap(t)


def diagonal_scatter(x, y, offset=0, axis1=0, axis2=1, name=None):
    return _wrap(torch.diagonal_scatter(T(x), T(y), offset, axis1, axis2))


def as_complex(x, name=None):
    return _wrap(torch.view_as_complex(T(x).contiguous()))


def as_real(x, name=None):
    return _wrap(torch.view_as_real(T(x)))


def tolist(x):
    return T(x).tolist()


def fill_(x, value):
    with torch.no_grad():
        x._t.fill_(value._t.item() if isinstance(value, Tensor) else value)
    return x


def zero_(x):
    with torch.no_grad():
        x._t.zero_()
    return x


def fill_diagonal_(x, value, offset=0, wrap=False, name=None):
    with torch.no_grad():
        t = x._t
        if offset == 0:
            t.fill_diagonal_(value, wrap)
        else:
            torch.diagonal(t, offset).fill_(value)
    return x


def fill_diagonal_tensor(x, y, offset=0, dim1=0, dim2=1, name=None):
    return _wrap(torch.diagonal_scatter(T(x), T(y), offset, dim1, dim2))


def fill_diagonal_tensor_(x, y, offset=0, dim1=0, dim2=1, name=None):
    """In-place paddle.Tensor.fill_diagonal_tensor_. Reference: python/paddle/tensor/manipulation.py."""
    with torch.no_grad():
        torch.diagonal(x._t, offset, dim1, dim2).copy_(T(y))
    return x
