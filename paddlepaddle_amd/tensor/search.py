"""Search / sort ops. Reference: python/paddle/tensor/search.py."""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor, _wrap
from ._helpers import T, TT, axis_arg, dtype_arg


def argmax(x, axis=None, keepdim=False, dtype="int64", name=None):
    t = T(x)
    if axis is None:
        r = torch.argmax(t.flatten())
        if keepdim:
            r = r.reshape([1] * t.dim())
    else:
        r = torch.argmax(t, int(axis), keepdim)
    return _wrap(r.to(dtype_arg(dtype)))


def argmin(x, axis=None, keepdim=False, dtype="int64", name=None):
    t = T(x)
    if axis is None:
        r = torch.argmin(t.flatten())
        if keepdim:
            r = r.reshape([1] * t.dim())
    else:
        r = torch.argmin(t, int(axis), keepdim)
    return _wrap(r.to(dtype_arg(dtype)))


def argsort(x, axis=-1, descending=False, stable=False, name=None):
    return _wrap(torch.argsort(T(x), dim=axis, descending=descending, stable=stable))


def sort(x, axis=-1, descending=False, stable=False, name=None):
    return _wrap(torch.sort(T(x), dim=axis, descending=descending, stable=stable).values)


def topk(x, k, axis=None, largest=True, sorted=True, name=None):
    kk = int(k._t.item()) if isinstance(k, Tensor) else int(k)
    ax = -1 if axis is None else int(axis)
    v, i = torch.topk(T(x), kk, dim=ax, largest=largest, sorted=sorted)
    return _wrap(v), _wrap(i)


def kthvalue(x, k, axis=None, keepdim=False, name=None):
    ax = -1 if axis is None else axis
    v, i = torch.kthvalue(T(x), k, ax, keepdim)
    return _wrap(v), _wrap(i)


def mode(x, axis=-1, keepdim=False, name=None):
    v, i = torch.mode(T(x), axis, keepdim)
    return _wrap(v), _wrap(i)


def where(condition, x=None, y=None, name=None):
    c = T(condition)
    if x is None and y is None:
        return nonzero(condition, as_tuple=True)
    tx, ty = T(x), T(y)
    if not isinstance(tx, torch.Tensor):
        tx = torch.as_tensor(tx, device=c.device, dtype=ty.dtype if isinstance(ty, torch.Tensor) else None)
    if not isinstance(ty, torch.Tensor):
        ty = torch.as_tensor(ty, device=c.device, dtype=tx.dtype)
    return _wrap(torch.where(c, tx, ty))


def where_(condition, x=None, y=None, name=None):
    x._t.copy_(where(condition, x, y)._t)
    return x


def nonzero(x, as_tuple=False):
    t = T(x)
    if as_tuple:
        return tuple(_wrap(v.unsqueeze(-1)) for v in torch.nonzero(t, as_tuple=True))
    return _wrap(torch.nonzero(t))


def searchsorted(sorted_sequence, values, out_int32=False, right=False, name=None):
    return _wrap(torch.searchsorted(T(sorted_sequence), T(values), out_int32=out_int32, right=right))


def bucketize(x, sorted_sequence, out_int32=False, right=False, name=None):
    return _wrap(torch.bucketize(T(x), T(sorted_sequence), out_int32=out_int32, right=right))


def index_of_max(x):
    return argmax(x)


def masked_argmax(x, mask, axis=-1):
    t = T(x).masked_fill(~T(mask), float("-inf"))
    return _wrap(torch.argmax(t, axis))


def top_p_sampling(x, ps, threshold=None, topp_seed=None, seed=-1, k=0, mode="truncated", return_top=False,
                   name=None):
    """Nucleus sampling over probabilities x [B, V] with per-row top-p ``ps`` [B] (reference
    tensor/search.py top_p_sampling): returns (scores [B, 1], ids [B, 1]) and, with return_top, the top-k
    (scores, ids). ``threshold`` drops candidates below a per-row probability; ``k`` > 0 caps the candidate
    count; ``seed`` >= 0 makes the draw reproducible."""
    import torch
    from ..framework.tensor import _wrap
    p = x._t.float()
    pp = ps._t.float().reshape(-1, 1)
    sp, si = p.sort(-1, descending=True)
    keep = (sp.cumsum(-1) - sp) < pp
    keep[:, 0] = True
    if threshold is not None:
        keep &= sp >= threshold._t.float().reshape(-1, 1)
        keep[:, 0] = True
    if k and k > 0:
        keep[:, k:] = False
    w = sp * keep
    g = None
    if seed is not None and seed >= 0:
        g = torch.Generator(device=p.device).manual_seed(int(seed))
    pick = torch.multinomial(w / w.sum(-1, keepdim=True), 1, generator=g)
    ids = si.gather(1, pick)
    scores = p.gather(1, ids).to(x._t.dtype)
    out = (_wrap(scores), _wrap(ids.to(torch.int64)))
    if return_top:
        kk = max(int(k), 1)
        out = out + (_wrap(sp[:, :kk].to(x._t.dtype)), _wrap(si[:, :kk]))
    return out
