"""paddle.sparse — COO / CSR tensors and ops. Reference: python/paddle/sparse/ (creation.py, unary.py,
binary.py, multiary.py, nn/).

Sparse tensors are device sparse buffers (COO: indices [ndim_sparse, nnz] + values; CSR: crows /
cols / values). Elementwise unary ops apply to the stored values only (zeros stay zeros); SpMM and
SDDMM (masked_matmul) run on the device sparse library; sparse convolutions densify the active sites,
convolve, and re-sparsify (submanifold convs keep the input's active set)."""
from __future__ import annotations

import torch
import torch.nn.functional as TF

from ..framework import dtype as _dt
from ..framework.tensor import Tensor, _wrap
from ..framework.place import to_torch_device


def _t(x):
    return x._t if isinstance(x, Tensor) else torch.as_tensor(x)


# ------------------------------------------------------------------------------ creation
def sparse_coo_tensor(indices, values, shape=None, dtype=None, place=None, stop_gradient=True):
    i = _t(indices).long()
    v = _t(values)
    if dtype is not None:
        v = v.to(_dt.to_torch_dtype(dtype))
    if shape is None:
        shape = [int(m) + 1 for m in i.max(1).values.tolist()] + list(v.shape[1:])
    t = torch.sparse_coo_tensor(i, v, tuple(shape))
    if place is not None:
        t = t.to(to_torch_device(place))
    if not stop_gradient:
        t = t.requires_grad_(True)
    return _wrap(t)


def sparse_csr_tensor(crows, cols, values, shape, dtype=None, place=None, stop_gradient=True):
    v = _t(values)
    if dtype is not None:
        v = v.to(_dt.to_torch_dtype(dtype))
    t = torch.sparse_csr_tensor(_t(crows).long(), _t(cols).long(), v, tuple(shape))
    if place is not None:
        t = t.to(to_torch_device(place))
    if not stop_gradient:
        t = t.requires_grad_(True)
    return _wrap(t)


# ------------------------------------------------------------------------------ Tensor methods
def _to_dense(self):
    return _wrap(self._t.to_dense()) if self._t.layout != torch.strided else self


def _to_sparse_coo(self, sparse_dim=None):
    t = self._t
    if t.layout == torch.sparse_coo:
        return self
    if t.layout == torch.sparse_csr:
        return _wrap(t.to_sparse_coo())
    return _wrap(t.to_sparse(sparse_dim) if sparse_dim is not None else t.to_sparse())


def _to_sparse_csr(self):
    t = self._t
    if t.layout == torch.sparse_csr:
        return self
    return _wrap(t.to_sparse_csr() if t.layout == torch.strided else t.to_dense().to_sparse_csr())


def _indices(self):
    return _wrap(self._t.coalesce().indices() if not self._t.is_coalesced() else self._t.indices())


def _values(self):
    t = self._t
    if t.layout == torch.sparse_coo:
        return _wrap(t.coalesce().values() if not t.is_coalesced() else t.values())
    return _wrap(t.values())


Tensor.to_dense = _to_dense
Tensor.to_sparse_coo = _to_sparse_coo
Tensor.to_sparse_csr = _to_sparse_csr
Tensor.indices = _indices
Tensor.values = _values
Tensor.crows = lambda self: _wrap(self._t.crow_indices())
Tensor.cols = lambda self: _wrap(self._t.col_indices())
Tensor.is_sparse = lambda self: self._t.layout in (torch.sparse_coo, torch.sparse_csr)
Tensor.is_sparse_coo = lambda self: self._t.layout == torch.sparse_coo
Tensor.is_sparse_csr = lambda self: self._t.layout == torch.sparse_csr
Tensor.nnz = lambda self: self._t._nnz()


# ------------------------------------------------------------------------------ unary (on values)
def _map_values(x, fn):
    t = x._t
    if t.layout == torch.sparse_coo:
        c = t.coalesce()
        return _wrap(torch.sparse_coo_tensor(c.indices(), fn(c.values()), c.shape))
    if t.layout == torch.sparse_csr:
        return _wrap(torch.sparse_csr_tensor(t.crow_indices(), t.col_indices(), fn(t.values()), t.shape))
    return _wrap(fn(t))


def _unary(fn):
    return lambda x, name=None: _map_values(x, fn)


sin = _unary(torch.sin)
tan = _unary(torch.tan)
asin = _unary(torch.asin)
atan = _unary(torch.atan)
sinh = _unary(torch.sinh)
tanh = _unary(torch.tanh)
asinh = _unary(torch.asinh)
atanh = _unary(torch.atanh)
sqrt = _unary(torch.sqrt)
square = _unary(torch.square)
log1p = _unary(torch.log1p)
abs = _unary(torch.abs)  # noqa: A001
neg = _unary(torch.neg)
expm1 = _unary(torch.expm1)
deg2rad = _unary(torch.deg2rad)
rad2deg = _unary(torch.rad2deg)
isnan = _unary(torch.isnan)
relu = _unary(torch.relu)


def pow(x, factor, name=None):  # noqa: A001
    return _map_values(x, lambda v: v.pow(factor))


def cast(x, index_dtype=None, value_dtype=None, name=None):
    t = x._t
    vd = _dt.to_torch_dtype(value_dtype) if value_dtype is not None else None
    idt = _dt.to_torch_dtype(index_dtype) if index_dtype is not None else None
    if t.layout == torch.sparse_coo:
        c = t.coalesce()
        i = c.indices() if idt is None else c.indices().to(idt)
        v = c.values() if vd is None else c.values().to(vd)
        return _wrap(torch.sparse_coo_tensor(i.long(), v, c.shape))
    v = t.values() if vd is None else t.values().to(vd)
    return _wrap(torch.sparse_csr_tensor(t.crow_indices(), t.col_indices(), v, t.shape))


def coalesce(x, name=None):
    return _wrap(x._t.coalesce())


def is_same_shape(x, y):
    return list(x.shape) == list(y.shape)


# ------------------------------------------------------------------------------ binary
def add(x, y, name=None):
    return _wrap(x._t + y._t)


def subtract(x, y, name=None):
    return _wrap(x._t - y._t)


def multiply(x, y, name=None):
    a, b = x._t, y._t
    if a.layout == torch.sparse_csr:
        a = a.to_sparse_coo()
    if b.layout == torch.sparse_csr:
        b = b.to_sparse_coo()
    out = a * b
    return _wrap(out.to_sparse_csr() if x._t.layout == torch.sparse_csr else out)


def divide(x, y, name=None):
    if isinstance(y, (int, float)):
        return _map_values(x, lambda v: v / y)
    return _wrap((x._t.to_dense() / y._t.to_dense()).to_sparse())


def matmul(x, y, name=None):
    """sparse @ dense -> dense; sparse @ sparse -> sparse."""
    return _wrap(torch.sparse.mm(x._t, y._t) if x._t.layout != torch.strided else torch.matmul(x._t, y._t))


def mv(x, vec, name=None):
    return _wrap(torch.mv(x._t, vec._t) if x._t.layout != torch.sparse_csr else (x._t @ vec._t[:, None])[:, 0])


def masked_matmul(x, y, mask, name=None):
    """SDDMM: (x @ y) evaluated only at mask's nonzeros."""
    m = mask._t
    mc = m.to_sparse_coo().coalesce() if m.layout == torch.sparse_csr else m.coalesce()
    r, c = mc.indices()
    vals = (x._t[r] * y._t.t()[c]).sum(-1)
    out = torch.sparse_coo_tensor(mc.indices(), vals, mc.shape)
    return _wrap(out.to_sparse_csr() if m.layout == torch.sparse_csr else out)


def addmm(input, x, y, beta=1.0, alpha=1.0, name=None):
    prod = torch.sparse.mm(x._t, y._t) if x._t.layout != torch.strided else x._t @ y._t
    inp = input._t
    if inp.layout != torch.strided and prod.layout == torch.strided:
        inp = inp.to_dense()
    return _wrap(beta * inp + alpha * prod)


def mask_as(x, mask, name=None):
    m = mask._t
    mc = m.to_sparse_coo().coalesce() if m.layout == torch.sparse_csr else m.coalesce()
    vals = x._t[tuple(mc.indices())]
    out = torch.sparse_coo_tensor(mc.indices(), vals, mc.shape)
    return _wrap(out.to_sparse_csr() if m.layout == torch.sparse_csr else out)


# ------------------------------------------------------------------------------ shape / reduce
def transpose(x, perm, name=None):
    t = x._t
    is_csr = t.layout == torch.sparse_csr
    c = (t.to_sparse_coo() if is_csr else t).coalesce()
    out = torch.sparse_coo_tensor(c.indices()[list(perm)], c.values(), tuple(c.shape[p] for p in perm)).coalesce()
    return _wrap(out.to_sparse_csr() if is_csr else out)


def reshape(x, shape, name=None):
    t = x._t
    is_csr = t.layout == torch.sparse_csr
    d = t.to_dense().reshape(shape)
    return _wrap(d.to_sparse_csr() if is_csr else d.to_sparse())


def sum(x, axis=None, dtype=None, keepdim=False, name=None):  # noqa: A001
    t = x._t
    if axis is None:
        s = torch.sparse.sum(t.to_sparse_coo() if t.layout == torch.sparse_csr else t)
        return _wrap(s.to(_dt.to_torch_dtype(dtype)) if dtype is not None else s)
    s = torch.sparse.sum(t.to_sparse_coo() if t.layout == torch.sparse_csr else t, dim=axis)
    if s.layout != torch.strided and keepdim:
        s = s.to_dense().unsqueeze(axis).to_sparse()
    return _wrap(s)


def slice(x, axes, starts, ends, name=None):  # noqa: A001
    import builtins
    d = x._t.to_dense()
    idx = [builtins.slice(None)] * d.dim()
    for a, s, e in zip(axes, starts, ends):
        idx[a] = builtins.slice(s, e)
    out = d[tuple(idx)]
    return _wrap(out.to_sparse_csr() if x._t.layout == torch.sparse_csr else out.to_sparse())


def pca_lowrank(x, q=None, center=True, niter=2, name=None):
    U, S, V = torch.pca_lowrank(x._t.to_dense() if x._t.layout != torch.strided else x._t, q=q, center=center,
                                niter=niter)
    return _wrap(U), _wrap(S), _wrap(V)


from . import nn  # noqa: E402,F401
