"""paddle.sparse — COO / CSR tensors and ops. Reference: python/paddle/sparse/ (creation.py, unary.py,
binary.py, multiary.py, nn/).

Sparse tensors are device index / value buffers (COO: indices [ndim_sparse, nnz] + values; CSR: crows /
cols / values); every op is this package's own sort / search / gather / scatter algorithm on them (see
_core.py): coalescing, union / intersection arithmetic, SpMM, SpGEMM, SDDMM, reductions, reshapes, slices
and rulebook (gather-GEMM-scatter) convolutions — nothing is densified. Elementwise unary ops apply to the
stored values only (zeros stay zeros)."""
from __future__ import annotations

import torch
import torch.nn.functional as TF

from ..framework import dtype as _dt
from ..framework.tensor import Tensor, _wrap
from ..framework.place import to_torch_device


def _t(x):
    return x._t if isinstance(x, Tensor) else torch.as_tensor(x)


from . import _core as K


# ------------------------------------------------------------------------------ creation
def sparse_coo_tensor(indices, values, shape=None, dtype=None, place=None, stop_gradient=True):
    i = _t(indices).long()
    v = _t(values)
    if dtype is not None:
        v = v.to(_dt.to_torch_dtype(dtype))
    elif not v.is_floating_point() and v.dtype not in (torch.int32, torch.int64, torch.bool) \
            and not isinstance(values, Tensor):
        v = v.float()
    if shape is None:
        shape = [int(m) + 1 for m in i.max(1).values.tolist()] + list(v.shape[1:])
    if place is not None:
        i, v = i.to(to_torch_device(place)), v.to(to_torch_device(place))
    ci, cv = K.coalesce(i, v, tuple(shape[:i.shape[0]]))
    t = K.make_coo(ci, cv, shape)
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
    t = self._t
    if t.layout == torch.sparse_coo:
        return _wrap(K.coo_to_dense(t))
    if t.layout == torch.sparse_csr:
        return _wrap(K.coo_to_dense(K.csr_to_coo(t)))
    return self


def _to_sparse_coo(self, sparse_dim=None):
    t = self._t
    if t.layout == torch.sparse_coo:
        return self
    if t.layout == torch.sparse_csr:
        return _wrap(K.csr_to_coo(t))
    return _wrap(K.dense_to_coo(t, sparse_dim))


def _to_sparse_csr(self):
    t = self._t
    if t.layout == torch.sparse_csr:
        return self
    return _wrap(K.coo_to_csr(K.to_coo(t)))


def _indices(self):
    return _wrap(K.coo_parts(self._t)[0])


def _values(self):
    t = self._t
    if t.layout == torch.sparse_coo:
        return _wrap(K.coo_parts(t)[1])
    return _wrap(t.values())


def _fmt(a):
    import numpy as np
    return np.array2string(a, separator=", ", prefix="       ")


def _sparse_repr(self):
    t = self._t
    dt = "paddle." + self.dtype.name
    head = (f"Tensor(shape={list(t.shape)}, dtype={dt}, place={self.place}, "
            f"stop_gradient={self.stop_gradient},\n")
    pad = "       "
    if t.layout == torch.sparse_coo:
        i, v, _, _ = K.coo_parts(t)
        ind = _fmt(i.cpu().numpy()).replace("\n", "\n" + " " * 8)
        return head + f"{pad}indices={ind},\n{pad}values={_fmt(_np(v))})"
    return (head + f"{pad}crows={_fmt(t.crow_indices().cpu().numpy())},\n{pad}cols={_fmt(t.col_indices().cpu().numpy())},"
            f"\n{pad}values={_fmt(_np(t.values()))})")


def _np(v):
    v = v.detach().cpu()
    return v.float().numpy() if v.dtype == torch.bfloat16 else v.numpy()


_dense_repr = Tensor.__repr__


def _repr(self):
    if self._t.layout in (torch.sparse_coo, torch.sparse_csr):
        return _sparse_repr(self)
    return _dense_repr(self)


Tensor.__repr__ = _repr
Tensor.__str__ = _repr
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
Tensor.nnz = lambda self: int(self._t._nnz())


# ------------------------------------------------------------------------------ unary (on values)
def _map_values(x, fn):
    t = x._t
    if t.layout in (torch.sparse_coo, torch.sparse_csr):
        return _wrap(K.map_values(t, fn))
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
    if t.layout == torch.sparse_coo:
        i, v, shape, _ = K.coo_parts(t)
        return _wrap(K.make_coo(i, v if vd is None else v.to(vd), shape))
    v = t.values() if vd is None else t.values().to(vd)
    return _wrap(torch.sparse_csr_tensor(t.crow_indices(), t.col_indices(), v, t.shape))


def coalesce(x, name=None):
    i, v, shape, _ = K.coo_parts(x._t)
    return _wrap(K.make_coo(i, v, shape))


def is_same_shape(x, y):
    return list(x.shape) == list(y.shape)


# ------------------------------------------------------------------------------ binary
def _sparse(t):
    return t.layout in (torch.sparse_coo, torch.sparse_csr)


def add(x, y, name=None):
    a, b = x._t, y._t
    if _sparse(a) and _sparse(b):
        return _wrap(K.same_layout(K.union(a, b), a))
    return _wrap((a.to_dense() if _sparse(a) else a) + (b.to_dense() if _sparse(b) else b))


def subtract(x, y, name=None):
    a, b = x._t, y._t
    if _sparse(a) and _sparse(b):
        return _wrap(K.same_layout(K.union(a, b, -1.0), a))
    return _wrap((_to_dense(x)._t) - (_to_dense(y)._t))


def multiply(x, y, name=None):
    a, b = x._t, y._t
    if isinstance(y, (int, float)):
        return _map_values(x, lambda v: v * y)
    if _sparse(a) and _sparse(b):
        return _wrap(K.same_layout(K.intersect(a, b, lambda p, q: p * q), a))
    if _sparse(a):  # sparse * dense: the sparse pattern survives
        i, v, shape, _ = K.coo_parts(K.to_coo(a))
        return _wrap(K.same_layout(K.make_coo(i, v * b[tuple(i)], shape), a))
    return _wrap(a * b)


def divide(x, y, name=None):
    if isinstance(y, (int, float)):
        return _map_values(x, lambda v: v / y)
    a, b = x._t, y._t
    if _sparse(a) and _sparse(b):
        # reference semantics: the quotient over every coordinate (0 / 0 gives nan), all entries stored
        q = K.coo_to_dense(K.to_coo(a)) / K.coo_to_dense(K.to_coo(b))
        idx = torch.ones_like(q, dtype=torch.bool).nonzero().t().contiguous()
        return _wrap(K.same_layout(K.make_coo(idx, q[tuple(idx)], q.shape), a))
    return _wrap(_to_dense(x)._t / _to_dense(y)._t)


def matmul(x, y, name=None):
    """sparse @ dense -> dense (row gather / scatter-add); sparse @ sparse -> sparse (SpGEMM)."""
    a, b = x._t, y._t
    if _sparse(a) and _sparse(b):
        return _wrap(K.same_layout(K.spgemm(a, b), a))
    if _sparse(a):
        return _wrap(K.spmm(a, b))
    return _wrap(torch.matmul(a, b))


def mv(x, vec, name=None):
    return _wrap(K.spmm(x._t, vec._t[:, None])[:, 0])


def masked_matmul(x, y, mask, name=None):
    """SDDMM: (x @ y) evaluated only at mask's nonzeros."""
    return _wrap(K.same_layout(K.sddmm(x._t, y._t, mask._t), mask._t))


def addmm(input, x, y, beta=1.0, alpha=1.0, name=None):
    prod = matmul(x, y)._t
    inp = input._t
    if _sparse(inp) and _sparse(prod):
        return _wrap(K.same_layout(K.union(K.map_values(inp, lambda v: v * beta), K.map_values(prod, lambda v: v * alpha)),
                                   inp))
    if _sparse(inp):
        inp = _to_dense(input)._t
    if _sparse(prod):
        prod = K.coo_to_dense(K.to_coo(prod))
    return _wrap(beta * inp + alpha * prod)


def mask_as(x, mask, name=None):
    i, _, shape, _ = K.coo_parts(K.to_coo(mask._t))
    return _wrap(K.same_layout(K.make_coo(i, x._t[tuple(i)], shape), mask._t))


# ------------------------------------------------------------------------------ shape / reduce
def transpose(x, perm, name=None):
    return _wrap(K.same_layout(K.permute(x._t, list(perm)), x._t))


def reshape(x, shape, name=None):
    return _wrap(K.same_layout(K.reshape(x._t, list(shape)), x._t))


def sum(x, axis=None, dtype=None, keepdim=False, name=None):  # noqa: A001
    out = K.reduce_sum(x._t, axis, keepdim)
    if dtype is not None:
        out = K.map_values(out, lambda v: v.to(_dt.to_torch_dtype(dtype)))
    if x._t.layout == torch.sparse_csr and out.sparse_dim() in (2, 3) and out.dense_dim() == 0:
        out = K.coo_to_csr(out)
    return _wrap(out)


def slice(x, axes, starts, ends, name=None):  # noqa: A001
    return _wrap(K.same_layout(K.slice_(x._t, list(axes), list(starts), list(ends)), x._t))


def pca_lowrank(x, q=None, center=True, niter=2, name=None):
    d = _to_dense(x)._t if _sparse(x._t) else x._t
    U, S, V = torch.pca_lowrank(d, q=q, center=center, niter=niter)
    return _wrap(U), _wrap(S), _wrap(V)


from . import nn  # noqa: E402,F401
