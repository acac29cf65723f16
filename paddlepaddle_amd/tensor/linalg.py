"""paddle.linalg. Reference: python/paddle/tensor/linalg.py, python/paddle/linalg.py.
Dense factorizations run on rocSOLVER through ATen's HIP backend."""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor, _wrap
from ._helpers import T, axis_arg
from .math import matmul, bmm, dot, mv, cross, inverse as inv  # noqa: F401


def norm(x, p=None, axis=None, keepdim=False, name=None):
    t = T(x)
    ax = axis_arg(axis)
    if p is None or p == "fro":
        if ax is None:
            return _wrap(torch.linalg.vector_norm(t.flatten(), 2) if t.dim() != 2 or p is None
                         else torch.linalg.matrix_norm(t, "fro", keepdim=keepdim))
        if isinstance(ax, tuple) and len(ax) == 2:
            return _wrap(torch.linalg.matrix_norm(t, "fro", dim=ax, keepdim=keepdim))
        return _wrap(torch.linalg.vector_norm(t, 2, dim=ax, keepdim=keepdim))
    if p == "nuc":
        return _wrap(torch.linalg.matrix_norm(t, "nuc", dim=ax or (-2, -1), keepdim=keepdim))
    if isinstance(ax, tuple) and len(ax) == 2:
        return _wrap(torch.linalg.matrix_norm(t, p, dim=ax, keepdim=keepdim))
    if ax is None:
        t = t.flatten()
    return _wrap(torch.linalg.vector_norm(t, float(p), dim=ax, keepdim=keepdim))


def vector_norm(x, p=2.0, axis=None, keepdim=False, name=None):
    return _wrap(torch.linalg.vector_norm(T(x), p, dim=axis_arg(axis), keepdim=keepdim))


def matrix_norm(x, p="fro", axis=[-2, -1], keepdim=False, name=None):
    return _wrap(torch.linalg.matrix_norm(T(x), p, dim=tuple(axis), keepdim=keepdim))


def cond(x, p=None, name=None):
    return _wrap(torch.linalg.cond(T(x), p))


def det(x, name=None):
    return _wrap(torch.linalg.det(T(x)))


def slogdet(x, name=None):
    s, l = torch.linalg.slogdet(T(x))
    return _wrap(torch.stack([s, l]))


def matrix_rank(x, tol=None, hermitian=False, atol=None, rtol=None, name=None):
    # phi's matrix_rank kernel returns int32 (reference docstring: dtype=int32)
    return _wrap(torch.linalg.matrix_rank(T(x), atol=atol if tol is None else tol, rtol=rtol,
                                          hermitian=hermitian).to(torch.int32))


def matrix_power(x, n, name=None):
    return _wrap(torch.linalg.matrix_power(T(x), n))


def matrix_exp(x, name=None):
    return _wrap(torch.linalg.matrix_exp(T(x)))


def cholesky(x, upper=False, name=None):
    return _wrap(torch.linalg.cholesky(T(x), upper=upper))


def cholesky_solve(x, y, upper=False, name=None):
    return _wrap(torch.cholesky_solve(T(x), T(y), upper))


def cholesky_inverse(x, upper=False, name=None):
    return _wrap(torch.cholesky_inverse(T(x), upper))


def qr(x, mode="reduced", name=None):
    q, r = torch.linalg.qr(T(x), mode)
    return (_wrap(r) if mode == "r" else (_wrap(q), _wrap(r)))


def lu(x, pivot=True, get_infos=False, name=None):
    lu_, piv, info = torch.linalg.lu_factor_ex(T(x), pivot=pivot)
    res = (_wrap(lu_), _wrap(piv.to(torch.int32)))
    return res + (_wrap(info.to(torch.int32)),) if get_infos else res


def lu_unpack(x, y, unpack_ludata=True, unpack_pivots=True, name=None):
    p, l, u = torch.lu_unpack(T(x), T(y))
    return _wrap(p), _wrap(l), _wrap(u)


def svd(x, full_matrices=False, name=None):
    u, s, vh = torch.linalg.svd(T(x), full_matrices=full_matrices)
    return _wrap(u), _wrap(s), _wrap(vh)


def svdvals(x, name=None):
    return _wrap(torch.linalg.svdvals(T(x)))


def svd_lowrank(x, q=None, niter=2, M=None, name=None):
    u, s, v = torch.svd_lowrank(T(x), q=q or 6, niter=niter, M=T(M))
    return _wrap(u), _wrap(s), _wrap(v)


def pca_lowrank(x, q=None, center=True, niter=2, name=None):
    u, s, v = torch.pca_lowrank(T(x), q=q, center=center, niter=niter)
    return _wrap(u), _wrap(s), _wrap(v)


def eig(x, name=None):
    w, v = torch.linalg.eig(T(x))
    return _wrap(w), _wrap(v)


def eigvals(x, name=None):
    return _wrap(torch.linalg.eigvals(T(x)))


def eigh(x, UPLO="L", name=None):
    w, v = torch.linalg.eigh(T(x), UPLO)
    return _wrap(w), _wrap(v)


def eigvalsh(x, UPLO="L", name=None):
    return _wrap(torch.linalg.eigvalsh(T(x), UPLO))


def solve(x, y, left=True, name=None):
    return _wrap(torch.linalg.solve(T(x), T(y), left=left))


def triangular_solve(x, y, upper=True, transpose=False, unitriangular=False, name=None):
    a = T(x)
    if transpose:
        a = a.transpose(-1, -2)
        upper = not upper
    return _wrap(torch.linalg.solve_triangular(a, T(y), upper=upper, unitriangular=unitriangular))


def lstsq(x, y, rcond=None, driver=None, name=None):
    r = torch.linalg.lstsq(T(x), T(y), rcond=rcond, driver=driver)
    return _wrap(r.solution), _wrap(r.residuals), _wrap(r.rank.to(torch.int32)), _wrap(r.singular_values)


def pinv(x, rcond=1e-15, hermitian=False, name=None):
    return _wrap(torch.linalg.pinv(T(x), rtol=rcond, hermitian=hermitian))


def multi_dot(x, name=None):
    return _wrap(torch.linalg.multi_dot([T(v) for v in x]))


def householder_product(x, tau, name=None):
    return _wrap(torch.linalg.householder_product(T(x), T(tau)))


def corrcoef(x, rowvar=True, name=None):
    t = T(x)
    return _wrap(torch.corrcoef(t if rowvar else t.T))


def cov(x, rowvar=True, ddof=True, fweights=None, aweights=None, name=None):
    t = T(x)
    return _wrap(torch.cov(t if rowvar else t.T, correction=1 if ddof else 0,
                           fweights=T(fweights), aweights=T(aweights)))


def ormqr(x, tau, y, left=True, transpose=False, name=None):
    return _wrap(torch.ormqr(T(x), T(tau), T(y), left, transpose))


def vecdot(x, y, axis=-1, name=None):
    return _wrap(torch.linalg.vecdot(T(x), T(y), dim=axis))


def histogramdd(*a, **k):
    from .math import histogramdd as h
    return h(*a, **k)
