"""Tensor creation ops. Reference: python/paddle/tensor/creation.py."""
from __future__ import annotations

import math as _pymath

import numpy as _np
np = _np
import torch

from ..framework import dtype as _dt
from ..framework.place import _get_torch_device, to_torch_device
from ..framework.tensor import Tensor, _wrap, to_tensor  # noqa: F401
from ._helpers import T, TT, dtype_arg, shape_arg


def _dev():
    return _get_torch_device()


def _fdtype(dtype):
    return dtype_arg(dtype) if dtype is not None else _dt.default_dtype().torch_dtype


def zeros(shape, dtype=None, name=None):
    return _wrap(torch.zeros(shape_arg(shape), dtype=_fdtype(dtype), device=_dev()))


def ones(shape, dtype=None, name=None):
    return _wrap(torch.ones(shape_arg(shape), dtype=_fdtype(dtype), device=_dev()))


def empty(shape, dtype=None, name=None):
    return _wrap(torch.empty(shape_arg(shape), dtype=_fdtype(dtype), device=_dev()))


def full(shape, fill_value, dtype=None, name=None):
    fv = fill_value._t.item() if isinstance(fill_value, Tensor) else fill_value
    if dtype is None:
        if isinstance(fv, bool):
            td = torch.bool
        elif isinstance(fv, int):
            td = _dt.default_dtype().torch_dtype
        else:
            td = _dt.default_dtype().torch_dtype
    else:
        td = dtype_arg(dtype)
    return _wrap(torch.full(shape_arg(shape), fv, dtype=td, device=_dev()))


def _like(x, dtype):
    t = T(x)
    return t, (dtype_arg(dtype) if dtype is not None else t.dtype)


def zeros_like(x, dtype=None, name=None):
    t, d = _like(x, dtype)
    return _wrap(torch.zeros_like(t, dtype=d))


def ones_like(x, dtype=None, name=None):
    t, d = _like(x, dtype)
    return _wrap(torch.ones_like(t, dtype=d))


def empty_like(x, dtype=None, name=None):
    t, d = _like(x, dtype)
    return _wrap(torch.empty_like(t, dtype=d))


def full_like(x, fill_value, dtype=None, name=None):
    t, d = _like(x, dtype)
    fv = fill_value._t.item() if isinstance(fill_value, Tensor) else fill_value
    return _wrap(torch.full_like(t, fv, dtype=d))


def arange(start=0, end=None, step=1, dtype=None, name=None):
    s = start._t.item() if isinstance(start, Tensor) else start
    e = end._t.item() if isinstance(end, Tensor) else end
    st = step._t.item() if isinstance(step, Tensor) else step
    if e is None:
        s, e = 0, s
    if dtype is None:
        dtype = "float32" if any(isinstance(v, float) for v in (s, e, st)) else "int64"
    return _wrap(torch.arange(s, e, st, dtype=dtype_arg(dtype), device=_dev()))


def linspace(start, stop, num, dtype=None, name=None):
    s = start._t.item() if isinstance(start, Tensor) else start
    e = stop._t.item() if isinstance(stop, Tensor) else stop
    n = int(num._t.item()) if isinstance(num, Tensor) else int(num)
    return _wrap(torch.linspace(s, e, n, dtype=_fdtype(dtype), device=_dev()))


def logspace(start, stop, num, base=10.0, dtype=None, name=None):
    s = start._t.item() if isinstance(start, Tensor) else start
    e = stop._t.item() if isinstance(stop, Tensor) else stop
    n = int(num._t.item()) if isinstance(num, Tensor) else int(num)
    return _wrap(torch.logspace(s, e, n, base=base, dtype=_fdtype(dtype), device=_dev()))


def eye(num_rows, num_columns=None, dtype=None, name=None):
    nc = num_rows if num_columns is None else num_columns
    return _wrap(torch.eye(int(num_rows), int(nc), dtype=_fdtype(dtype), device=_dev()))


def diag(x, offset=0, padding_value=0, name=None):
    t = T(x)
    if t.dim() == 1 and padding_value != 0:
        n = t.shape[0] + abs(offset)
        out = torch.full((n, n), padding_value, dtype=t.dtype, device=t.device)
        out = out + torch.diag(t, offset) - torch.diag(torch.full_like(t, padding_value), offset)
        return _wrap(out)
    return _wrap(torch.diag(t, offset))


def diagflat(x, offset=0, name=None):
    return _wrap(torch.diagflat(T(x), offset))


def diag_embed(input, offset=0, dim1=-2, dim2=-1):
    return _wrap(torch.diag_embed(T(input), offset, dim1, dim2))


def meshgrid(*args, **kwargs):
    if len(args) == 1 and isinstance(args[0], (list, tuple)):
        args = args[0]
    return [_wrap(t) for t in torch.meshgrid(*[T(a) for a in args], indexing="ij")]


def tril(x, diagonal=0, name=None):
    return _wrap(torch.tril(T(x), diagonal))


def triu(x, diagonal=0, name=None):
    return _wrap(torch.triu(T(x), diagonal))


def tril_(x, diagonal=0, name=None):
    x._t.tril_(diagonal)
    return x


def triu_(x, diagonal=0, name=None):
    x._t.triu_(diagonal)
    return x


def tril_indices(row, col, offset=0, dtype="int64"):
    return _wrap(torch.tril_indices(row, col, offset, dtype=dtype_arg(dtype), device=_dev()))


def triu_indices(row, col=None, offset=0, dtype="int64"):
    col = row if col is None else col
    return _wrap(torch.triu_indices(row, col, offset, dtype=dtype_arg(dtype), device=_dev()))


def assign(x, output=None):
    if isinstance(x, Tensor):
        t = x._t.clone()
    else:
        t = torch.as_tensor(np.asarray(x), device=_dev())
        if t.dtype == torch.float64 and not isinstance(x, np.ndarray):
            t = t.float()
    if output is not None:
        with torch.no_grad():
            if tuple(output._t.shape) != tuple(t.shape) or output._t.dtype != t.dtype:
                # paddle's assign(x, output) gives output x's shape and dtype (the variable is re-bound)
                output._t = t.detach().clone() if output.stop_gradient else t.detach().clone().requires_grad_(True)
            else:
                output._t.copy_(t)
        return output
    return _wrap(t)


def clone(x, name=None):
    return _wrap(T(x).clone())


def complex(real, imag, name=None):
    return _wrap(torch.complex(T(real), T(imag)))


def polar(abs, angle, name=None):
    return _wrap(torch.polar(T(abs), T(angle)))


def cartesian_prod(x, name=None):
    return _wrap(torch.cartesian_prod(*[T(v) for v in x]))


def vander(x, n=None, increasing=False, name=None):
    return _wrap(torch.vander(T(x), N=n, increasing=increasing))


def create_tensor(dtype, name=None, persistable=False):
    t = _wrap(torch.empty(0, dtype=dtype_arg(dtype), device=_dev()))
    t.persistable = persistable
    return t


def fill_constant(shape, dtype, value, force_cpu=False, out=None, name=None):
    r = full(shape, value, dtype)
    if out is not None:
        out._t = r._t
        return out
    return r


def range(start=0, end=None, step=1, dtype=None, name=None):  # noqa: A001
    return arange(start, end, step, dtype)


# ----------------------------------------------------------------------------- tensor arrays
# paddle.tensor.array_*: in dygraph a TensorArray is a plain Python list of Tensors
# (reference: python/paddle/tensor/array.py; the static LOD_TENSOR_ARRAY variable is the graph form).
def create_array(dtype, initialized_list=None):
    arr = []
    for v in initialized_list or []:
        if not isinstance(v, Tensor):
            raise TypeError("create_array: initialized_list must hold Tensors")
        arr.append(v)
    return arr


def _array_index(i):
    return int(i.item()) if isinstance(i, Tensor) else int(i)


def array_write(x, i, array=None):
    if array is None:
        array = []
    k = _array_index(i)
    if k < len(array):
        array[k] = x
    elif k == len(array):
        array.append(x)
    else:
        raise IndexError(f"array_write: index {k} is past the end of an array of length {len(array)}")
    return array


def array_read(array, i):
    return array[_array_index(i)]


def array_length(array):
    return len(array)  # dygraph: a Python int (reference: python/paddle/tensor/array.py array_length)


def _memcpy(input, place=None, output=None):
    """paddle._memcpy: copy ``input`` to ``place`` (reference: python/paddle/tensor/creation.py _memcpy)."""
    from ..framework.place import to_torch_device
    t = input._t.detach().to(to_torch_device(place) if place is not None else input._t.device, copy=True)
    if output is not None:
        output._t = t
        return output
    return _wrap(t)
