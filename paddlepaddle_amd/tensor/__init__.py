"""paddle.tensor namespace + Tensor method binding.
Reference: python/paddle/tensor/__init__.py (tensor_method_func list patched onto the eager Tensor)."""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor, _wrap, to_tensor  # noqa: F401
from . import creation, einsum as _einsum_mod, linalg, logic, manipulation, math, random, search, stat  # noqa: F401
from .creation import *  # noqa: F401,F403
from .einsum import einsum  # noqa: F401
from .logic import *  # noqa: F401,F403
from .manipulation import *  # noqa: F401,F403
from .math import *  # noqa: F401,F403
from .random import *  # noqa: F401,F403
from .search import *  # noqa: F401,F403
from .stat import *  # noqa: F401,F403
from ._helpers import T as _T
from . import creation, linalg, logic, manipulation, math, random, search, stat  # noqa: F811,E402

_MODULES = [creation, logic, manipulation, math, random, search, stat, linalg]

_SKIP = {"T", "TT", "to_tensor", "shape_arg", "axis_arg", "dtype_arg", "wrap", "wraps", "scalar", "annotations",
         "is_tensor", "builtins_slice", "create_tensor", "fill_constant", "range", "meshgrid", "arange",
         "zeros", "ones", "empty", "full", "eye", "linspace", "logspace", "rand", "randn", "randint", "randperm",
         "uniform", "normal", "standard_normal", "tril_indices", "triu_indices", "assign", "add_n", "concat",
         "stack", "broadcast_tensors", "multiplex", "cartesian_prod", "hstack", "vstack", "dstack",
         "column_stack", "row_stack", "complex", "polar", "log_normal", "scatter_nd", "broadcast_shape",
         "create_array", "array_write", "array_read", "array_length", "uniform_random_batch_size_like"}

_VARARG_SHAPE = {"reshape", "reshape_", "tile", "expand", "broadcast_to", "view"}


def _bind_methods():
    import inspect
    for mod in _MODULES:
        for name, fn in list(vars(mod).items()):
            if name.startswith("_") or name in _SKIP or not inspect.isfunction(fn):
                continue
            if getattr(fn, "__module__", "").split(".")[-1] not in ("creation", "logic", "manipulation", "math",
                                                                      "random", "search", "stat", "linalg"):
                continue
            if hasattr(Tensor, name) and name not in ("abs",):
                # keep explicit Tensor methods (e.g. astype, clone, detach, to)
                if name in Tensor.__dict__:
                    continue
            if name in _VARARG_SHAPE:
                def _m(self, *shape, _fn=fn, **kw):
                    if len(shape) == 1 and isinstance(shape[0], (list, tuple, Tensor)):
                        return _fn(self, shape[0], **kw)
                    if len(shape) == 0:
                        return _fn(self, **kw)
                    if all(isinstance(s, int) for s in shape):
                        return _fn(self, list(shape), **kw)
                    return _fn(self, *shape, **kw)
                setattr(Tensor, name, _m)
            else:
                setattr(Tensor, name, fn)
    # aliases that differ between function and method names
    Tensor.transpose = lambda self, perm=None, *rest, **k: manipulation.transpose(
        self, list(perm) if rest == () and isinstance(perm, (list, tuple)) else [perm, *rest])
    Tensor.dim = lambda self: self._t.dim()
    Tensor.matmul = math.matmul
    Tensor.norm = linalg.norm
    Tensor.cholesky = linalg.cholesky
    Tensor.inverse = math.inverse
    Tensor.det = linalg.det
    Tensor.fill_ = manipulation.fill_
    Tensor.zero_ = manipulation.zero_
    Tensor.uniform_ = random.uniform_
    Tensor.normal_ = random.normal_
    Tensor.exponential_ = random.exponential_
    Tensor.bernoulli_ = random.bernoulli_
    Tensor.cauchy_ = random.cauchy_
    Tensor.geometric_ = random.geometric_
    Tensor.log_normal_ = random.log_normal_
    Tensor.numel = lambda self: _wrap(torch.tensor(self._t.numel(), dtype=torch.int64))
    Tensor.expand_as = manipulation.expand_as
    Tensor.unbind = manipulation.unbind


def _binop(op, rev=False):
    tm = getattr(torch.Tensor, op)

    def f(self, other):
        o = other._t if isinstance(other, Tensor) else other
        r = tm(self._t, o)
        if r is NotImplemented:
            return r
        return _wrap(r)
    f.__name__ = op
    return f


for _op in ("__add__", "__radd__", "__sub__", "__rsub__", "__mul__", "__rmul__", "__truediv__",
            "__rtruediv__", "__floordiv__", "__rfloordiv__", "__mod__", "__rmod__", "__pow__", "__rpow__",
            "__matmul__", "__rmatmul__", "__and__", "__rand__", "__or__", "__ror__", "__xor__", "__rxor__",
            "__lt__", "__le__", "__gt__", "__ge__", "__eq__", "__ne__", "__lshift__", "__rshift__"):
    setattr(Tensor, _op, _binop(_op))

Tensor.__neg__ = lambda self: _wrap(-self._t)
Tensor.__pos__ = lambda self: self
Tensor.__abs__ = lambda self: _wrap(self._t.abs())
Tensor.__invert__ = lambda self: _wrap(~self._t)
Tensor.__hash__ = lambda self: id(self)


def _matmul_amp(self, other):
    return math.matmul(self, other)


Tensor.__matmul__ = _matmul_amp
Tensor.__rmatmul__ = lambda self, other: math.matmul(other, self)

_bind_methods()


def _bind_reference_extras():
    """Functions the reference also exposes as Tensor methods (tensor_method_func) although they take
    several tensors or none: x.concat([y]) etc. follow the function signatures."""
    import paddlepaddle_amd as _p
    from .. import signal as _signal
    for name in ("create_parameter", "create_tensor", "multiplex", "block_diag", "add_n", "broadcast_shape",
                 "is_tensor", "concat", "scatter_nd", "stack", "rank", "broadcast_tensors", "polar"):
        fn = getattr(_p, name, None)
        if fn is not None and not hasattr(Tensor, name):
            setattr(Tensor, name, fn)
    if not hasattr(Tensor, "top_p_sampling"):
        Tensor.top_p_sampling = search.top_p_sampling
    if not hasattr(Tensor, "stft"):
        Tensor.stft = _signal.stft
        Tensor.istft = _signal.istft

    def set_(self, source=None, shape=None, stride=None, offset=0, name=None):
        """Make this tensor share ``source``'s storage (optionally as a strided view); ``offset`` is in BYTES
        from the start of ``source``'s data (reference: python/paddle/tensor/creation.py set_)."""
        import torch
        if source is None:
            self._t = torch.empty(0, dtype=self._t.dtype, device=self._t.device)
            return self
        src = source._t if isinstance(source, Tensor) else torch.as_tensor(source)
        if shape is not None or offset:
            shp = list(shape) if shape is not None else list(src.shape)
            st = list(stride) if stride is not None else list(torch.empty(shp, device="meta").stride())
            src = src.as_strided(shp, st, src.storage_offset() + offset // src.element_size())
        self._t = src
        return self
    if not hasattr(Tensor, "set_"):
        Tensor.set_ = set_
