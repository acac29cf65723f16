"""The paddle ``Tensor`` for MI355X.

Reference: paddle/fluid/eager/eager_tensor.h, python/paddle/base/dygraph/tensor_patch_methods.py,
python/paddle/tensor/ (methods patched onto the eager tensor).

Design: a ``Tensor`` is a thin handle over a device buffer owned by the PyTorch-ROCm caching
allocator (``self._t``). Paddle semantics live here (``stop_gradient``, list shapes, places,
names, paddle method signatures); compute dispatches to hand-written HIP kernels (``ops``)
or ATen-on-HIP kernels. Gradient graph traversal uses the native (C++) autograd engine of the
HIP runtime: every op that we implement with a HIP kernel registers its own backward kernel.
"""
from __future__ import annotations

import itertools
import weakref

import numpy as np
import torch

from . import dtype as _dt
from .place import CPUPlace, CUDAPlace, Place, _get_torch_device, place_from_torch_device, to_torch_device

_name_counter = itertools.count()
_PARAM_OF = weakref.WeakValueDictionary()  # id(parameter buffer) -> Parameter (static graph lookups)


def _unwrap(x):
    """Tensor -> torch.Tensor; leave everything else untouched."""
    return x._t if isinstance(x, Tensor) else x


def _unwrap_nested(x):
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, (list, tuple)):
        return type(x)(_unwrap_nested(v) for v in x)
    if isinstance(x, dict):
        return {k: _unwrap_nested(v) for k, v in x.items()}
    return x


def _wrap(t):
    """torch.Tensor -> Tensor (fast path, no copies)."""
    if t is None:
        return None
    obj = object.__new__(Tensor)
    obj._t = t
    obj._name = None
    obj._persistable = False
    return obj


def _wrap_nested(x):
    if isinstance(x, torch.Tensor):
        return _wrap(x)
    if isinstance(x, (list, tuple)):
        return type(x)(_wrap_nested(v) for v in x)
    return x


class _FnRemover:
    def __init__(self, fn):
        self.remove = fn


class _HookHandle:
    def __init__(self, h):
        self._h = h

    def remove(self):
        if self._h is not None:
            self._h.remove()
            self._h = None
            return True
        return False


def _index_to_torch(idx):
    if isinstance(idx, Tensor):
        return idx._t
    if isinstance(idx, tuple):
        return tuple(_index_to_torch(i) for i in idx)
    if isinstance(idx, list):
        if any(isinstance(i, Tensor) for i in idx):
            return [(_index_to_torch(i)) for i in idx]
        return idx
    if isinstance(idx, np.ndarray):
        return torch.from_numpy(idx)
    return idx


class Tensor:
    """Paddle eager Tensor. See module docstring."""

    __slots__ = ("_t", "_name", "_persistable", "__weakref__", "__dict__")
    __array_priority__ = 100

    def __init__(self, data=None, dtype=None, place=None, stop_gradient=True, name=None, **kw):
        if data is None:
            t = torch.empty(0)
        elif isinstance(data, Tensor):
            t = data._t
        else:
            t = _to_torch_tensor(data, dtype, place)
        if dtype is not None:
            t = t.to(_dt.to_torch_dtype(dtype))
        if stop_gradient or t.is_floating_point() or t.is_complex():
            self._t = t if stop_gradient else t.requires_grad_(True)
        else:  # paddle lets integer / bool tensors carry stop_gradient=False (no gradient ever flows to them)
            self._t = t
            self.__dict__["_sg_override"] = False
        self._name = name
        self._persistable = False

    # ---------------------------------------------------------------- properties
    @property
    def shape(self):
        return list(self._t.shape)

    @property
    def ndim(self):
        return self._t.dim()

    def dim(self):
        return self._t.dim()

    ndimension = dim

    @property
    def dtype(self):
        return _dt.from_torch_dtype(self._t.dtype)

    @property
    def place(self):
        return place_from_torch_device(self._t.device)

    @property
    def size(self):
        return self._t.numel()

    def numel(self):
        return _wrap(torch.tensor(self._t.numel(), dtype=torch.int64))

    @property
    def name(self):
        if self._name is None:
            self._name = f"generated_tensor_{next(_name_counter)}"
        return self._name

    @name.setter
    def name(self, v):
        self._name = v

    @property
    def persistable(self):
        return self._persistable

    @persistable.setter
    def persistable(self, v):
        self._persistable = bool(v)

    @property
    def stop_gradient(self):
        if self._t.requires_grad:
            return False
        return self.__dict__.get("_sg_override", True)

    @stop_gradient.setter
    def stop_gradient(self, v):
        v = bool(v)
        t = self._t
        self.__dict__.pop("_sg_override", None)
        if not (t.is_floating_point() or t.is_complex()):
            if not v:
                self.__dict__["_sg_override"] = False
            return
        if v:
            if t.requires_grad:
                self._t = t.detach() if not t.is_leaf else t.requires_grad_(False)
        else:
            if not t.requires_grad:
                if t.is_leaf:
                    t.requires_grad_(True)
                else:
                    # non-leaf that was created under no_grad: make it a new leaf
                    self._t = t.detach().requires_grad_(True)

    @property
    def is_leaf(self):
        return self._t.is_leaf

    @property
    def grad(self):
        g = self._t.grad
        if g is None:
            return None
        w = _wrap(g)
        w.__dict__["_sg_override"] = False  # paddle's gradient tensors report stop_gradient=False
        return w

    @grad.setter
    def grad(self, v):
        self._t.grad = None if v is None else _unwrap(v)

    @property
    def grad_(self):
        return self.grad

    @property
    def T(self):
        return _wrap(self._t.permute(*reversed(range(self._t.dim()))))

    @property
    def mT(self):
        return _wrap(self._t.transpose(-2, -1))

    @property
    def data(self):
        return _wrap(self._t.detach())

    @data.setter
    def data(self, v):
        with torch.no_grad():
            self._t.data = _unwrap(v).data

    @property
    def strides(self):
        return list(self._t.stride())

    def get_strides(self):
        return list(self._t.stride())

    @property
    def offset(self):
        return self._t.storage_offset()

    @property
    def layout(self):
        return "NCHW"

    @property
    def type(self):
        return "DENSE_TENSOR"

    # ---------------------------------------------------------------- conversion
    def numpy(self):
        t = self._t.detach()
        if t.dtype == torch.bfloat16:
            # paddle returns bf16 as uint16 raw bits; we return float32 values which is more useful
            t = t.float()
        elif t.dtype in (torch.float8_e4m3fn, torch.float8_e5m2):
            t = t.float()
        return t.cpu().numpy()

    def __array__(self, dtype=None, copy=None):
        a = self.numpy()
        return a.astype(dtype) if dtype is not None else a

    def item(self, *args):
        if args:
            return self._t[args].item() if len(args) > 1 else self._t.flatten()[args[0]].item()
        return self._t.item()

    def tolist(self):
        return self._t.tolist()

    def __float__(self):
        return float(self._t.item())

    def __int__(self):
        return int(self._t.item())

    def __index__(self):
        return int(self._t.item())

    def __bool__(self):
        return bool(self._t)

    def __len__(self):
        return len(self._t)

    def __iter__(self):
        for i in range(len(self._t)):
            yield _wrap(self._t[i])

    def __hash__(self):
        return id(self)

    def __repr__(self):
        grad_info = f", stop_gradient={self.stop_gradient}"
        data = np.array2string(self.numpy(), separator=", ", prefix="       ")
        return (f"Tensor(shape={self.shape}, dtype={self.dtype.name}, place={self.place}{grad_info},\n"
                f"       {data})")

    __str__ = __repr__

    def __format__(self, spec):
        if self._t.dim() == 0:
            return format(self._t.item(), spec)
        return repr(self)

    def __deepcopy__(self, memo):
        t = self._t.detach().clone()
        if self._t.requires_grad:
            t.requires_grad_(True)
        new = _wrap(t) if type(self) is Tensor else self._clone_as_same_type(t)
        new._name = self._name
        new._persistable = self._persistable
        memo[id(self)] = new
        return new

    def _clone_as_same_type(self, t):
        new = object.__new__(type(self))
        new._t = t
        new._name = None
        new._persistable = self._persistable
        for k, v in self.__dict__.items():
            new.__dict__[k] = v
        return new

    def __reduce_ex__(self, proto):
        # paddle.save format: (name, ndarray) tuples. Plain pickling of a Tensor keeps that.
        return (_rebuild_tensor, (self.numpy(), self.dtype.name, self.stop_gradient, self._name))

    # ---------------------------------------------------------------- device / dtype movement
    def cpu(self):
        return _wrap(self._t.cpu())

    def cuda(self, device_id=None, blocking=True):
        dev = torch.device("cuda", device_id) if device_id is not None else torch.device("cuda", torch.cuda.current_device())
        return _wrap(self._t.to(dev, non_blocking=not blocking))

    def pin_memory(self):
        """Page-locked copy from the native pinned pool (csrc/runtime/pinned_pool.cpp)."""
        from ..device import pinned
        return _wrap(pinned.pin(self._t.cpu()))

    def to(self, *args, **kwargs):
        device = kwargs.pop("device", None)
        dtype = kwargs.pop("dtype", None)
        blocking = kwargs.pop("blocking", True)
        for a in args:
            if isinstance(a, (Place, torch.device)) or (isinstance(a, str) and (a.startswith(("cpu", "gpu", "cuda")))):
                device = a
            elif isinstance(a, Tensor):
                device, dtype = a.place, a.dtype
            elif a is not None:
                dtype = a
        t = self._t
        if device is not None:
            t = t.to(to_torch_device(device), non_blocking=not blocking)
        if dtype is not None:
            t = t.to(_dt.to_torch_dtype(dtype))
        return _wrap(t)

    def astype(self, dtype):
        td = _dt.to_torch_dtype(dtype)
        if td == self._t.dtype:
            return self
        from ..amp.state import cast_tensor_raw
        return _wrap(cast_tensor_raw(self._t, td))

    def cast(self, dtype):
        return self.astype(dtype)

    def element_size(self):
        return self._t.element_size()

    def is_contiguous(self):
        return self._t.is_contiguous()

    def contiguous(self):
        return _wrap(self._t.contiguous())

    def data_ptr(self):
        return self._t.data_ptr()

    def value(self):
        return self

    def get_tensor(self):
        return self

    def _local_value(self):
        return self

    def is_dense(self):
        return True

    def is_dist(self):
        return False

    def _is_initialized(self):
        return True

    def is_floating_point(self):
        return self._t.is_floating_point()

    def is_complex(self):
        return self._t.is_complex()

    def is_integer(self):
        return not self._t.is_floating_point() and not self._t.is_complex() and self._t.dtype != torch.bool

    def _numel(self):
        return self._t.numel()

    def _is_shared_buffer_with(self, other):
        return self._t.untyped_storage().data_ptr() == _unwrap(other).untyped_storage().data_ptr()

    # ---------------------------------------------------------------- autograd
    def backward(self, grad_tensor=None, retain_graph=False):
        g = _unwrap(grad_tensor)
        if g is None:
            g = torch.ones_like(self._t)
        from ..autograd import engine as _eng
        if _eng.use_native():
            _eng.backward([self._t], [g], retain_graph=retain_graph)
            return
        self._t.backward(g, retain_graph=retain_graph)

    def gradient(self):
        """The accumulated gradient as a numpy array (None before backward) — legacy dygraph API."""
        g = self._t.grad
        return None if g is None else g.detach().cpu().numpy()

    def clear_grad(self, set_to_zero=True):
        g = self._t.grad
        if g is None:
            return
        if set_to_zero:
            g.zero_()
        else:
            self._t.grad = None

    clear_gradient = clear_grad

    def _clear_grad(self):
        self._t.grad = None

    def register_hook(self, hook):
        def _h(g):
            r = hook(_wrap(g))
            return None if r is None else _unwrap(r)
        from ..autograd import engine as _eng
        if _eng.use_native() and not _eng.runs_tensor_hooks():
            # pybind fallback traversal: it applies hooks from the (node, slot) table only
            return _HookHandle(_FnRemover(_eng.add_hook(self._t, _h)))
        # torch's tensor hook list: run by torch's engine and by the native executor alike
        return _HookHandle(self._t.register_hook(_h))

    def retain_grads(self):
        from ..autograd import engine as _eng
        if _eng.use_native():
            _eng.retain(self._t)  # paddle order: the retained value is the slot gradient at registration order
            return
        self._t.retain_grad()

    def detach(self):
        return _wrap(self._t.detach())

    def detach_(self):
        self._t = self._t.detach()
        return self

    def clone(self):
        return _wrap(self._t.clone())

    def _copy_to(self, place, blocking=True):
        return _wrap(self._t.to(to_torch_device(place), non_blocking=not blocking))

    def set_value(self, value):
        v = value._t if isinstance(value, Tensor) else torch.as_tensor(np.asarray(value))
        with torch.no_grad():
            if list(v.shape) != list(self._t.shape):
                raise ValueError(f"set_value shape mismatch {list(v.shape)} vs {self.shape}")
            self._t.copy_(v.to(self._t.device, self._t.dtype))
        return self

    def copy_(self, src, blocking=True):
        with torch.no_grad():
            self._t.copy_(_unwrap(src))
        return self

    def share_buffer_to(self, other):
        other._t = self._t

    def _share_buffer_to(self, other):
        other._t = self._t

    def _to_torch(self):
        return self._t

    # ---------------------------------------------------------------- indexing
    def __getitem__(self, idx):
        return _wrap(self._t[_index_to_torch(idx)])

    def __setitem__(self, idx, value):
        v = _unwrap(value)
        if isinstance(v, np.ndarray):
            v = torch.from_numpy(v)
        if isinstance(v, torch.Tensor):
            v = v.to(self._t.device)
            if v.dtype != self._t.dtype:
                v = v.to(self._t.dtype)
        t = self._t
        if t.is_leaf and t.requires_grad:
            with torch.no_grad():
                t[_index_to_torch(idx)] = v
        else:
            t[_index_to_torch(idx)] = v


def _rebuild_tensor(arr, dtype_name, stop_gradient, name):
    t = torch.from_numpy(np.asarray(arr)).to(_dt.to_torch_dtype(dtype_name))
    w = _wrap(t)
    w._name = name
    if not stop_gradient:
        w.stop_gradient = False
    return w


def _to_torch_tensor(data, dtype=None, place=None):
    dev = to_torch_device(place)
    td = _dt.to_torch_dtype(dtype) if dtype is not None else None
    if isinstance(data, Tensor):
        t = data._t
        return t.to(device=dev, dtype=td or t.dtype)
    if isinstance(data, torch.Tensor):
        return data.to(device=dev, dtype=td or data.dtype)
    if isinstance(data, np.ndarray):
        if data.dtype == np.float64 and td is None:
            t = torch.from_numpy(np.ascontiguousarray(data))
        else:
            t = torch.from_numpy(np.ascontiguousarray(data))
        return t.to(device=dev, dtype=td or t.dtype)
    if isinstance(data, np.generic):
        t = torch.from_numpy(np.asarray(data))
        return t.to(device=dev, dtype=td or t.dtype)
    # python scalars / nested lists (may contain Tensors)
    if isinstance(data, (list, tuple)) and any(isinstance(v, Tensor) for v in _flatten_list(data)):
        data = _nested_to_numpy(data)
        t = torch.from_numpy(np.ascontiguousarray(data))
        return t.to(device=dev, dtype=td or t.dtype)
    if td is None:
        flat = _flatten_list(data) if isinstance(data, (list, tuple)) else [data]
        if any(isinstance(v, complex) for v in flat):
            td = torch.complex64
        elif any(isinstance(v, float) for v in flat):
            td = _dt.default_dtype().torch_dtype
        elif all(isinstance(v, (bool, np.bool_)) for v in flat) and flat:
            td = torch.bool
        else:
            td = torch.int64
    return torch.tensor(data, dtype=td, device=dev)


def _flatten_list(x):
    out = []
    stack = [x]
    while stack:
        v = stack.pop()
        if isinstance(v, (list, tuple)):
            stack.extend(v)
        else:
            out.append(v)
    return out


def _nested_to_numpy(x):
    if isinstance(x, Tensor):
        return x.numpy()
    if isinstance(x, (list, tuple)):
        return np.stack([np.asarray(_nested_to_numpy(v)) for v in x])
    return np.asarray(x)


def to_tensor(data, dtype=None, place=None, stop_gradient=True):
    """paddle.to_tensor. Reference: python/paddle/tensor/creation.py to_tensor."""
    if isinstance(data, Tensor):
        t = data._t.detach()
        t = t.to(device=to_torch_device(place) if place is not None else t.device,
                 dtype=_dt.to_torch_dtype(dtype) if dtype is not None else t.dtype)
        if t is data._t or t.data_ptr() == data._t.data_ptr():
            t = t.clone()
    else:
        t = _to_torch_tensor(data, dtype, place)
    if not stop_gradient:
        if not (t.is_floating_point() or t.is_complex()):
            w = _wrap(t)
            w.__dict__["_sg_override"] = False
            return w
        t = t.detach().requires_grad_(True) if t.requires_grad else t.requires_grad_(True)
    return _wrap(t)


class Parameter(Tensor):
    """EagerParamBase. Reference: python/paddle/base/framework.py EagerParamBase."""

    __slots__ = ()

    def __init__(self, t, trainable=True, name=None, **attrs):
        if isinstance(t, Tensor):
            t = t._t
        t = t.detach()
        if trainable and (t.is_floating_point() or t.is_complex()):
            t.requires_grad_(True)
        self._t = t
        self._name = name
        self._persistable = True
        _PARAM_OF[id(t)] = self
        self.trainable = trainable
        self.optimize_attr = attrs.get("optimize_attr", {"learning_rate": 1.0})
        self.regularizer = attrs.get("regularizer", None)
        self.need_clip = attrs.get("need_clip", True)
        self.is_distributed = attrs.get("is_distributed", False)
        self.do_model_average = attrs.get("do_model_average", None)

    def initialize(self):
        """Materialise a parameter created under paddle.LazyGuard: allocate it on its device and run its
        initializer (no-op for an ordinary parameter)."""
        lazy = self.__dict__.pop("_lazy_init", None)
        if lazy is None:
            return self
        init, dev = lazy
        old = self._t
        t = torch.empty(old.shape, dtype=old.dtype, device=dev)
        with torch.no_grad():
            init._init(t)
        if old.requires_grad:
            t.requires_grad_(True)
        _PARAM_OF.pop(id(old), None)
        self._t = t
        _PARAM_OF[id(t)] = self
        return self

    @property
    def trainable(self):
        return self.__dict__.get("_trainable", True)

    @trainable.setter
    def trainable(self, v):
        self.__dict__["_trainable"] = bool(v)
        if self._t.is_floating_point() or self._t.is_complex():
            self._t.requires_grad_(bool(v))

    def __repr__(self):
        return "Parameter containing:\n" + super().__repr__()

    __str__ = __repr__

    def _replace_data(self, t):
        """Swap the underlying buffer (used by sharding / amp decorate) keeping identity."""
        req = self._t.requires_grad or self.__dict__.get("_sg_override") is False
        if req and not (t.is_floating_point() or t.is_complex()):
            self._t = t.detach()  # e.g. Layer.astype("int8"): keeps stop_gradient=False, no grad flows
            self.__dict__["_sg_override"] = False
        else:
            self._t = t.detach().requires_grad_(req)
            self.__dict__.pop("_sg_override", None)
        _PARAM_OF[id(self._t)] = self


EagerParamBase = Parameter


def is_tensor(x):
    return isinstance(x, Tensor)
