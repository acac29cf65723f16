"""paddle.save / paddle.load. Reference: python/paddle/framework/io.py:773 save, :1020 load.

On-disk format = paddle's: a pickle (protocol 4) in which every Tensor is reduced to a
``(name, numpy.ndarray)`` tuple (state dicts) — so files are interchangeable with paddle's
``.pdparams`` / ``.pdopt``. Loading uses a *restricted* unpickler that only reconstructs numpy
arrays, numpy dtypes and plain containers; it never imports or calls anything else from the file.
"""
from __future__ import annotations

import copyreg
import io as _io
import os
import pickle

import numpy as np
import torch

from .tensor import Parameter, Tensor, _wrap


def _reduce_tensor(t):
    arr = t.numpy()
    if t._t.dtype == torch.bfloat16:
        # paddle stores bf16 as uint16 bit patterns
        arr = t._t.detach().cpu().view(torch.int16).numpy().view(np.uint16)
    return (tuple, ((t.name, arr),))


def save(obj, path, protocol=4, **configs):
    if isinstance(path, (str, os.PathLike)):
        d = os.path.dirname(str(path))
        if d:
            os.makedirs(d, exist_ok=True)
        f = open(path, "wb")
        close = True
    else:
        f, close = path, False
    try:
        p = pickle.Pickler(f, protocol)
        p.dispatch_table = copyreg.dispatch_table.copy()
        p.dispatch_table[Tensor] = _reduce_tensor
        p.dispatch_table[Parameter] = _reduce_tensor
        obj2 = _prep(obj)
        p.dump(obj2)
    finally:
        if close:
            f.close()


def _prep(obj):
    from ..nn.layer.layers import Layer
    if isinstance(obj, Layer):
        raise ValueError("paddle do not support saving `paddle.nn.Layer` object.")
    return obj


_ALLOWED = {
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
    ("numpy._core.multiarray", "scalar"), ("collections", "OrderedDict"), ("builtins", "tuple"),
    ("builtins", "list"), ("builtins", "dict"), ("builtins", "set"), ("builtins", "frozenset"),
    ("builtins", "slice"), ("builtins", "complex"), ("_codecs", "encode"),
}


class _SafeUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load global {module}.{name} (restricted loader)")


def _to_tensor_tree(obj, return_numpy, keep_name_table=False):
    if isinstance(obj, tuple) and len(obj) == 2 and isinstance(obj[0], str) and isinstance(obj[1], np.ndarray):
        arr = obj[1]
        if return_numpy:
            return arr
        if arr.dtype == np.uint16:
            t = torch.from_numpy(arr.view(np.int16).copy()).view(torch.bfloat16)
        else:
            t = torch.from_numpy(np.ascontiguousarray(arr))
        from .place import _get_torch_device
        w = _wrap(t.to(_get_torch_device()))
        w.name = obj[0]
        return w
    if isinstance(obj, np.ndarray):
        if return_numpy:
            return obj
        from .place import _get_torch_device
        return _wrap(torch.from_numpy(np.ascontiguousarray(obj)).to(_get_torch_device()))
    if isinstance(obj, dict):
        return type(obj)((k, _to_tensor_tree(v, return_numpy)) for k, v in obj.items()) \
            if not isinstance(obj, type({}.keys())) else obj
    if isinstance(obj, list):
        return [_to_tensor_tree(v, return_numpy) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_to_tensor_tree(v, return_numpy) for v in obj)
    return obj


def load(path, **configs):
    return_numpy = configs.get("return_numpy", False)
    if isinstance(path, (str, os.PathLike)):
        with open(path, "rb") as f:
            obj = _SafeUnpickler(f).load()
    else:
        obj = _SafeUnpickler(path).load()
    return _to_tensor_tree(obj, return_numpy)
