"""paddle.save / paddle.load. Reference: python/paddle/framework/io.py:773 save, :1020 load.

On-disk format = paddle's: a pickle (protocol 4). A state dict (a dict whose values are Tensors, or dicts
holding no Tensor) is stored as ``{key: numpy.ndarray, ..., "StructuredToParameterName@@": {key: tensor name}}``
(reference io.py:163 _build_saved_state_dict, :518 _is_state_dict); a Tensor anywhere else is reduced to a
``(name, numpy.ndarray)`` tuple — so files are interchangeable with paddle's ``.pdparams`` / ``.pdopt``.
bf16 is stored as its uint16 bit pattern, as paddle does. Loading uses a *restricted* unpickler that only
reconstructs numpy arrays, numpy dtypes, plain containers and the distributed-checkpoint metadata records; it
never imports or calls anything else from the file.
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
    return (tuple, ((t.name, _array_of(t)),))


_NAME_TABLE = "StructuredToParameterName@@"


def _contains_tensor(v):
    if isinstance(v, Tensor):
        return True
    if isinstance(v, dict):
        return any(_contains_tensor(x) for x in v.values())
    if isinstance(v, (list, tuple)):
        return any(_contains_tensor(x) for x in v)
    return False


def _is_state_dict(obj):
    if not isinstance(obj, dict):
        return False
    for v in obj.values():
        if isinstance(v, dict):
            if any(_contains_tensor(x) for x in v.values()):
                return False
        elif not isinstance(v, Tensor):
            return False
    return True


def _array_of(t):
    if t._t.dtype == torch.bfloat16:
        return t._t.detach().cpu().view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def _build_saved_state_dict(sd):
    out, names = type(sd)() if isinstance(sd, dict) else {}, {}
    for k, v in sd.items():
        if isinstance(v, Tensor):
            out[k] = _array_of(v)
            names[k] = v.name
        else:
            out[k] = v
    out[_NAME_TABLE] = names
    return out


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
    if _is_state_dict(obj):
        return _build_saved_state_dict(obj)
    return obj


_ALLOWED = {
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
    ("numpy._core.multiarray", "scalar"), ("collections", "OrderedDict"), ("builtins", "tuple"),
    ("builtins", "list"), ("builtins", "dict"), ("builtins", "set"), ("builtins", "frozenset"),
    ("builtins", "slice"), ("builtins", "complex"), ("_codecs", "encode"),
}


_CKPT_MODULES = ("paddle.distributed.checkpoint.metadata", "paddlepaddle_amd.distributed.checkpoint.metadata")


class _SafeUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED:
            return super().find_class(module, name)
        if module in _CKPT_MODULES:
            from ..distributed.checkpoint.metadata import CLASSES
            if name in CLASSES:
                return CLASSES[name]
        raise pickle.UnpicklingError(f"refusing to load global {module}.{name} (restricted loader)")


def _ndarray_tensor(arr, name=None):
    if arr.dtype == np.uint16:
        t = torch.from_numpy(arr.view(np.int16).copy()).view(torch.bfloat16)
    else:
        t = torch.from_numpy(np.ascontiguousarray(arr))
    from .place import _get_torch_device
    w = _wrap(t.to(_get_torch_device()))
    if name:
        w.name = name
    return w


def _to_tensor_tree(obj, return_numpy, keep_name_table=False):
    if isinstance(obj, dict) and isinstance(obj.get(_NAME_TABLE), dict):
        names = obj[_NAME_TABLE]
        out = type(obj)()
        for k, v in obj.items():
            if k == _NAME_TABLE:
                if keep_name_table:
                    out[k] = v
            elif k in names and isinstance(v, np.ndarray):
                out[k] = v if return_numpy else _ndarray_tensor(v, names[k])
            else:
                out[k] = _to_tensor_tree(v, return_numpy)
        return out
    if isinstance(obj, tuple) and len(obj) == 2 and isinstance(obj[0], str) and isinstance(obj[1], np.ndarray):
        return obj[1] if return_numpy else _ndarray_tensor(obj[1], obj[0])
    if isinstance(obj, np.ndarray):
        if return_numpy:
            return obj
        return _ndarray_tensor(obj)
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
    return _to_tensor_tree(obj, return_numpy, configs.get("keep_name_table", False))
