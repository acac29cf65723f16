"""Paddle data types mapped onto device storage dtypes.

Reference: python/paddle/framework/dtype.py (DataType enum exposed as paddle.float32 …).
gfx950 uses OCP fp8 (e4m3fn / e5m2), *not* the MI300 fnuz variants, so float8_e4m3fn maps to
torch.float8_e4m3fn.
"""
from __future__ import annotations

import numpy as np
import torch


class DType:
    """A paddle dtype. Compares equal to other DType objects and to its name string."""

    __slots__ = ("name", "torch_dtype", "np_dtype", "_hash")

    def __init__(self, name, torch_dtype, np_dtype):
        self.name = name
        self.torch_dtype = torch_dtype
        self.np_dtype = np_dtype
        self._hash = hash(("paddle.dtype", name))

    def __repr__(self):
        return f"paddle.{self.name}"

    __str__ = __repr__

    def __eq__(self, other):
        if isinstance(other, DType):
            return self.name == other.name
        if isinstance(other, str):
            return _canon_name(other) == self.name
        if isinstance(other, torch.dtype):
            return other == self.torch_dtype
        if isinstance(other, (np.dtype, type)):
            try:
                return np.dtype(other) == self.np_dtype and self.np_dtype is not None
            except TypeError:
                return False
        return NotImplemented

    def __ne__(self, other):
        r = self.__eq__(other)
        return r if r is NotImplemented else not r

    def __hash__(self):
        return self._hash

    @property
    def is_floating_point(self):
        return self.torch_dtype.is_floating_point

    @property
    def is_complex(self):
        return self.torch_dtype.is_complex

    @property
    def itemsize(self):
        return torch.empty((), dtype=self.torch_dtype).element_size()


uint8 = DType("uint8", torch.uint8, np.uint8)
int8 = DType("int8", torch.int8, np.int8)
int16 = DType("int16", torch.int16, np.int16)
int32 = DType("int32", torch.int32, np.int32)
int64 = DType("int64", torch.int64, np.int64)
float16 = DType("float16", torch.float16, np.float16)
bfloat16 = DType("bfloat16", torch.bfloat16, None)
float32 = DType("float32", torch.float32, np.float32)
float64 = DType("float64", torch.float64, np.float64)
bool_ = DType("bool", torch.bool, np.bool_)
complex64 = DType("complex64", torch.complex64, np.complex64)
complex128 = DType("complex128", torch.complex128, np.complex128)
float8_e4m3fn = DType("float8_e4m3fn", torch.float8_e4m3fn, None)
float8_e5m2 = DType("float8_e5m2", torch.float8_e5m2, None)
uint16 = DType("uint16", torch.uint16 if hasattr(torch, "uint16") else torch.int16, np.uint16)

_ALL = [uint8, int8, int16, int32, int64, float16, bfloat16, float32, float64, bool_,
        complex64, complex128, float8_e4m3fn, float8_e5m2, uint16]
_BY_NAME = {d.name: d for d in _ALL}
_BY_TORCH = {}
for _d in _ALL:
    _BY_TORCH.setdefault(_d.torch_dtype, _d)

_ALIASES = {
    "float": "float32", "fp32": "float32", "double": "float64", "fp64": "float64",
    "half": "float16", "fp16": "float16", "bf16": "bfloat16", "int": "int32", "long": "int64",
    "bool_": "bool", "float8_e4m3": "float8_e4m3fn", "fp8": "float8_e4m3fn",
}


def _canon_name(s: str) -> str:
    s = s.replace("paddle.", "")
    return _ALIASES.get(s, s)


def convert_dtype(d) -> DType:
    """Convert any dtype spelling (DType, str, torch.dtype, numpy dtype) to a DType."""
    if d is None:
        return None
    if isinstance(d, DType):
        return d
    if isinstance(d, str):
        n = _canon_name(d)
        if n in _BY_NAME:
            return _BY_NAME[n]
        raise TypeError(f"unsupported dtype {d!r}")
    if isinstance(d, torch.dtype):
        return _BY_TORCH[d]
    if d is bool:
        return bool_
    if d is int:
        return int64
    if d is float:
        return float32
    try:
        nd = np.dtype(d)
    except TypeError:
        raise TypeError(f"unsupported dtype {d!r}")
    for x in _ALL:
        if x.np_dtype is not None and np.dtype(x.np_dtype) == nd:
            return x
    raise TypeError(f"unsupported dtype {d!r}")


def to_torch_dtype(d):
    if d is None:
        return None
    if isinstance(d, torch.dtype):
        return d
    return convert_dtype(d).torch_dtype


def from_torch_dtype(td) -> DType:
    return _BY_TORCH[td]


_default_dtype = float32


def set_default_dtype(d):
    global _default_dtype
    d = convert_dtype(d)
    if d not in (float16, float32, float64, bfloat16):
        raise TypeError("set_default_dtype only supports floating dtypes")
    _default_dtype = d


def get_default_dtype():
    return _default_dtype.name


def default_dtype() -> DType:
    return _default_dtype


class finfo:
    def __init__(self, dtype):
        fi = torch.finfo(to_torch_dtype(dtype))
        self.dtype = convert_dtype(dtype).name
        self.bits = fi.bits
        self.eps = fi.eps
        self.min = fi.min
        self.max = fi.max
        self.tiny = fi.tiny
        self.smallest_normal = fi.smallest_normal
        self.resolution = fi.resolution


class iinfo:
    def __init__(self, dtype):
        ii = torch.iinfo(to_torch_dtype(dtype))
        self.dtype = convert_dtype(dtype).name
        self.bits = ii.bits
        self.min = ii.min
        self.max = ii.max

    def __repr__(self):
        return f"paddle.iinfo(min={self.min}, max={self.max}, bits={self.bits}, dtype={self.dtype})"
