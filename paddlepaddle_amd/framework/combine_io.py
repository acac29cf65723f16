"""Combined tensor files in the reference's ``save_combine`` layout (``.pdiparams``).

Reference: paddle/phi/core/framework/dense_tensor_serialize.cc (SerializeToStream) and dense_tensor_tostream.cc
(TensorToStream), framework.proto (VarType.TensorDesc). Each tensor record is
    uint32 version (0) | uint64 lod_level (0 here; lod levels are skipped when read)
    uint32 version (0) | int32 desc_size | TensorDesc protobuf (field 1 data_type, field 2 dims)
    raw little-endian data (numel x itemsize bytes)
and records follow each other in the order of the variable names (sorted, as save_inference_model writes
them). The protobuf is written / parsed here directly (varints), so no schema compiler is needed.
"""
from __future__ import annotations

import struct

import numpy as np
import torch

# framework.proto VarType.Type
_PROTO = {torch.bool: 0, torch.int16: 1, torch.int32: 2, torch.int64: 3, torch.float16: 4, torch.float32: 5,
          torch.float64: 6, torch.uint8: 20, torch.int8: 21, torch.bfloat16: 22, torch.complex64: 23,
          torch.complex128: 24}
_FROM_PROTO = {v: k for k, v in _PROTO.items()}


def _varint(n):
    n &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf, pos):
    shift = val = 0
    while True:
        b = buf[pos]
        pos += 1
        val |= (b & 0x7F) << shift
        if not b & 0x80:
            return val, pos
        shift += 7


def _signed64(v):
    return v - (1 << 64) if v >= (1 << 63) else v


def tensor_desc(dtype, dims):
    out = b"\x08" + _varint(_PROTO[dtype])
    for d in dims:
        out += b"\x10" + _varint(int(d))
    return out


def parse_desc(buf):
    pos, dtype, dims = 0, None, []
    while pos < len(buf):
        key, pos = _read_varint(buf, pos)
        field, wire = key >> 3, key & 7
        if wire == 0:
            v, pos = _read_varint(buf, pos)
            if field == 1:
                dtype = v
            elif field == 2:
                dims.append(_signed64(v))
        elif wire == 2:  # packed repeated dims (or an unknown length-delimited field)
            ln, pos = _read_varint(buf, pos)
            end = pos + ln
            if field == 2:
                while pos < end:
                    v, pos = _read_varint(buf, pos)
                    dims.append(_signed64(v))
            pos = end
        elif wire == 1:
            pos += 8
        elif wire == 5:
            pos += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wire}")
    return _FROM_PROTO[dtype], dims


def _raw(t):
    t = t.detach().cpu().contiguous()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().tobytes()
    return t.numpy().tobytes()


def combined_bytes(tensors):
    """The save_combine byte stream of ``tensors`` (in order)."""
    out = bytearray()
    for t in tensors:
        out += struct.pack("<IQ", 0, 0)
        desc = tensor_desc(t.dtype, list(t.shape))
        out += struct.pack("<Ii", 0, len(desc))
        out += desc
        out += _raw(t)
    return bytes(out)


def write_combined(path, tensors):
    """tensors: iterable of torch tensors, written in order."""
    with open(path, "wb") as f:
        for t in tensors:
            f.write(combined_bytes([t]))


def read_combined(path):
    """-> list of torch tensors in file order."""
    with open(path, "rb") as f:
        return parse_combined(f.read())


def parse_combined(data):
    """save_combine byte stream -> list of torch tensors."""
    out = []
    pos = 0
    while pos < len(data):
        _ver, lod_level = struct.unpack_from("<IQ", data, pos)
        pos += 12
        for _ in range(lod_level):
            (n,) = struct.unpack_from("<Q", data, pos)
            pos += 8 + n
        _ver2, dsize = struct.unpack_from("<Ii", data, pos)
        pos += 8
        dtype, dims = parse_desc(data[pos:pos + dsize])
        pos += dsize
        numel = int(np.prod(dims)) if dims else 1
        item = torch.empty(0, dtype=dtype).element_size()
        raw = data[pos:pos + numel * item]
        pos += numel * item
        if dtype == torch.bfloat16:
            t = torch.from_numpy(np.frombuffer(raw, dtype=np.int16).copy()).view(torch.bfloat16)
        else:
            npdt = torch.empty(0, dtype=dtype).numpy().dtype
            t = torch.from_numpy(np.frombuffer(raw, dtype=npdt).copy())
        out.append(t.reshape(dims))
    return out


def is_combined(path):
    """True for a save_combine file (starts with the uint32 version 0), False for a pickle."""
    with open(path, "rb") as f:
        head = f.read(4)
    return len(head) == 4 and head == b"\x00\x00\x00\x00"
