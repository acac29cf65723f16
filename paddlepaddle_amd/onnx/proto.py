"""Minimal protobuf wire-format writer / reader for the ONNX messages the exporter emits (field numbers of
onnx/onnx.proto3: ModelProto, GraphProto, NodeProto, AttributeProto, TensorProto, ValueInfoProto, TypeProto,
TensorShapeProto, OperatorSetIdProto). No dependency on the onnx package (not in this image)."""
from __future__ import annotations

import struct

import numpy as np

# TensorProto.DataType
FLOAT, UINT8, INT8, INT32, INT64, BOOL, FLOAT16, DOUBLE, BFLOAT16 = 1, 2, 3, 6, 7, 9, 10, 11, 16
NP2ONNX = {np.dtype("float32"): FLOAT, np.dtype("uint8"): UINT8, np.dtype("int8"): INT8, np.dtype("int32"): INT32,
           np.dtype("int64"): INT64, np.dtype("bool"): BOOL, np.dtype("float16"): FLOAT16, np.dtype("float64"): DOUBLE}
ONNX2NP = {v: k for k, v in NP2ONNX.items()}
# AttributeProto.AttributeType
A_FLOAT, A_INT, A_STRING, A_TENSOR, A_FLOATS, A_INTS = 1, 2, 3, 4, 6, 7


# ------------------------------------------------------------------------------------------------ writer
def _varint(v):
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field, wt):
    return _varint((field << 3) | wt)


def f_int(field, v):
    return _key(field, 0) + _varint(int(v))


def f_bytes(field, b):
    if isinstance(b, str):
        b = b.encode()
    return _key(field, 2) + _varint(len(b)) + b


def f_float(field, v):
    return _key(field, 5) + struct.pack("<f", float(v))


def f_packed_int(field, vals):
    body = b"".join(_varint(int(v)) for v in vals)
    return f_bytes(field, body)


def f_packed_float(field, vals):
    return f_bytes(field, struct.pack(f"<{len(vals)}f", *[float(v) for v in vals]))


def tensor(name, arr):
    arr = np.ascontiguousarray(arr)
    if arr.dtype not in NP2ONNX:
        raise TypeError(f"ONNX export: unsupported initializer dtype {arr.dtype}")
    return (f_packed_int(1, arr.shape) if arr.ndim else b"") + f_int(2, NP2ONNX[arr.dtype]) + f_bytes(8, name) + \
        f_bytes(9, arr.tobytes())


def attribute(name, v):
    body = f_bytes(1, name)
    if isinstance(v, bool) or isinstance(v, (int, np.integer)):
        return body + f_int(20, A_INT) + f_int(3, int(v))
    if isinstance(v, float):
        return body + f_int(20, A_FLOAT) + f_float(2, v)
    if isinstance(v, str):
        return body + f_int(20, A_STRING) + f_bytes(4, v)
    if isinstance(v, np.ndarray):
        return body + f_int(20, A_TENSOR) + f_bytes(5, tensor("", v))
    if isinstance(v, (list, tuple)):
        if all(isinstance(x, (int, np.integer)) and not isinstance(x, bool) for x in v):
            return body + f_int(20, A_INTS) + f_packed_int(8, v)
        return body + f_int(20, A_FLOATS) + f_packed_float(7, v)
    raise TypeError(f"ONNX export: unsupported attribute {name}={v!r}")


def node(op_type, inputs, outputs, name="", **attrs):
    b = b"".join(f_bytes(1, i) for i in inputs) + b"".join(f_bytes(2, o) for o in outputs)
    b += f_bytes(3, name) + f_bytes(4, op_type)
    for k in sorted(attrs):
        b += f_bytes(5, attribute(k, attrs[k]))
    return b


def value_info(name, elem_type, shape):
    dims = b"".join(f_bytes(1, f_int(1, d) if isinstance(d, int) and d >= 0 else f_bytes(2, str(d) if d else "N"))
                    for d in shape)
    ttype = f_int(1, elem_type) + f_bytes(2, dims)
    return f_bytes(1, name) + f_bytes(2, f_bytes(1, ttype))


def model(graph_nodes, name, initializers, inputs, outputs, opset=17, producer="paddlepaddle_amd"):
    g = b"".join(f_bytes(1, n) for n in graph_nodes) + f_bytes(2, name)
    g += b"".join(f_bytes(5, t) for t in initializers)
    g += b"".join(f_bytes(11, v) for v in inputs) + b"".join(f_bytes(12, v) for v in outputs)
    opset_b = f_bytes(1, "") + f_int(2, opset)
    return f_int(1, 8) + f_bytes(2, producer) + f_bytes(3, "3.0") + f_bytes(7, g) + f_bytes(8, opset_b)


# ------------------------------------------------------------------------------------------------ reader
def _read_varint(b, i):
    shift = r = 0
    while True:
        c = b[i]
        i += 1
        r |= (c & 0x7F) << shift
        if not c & 0x80:
            return r, i
        shift += 7


def fields(b):
    """[(field number, wire type, value)] of one message (value: int, bytes or 4-byte float)."""
    out, i = [], 0
    while i < len(b):
        k, i = _read_varint(b, i)
        f, wt = k >> 3, k & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 2:
            n, i = _read_varint(b, i)
            v = bytes(b[i:i + n])
            i += n
        elif wt == 5:
            v = struct.unpack("<f", b[i:i + 4])[0]
            i += 4
        elif wt == 1:
            v = struct.unpack("<d", b[i:i + 8])[0]
            i += 8
        else:
            raise ValueError(f"wire type {wt}")
        out.append((f, wt, v))
    return out


def _signed(v):
    return v - (1 << 64) if v >= 1 << 63 else v


def _packed_ints(v):
    out, i = [], 0
    while i < len(v):
        x, i = _read_varint(v, i)
        out.append(_signed(x))
    return out


def read_tensor(b):
    dims, dt, name, raw = [], FLOAT, "", b""
    for f, wt, v in fields(b):
        if f == 1:
            dims += _packed_ints(v) if wt == 2 else [_signed(v)]
        elif f == 2:
            dt = v
        elif f == 8:
            name = v.decode()
        elif f == 9:
            raw = v
    return name, np.frombuffer(raw, dtype=ONNX2NP[dt]).reshape(dims).copy()


def read_attribute(b):
    name, typ, val = "", 0, None
    ints, floats = [], []
    for f, wt, v in fields(b):
        if f == 1:
            name = v.decode()
        elif f == 20:
            typ = v
        elif f == 2:
            val = v
        elif f == 3:
            val = _signed(v)
        elif f == 4:
            val = v.decode()
        elif f == 5:
            val = read_tensor(v)[1]
        elif f == 7:
            floats += list(struct.unpack(f"<{len(v) // 4}f", v)) if wt == 2 else [v]
        elif f == 8:
            ints += _packed_ints(v) if wt == 2 else [_signed(v)]
    if typ == A_INTS:
        val = ints
    elif typ == A_FLOATS:
        val = floats
    return name, val


def read_model(b):
    """{"opset", "nodes": [(op, inputs, outputs, attrs)], "initializers": {name: array}, "inputs", "outputs"}."""
    m = {"opset": None, "nodes": [], "initializers": {}, "inputs": [], "outputs": []}
    for f, _, v in fields(b):
        if f == 8:
            for f2, _, v2 in fields(v):
                if f2 == 2:
                    m["opset"] = v2
        elif f == 7:
            for f2, _, v2 in fields(v):
                if f2 == 1:
                    ins, outs, op, attrs = [], [], "", {}
                    for f3, _, v3 in fields(v2):
                        if f3 == 1:
                            ins.append(v3.decode())
                        elif f3 == 2:
                            outs.append(v3.decode())
                        elif f3 == 4:
                            op = v3.decode()
                        elif f3 == 5:
                            k, a = read_attribute(v3)
                            attrs[k] = a
                    m["nodes"].append((op, ins, outs, attrs))
                elif f2 == 5:
                    name, arr = read_tensor(v2)
                    m["initializers"][name] = arr
                elif f2 in (11, 12):
                    name = next(x for ff, _, x in fields(v2) if ff == 1).decode()
                    m["inputs" if f2 == 11 else "outputs"].append(name)
    return m
