"""Reference-format program files: the ``ProgramDesc`` protobuf of ``.pdmodel`` inference models.

Reference: paddle/fluid/framework/framework.proto (ProgramDesc / BlockDesc / VarDesc / OpDesc / OpDesc.Attr /
VarType), python/paddle/static/io.py:513 save_inference_model / :848 load_inference_model. A model exported by
the reference (``paddle.jit.save`` / ``paddle.static.save_inference_model`` in the legacy program format) is a
``.pdmodel`` ProgramDesc plus a ``.pdiparams`` save_combine file holding the persistable variables sorted by
name (framework/combine_io.py).

This module
  * encodes / decodes the protobuf wire format directly against the framework.proto field numbers (no schema
    compiler, nothing executed from the file);
  * runs block 0 of a decoded program with an op table mapping the reference's operator types (feed / fetch,
    matmul_v2, elementwise_*, conv2d, batch_norm, layer_norm, pool2d, reshape2, transpose2, softmax, ...) onto
    this framework's functional ops, so the HIP kernels serve the model (``ProgramDescRunner``);
  * builds ProgramDescs (``ProgramDescBuilder``) and writes ``.pdmodel`` + ``.pdiparams`` pairs in that layout.
"""
from __future__ import annotations

import struct

import numpy as np
import torch

from .combine_io import _FROM_PROTO, _PROTO, _read_varint, _signed64, _varint

# ----------------------------------------------------------------------------------------------- wire codec
# field kinds: "v" varint (int / bool / enum), "sv" signed varint stored as int64 two's complement, "f32" fixed32
# float, "f64" fixed64 double, "s" string, "m:<Msg>" nested message; a leading "*" marks repeated fields.
SCHEMA = {
    "ProgramDesc": {1: ("blocks", "*m:BlockDesc"), 4: ("version", "m:Version"), 5: ("op_version_map", "m:OpVersionMap")},
    "Version": {1: ("version", "sv")},
    "OpVersionMap": {1: ("pair", "*m:OpVersionPair")},
    "OpVersionPair": {1: ("op_name", "s"), 2: ("op_version", "m:OpVersion")},
    "OpVersion": {1: ("version", "sv")},
    "BlockDesc": {1: ("idx", "sv"), 2: ("parent_idx", "sv"), 3: ("vars", "*m:VarDesc"), 4: ("ops", "*m:OpDesc"),
                  5: ("forward_block_idx", "sv")},
    "VarDesc": {1: ("name", "s"), 2: ("type", "m:VarType"), 3: ("persistable", "v"), 4: ("need_check_feed", "v"),
                5: ("is_parameter", "v"), 6: ("stop_gradient", "v"), 7: ("attrs", "*m:VarAttr")},
    "VarAttr": {1: ("name", "s"), 2: ("type", "v"), 3: ("i", "sv"), 4: ("s", "s"), 5: ("ints", "*sv")},
    "VarType": {1: ("type", "v"), 2: ("selected_rows", "m:TensorDesc"), 3: ("dense_tensor", "m:DenseTensorDesc"),
                4: ("tensor_array", "m:DenseTensorDesc")},
    "DenseTensorDesc": {1: ("tensor", "m:TensorDesc"), 2: ("legacy_lod_level", "sv")},
    "TensorDesc": {1: ("data_type", "v"), 2: ("dims", "*sv")},
    "OpDesc": {3: ("type", "s"), 1: ("inputs", "*m:OpVar"), 2: ("outputs", "*m:OpVar"), 4: ("attrs", "*m:OpAttr"),
               5: ("is_target", "v")},
    "OpVar": {1: ("parameter", "s"), 2: ("arguments", "*s")},
    "OpAttr": {1: ("name", "s"), 2: ("type", "v"), 3: ("i", "sv"), 4: ("f", "f32"), 5: ("s", "s"), 6: ("ints", "*sv"),
               7: ("floats", "*f32"), 8: ("strings", "*s"), 10: ("b", "v"), 11: ("bools", "*v"),
               12: ("block_idx", "sv"), 13: ("l", "sv"), 14: ("blocks_idx", "*sv"), 15: ("longs", "*sv"),
               16: ("float64s", "*f64"), 17: ("var_name", "s"), 18: ("vars_name", "*s"), 19: ("float64", "f64"),
               20: ("scalar", "m:Scalar"), 21: ("scalars", "*m:Scalar")},
    "Scalar": {1: ("type", "v"), 2: ("b", "v"), 3: ("i", "sv"), 4: ("r", "f64"), 5: ("c", "m:Complex")},
    "Complex": {1: ("r", "f64"), 2: ("i", "f64")},
}

# framework.proto AttrType
INT, FLOAT, STRING, INTS, FLOATS, STRINGS, BOOLEAN, BOOLEANS, BLOCK, LONG, BLOCKS, LONGS, FLOAT64S, VAR, VARS, \
    FLOAT64, SCALAR, SCALARS = range(18)
_ATTR_FIELD = {INT: "i", FLOAT: "f", STRING: "s", INTS: "ints", FLOATS: "floats", STRINGS: "strings", BOOLEAN: "b",
               BOOLEANS: "bools", BLOCK: "block_idx", LONG: "l", BLOCKS: "blocks_idx", LONGS: "longs",
               FLOAT64S: "float64s", VAR: "var_name", VARS: "vars_name", FLOAT64: "float64", SCALAR: "scalar",
               SCALARS: "scalars"}
DENSE_TENSOR, FEED_MINIBATCH, FETCH_LIST = 7, 9, 10


def _kind(spec):
    rep = spec.startswith("*")
    return rep, spec[1:] if rep else spec


def decode(buf, msg="ProgramDesc"):
    """Decode ``buf`` as message ``msg`` into a dict (repeated fields -> lists; unknown fields skipped)."""
    sch = SCHEMA[msg]
    out = {}
    pos, end = 0, len(buf)
    while pos < end:
        key, pos = _read_varint(buf, pos)
        fno, wt = key >> 3, key & 7
        if wt == 0:
            raw, pos = _read_varint(buf, pos)
        elif wt == 1:
            raw = buf[pos:pos + 8]
            pos += 8
        elif wt == 5:
            raw = buf[pos:pos + 4]
            pos += 4
        elif wt == 2:
            n, pos = _read_varint(buf, pos)
            raw = bytes(buf[pos:pos + n])
            pos += n
        else:
            raise ValueError(f"ProgramDesc: unsupported wire type {wt} in {msg}")
        if fno not in sch:
            continue
        name, spec = sch[fno]
        rep, kind = _kind(spec)
        if wt == 2 and kind in ("v", "sv", "f32", "f64"):  # packed repeated scalars
            vals, p = [], 0
            while p < len(raw):
                if kind in ("v", "sv"):
                    v, p = _read_varint(raw, p)
                    vals.append(_signed64(v) if kind == "sv" else v)
                elif kind == "f32":
                    vals.append(struct.unpack_from("<f", raw, p)[0])
                    p += 4
                else:
                    vals.append(struct.unpack_from("<d", raw, p)[0])
                    p += 8
            out.setdefault(name, []).extend(vals)
            continue
        if kind == "v":
            val = raw
        elif kind == "sv":
            val = _signed64(raw)
        elif kind == "f32":
            val = struct.unpack("<f", raw)[0]
        elif kind == "f64":
            val = struct.unpack("<d", raw)[0]
        elif kind == "s":
            val = raw.decode("utf-8")
        else:
            val = decode(raw, kind[2:])
        if rep:
            out.setdefault(name, []).append(val)
        else:
            out[name] = val
    return out


def encode(d, msg="ProgramDesc"):
    """Encode dict ``d`` as message ``msg`` (fields in field-number order; repeated scalars unpacked, as
    proto2 writes them)."""
    sch = SCHEMA[msg]
    out = bytearray()
    for fno in sorted(sch):
        name, spec = sch[fno]
        if name not in d or d[name] is None:
            continue
        rep, kind = _kind(spec)
        vals = d[name] if rep else [d[name]]
        for v in vals:
            if kind in ("v", "sv"):
                out += _varint(fno << 3) + _varint(int(v))
            elif kind == "f32":
                out += _varint(fno << 3 | 5) + struct.pack("<f", float(v))
            elif kind == "f64":
                out += _varint(fno << 3 | 1) + struct.pack("<d", float(v))
            else:
                b = v.encode("utf-8") if kind == "s" else encode(v, kind[2:])
                out += _varint(fno << 3 | 2) + _varint(len(b)) + b
    return bytes(out)


# ------------------------------------------------------------------------------------------ decoded views
def op_attrs(op):
    res = {}
    for a in op.get("attrs", []):
        f = _ATTR_FIELD.get(a.get("type", INT), "i")
        default = [] if f in ("ints", "floats", "strings", "bools", "blocks_idx", "longs", "float64s",
                              "vars_name", "scalars") else None
        v = a.get(f, default)
        if f == "b" or f == "bools":
            v = bool(v) if f == "b" else [bool(x) for x in v]
        elif f == "scalar" and v is not None:
            v = _scalar_value(v)
        res[a["name"]] = v
    return res


def _scalar_value(s):
    t = s.get("type")
    return bool(s.get("b")) if t == 1 else s.get("i") if t == 2 else s.get("r") if t == 3 else \
        complex(s["c"]["r"], s["c"]["i"])


def _io(op, key):
    res = {}
    for v in op.get(key, []):
        res[v["parameter"]] = list(v.get("arguments", []))
    return res


class Program:
    """A decoded reference program: block 0 vars and ops, plus the feed / fetch targets."""

    def __init__(self, desc):
        self.desc = desc
        blk = desc["blocks"][0]
        self.vars = {}
        for v in blk.get("vars", []):
            ty = v.get("type", {})
            td = ty.get("dense_tensor", {}).get("tensor", {})
            self.vars[v["name"]] = {"type": ty.get("type", DENSE_TENSOR), "persistable": bool(v.get("persistable")),
                                    "dtype": _FROM_PROTO.get(td.get("data_type")), "shape": td.get("dims", [])}
        self.ops = [{"type": o["type"], "inputs": _io(o, "inputs"), "outputs": _io(o, "outputs"),
                     "attrs": op_attrs(o)} for o in blk.get("ops", [])]
        feeds = sorted((o["attrs"].get("col", 0), o["outputs"]["Out"][0]) for o in self.ops if o["type"] == "feed")
        fetches = sorted((o["attrs"].get("col", 0), o["inputs"]["X"][0]) for o in self.ops if o["type"] == "fetch")
        self.feed_names = [n for _, n in feeds]
        self.fetch_names = [n for _, n in fetches]

    def persistable_names(self):
        """The .pdiparams record order: persistable dense tensors except feed / fetch holders, sorted."""
        return sorted(n for n, v in self.vars.items()
                      if v["persistable"] and v["type"] not in (FEED_MINIBATCH, FETCH_LIST))


def parse(data):
    return Program(decode(data))


def is_program_desc(path):
    with open(path, "rb") as f:
        head = f.read(1)
    return head == b"\x0a"  # field 1 (blocks), wire type 2


# ------------------------------------------------------------------------------------------------ op table
def _F():
    from ..nn import functional as F
    return F


def _P():
    import paddlepaddle_amd as paddle
    return paddle


def _bcast_y(x, y, axis):
    """elementwise_* legacy broadcast: Y's dims line up with X's starting at ``axis`` (-1 = trailing)."""
    if axis is None or axis == -1 or y.ndim == x.ndim:
        return y
    tail = x.ndim - axis - y.ndim
    return y.reshape(list(y.shape) + [1] * tail) if tail > 0 else y


def _ew(fn):
    def run(ins, a):
        x, y = ins["X"][0], ins["Y"][0]
        return {"Out": [fn(x, _bcast_y(x, y, a.get("axis", -1)))]}
    return run


def _unary(fn):
    return lambda ins, a: {"Out": [fn(ins["X"][0], a)]}


def _matmul_v2(ins, a):
    P = _P()
    return {"Out": [P.matmul(ins["X"][0], ins["Y"][0], transpose_x=bool(a.get("trans_x")),
                             transpose_y=bool(a.get("trans_y")))]}


def _matmul_v1(ins, a):
    P = _P()
    out = P.matmul(ins["X"][0], ins["Y"][0], transpose_x=bool(a.get("transpose_X")),
                   transpose_y=bool(a.get("transpose_Y")))
    alpha = a.get("alpha", 1.0)
    return {"Out": [out if alpha in (None, 1.0) else out * alpha]}


def _mul(ins, a):
    P = _P()
    x, y = ins["X"][0], ins["Y"][0]
    xn, yn = a.get("x_num_col_dims", 1), a.get("y_num_col_dims", 1)
    xs, ys = list(x.shape), list(y.shape)
    x2 = x.reshape([int(np.prod(xs[:xn])), int(np.prod(xs[xn:]))])
    y2 = y.reshape([int(np.prod(ys[:yn])), int(np.prod(ys[yn:]))])
    return {"Out": [P.matmul(x2, y2).reshape(xs[:xn] + ys[yn:])]}


def _fc(ins, a):
    P = _P()
    x, w = ins["Input"][0], ins["W"][0]
    n = a.get("in_num_col_dims", 1)
    xs = list(x.shape)
    out = P.matmul(x.reshape([int(np.prod(xs[:n])), -1]), w)
    if ins.get("Bias"):
        out = out + ins["Bias"][0].reshape([-1])
    if a.get("activation_type") == "relu":
        out = _F().relu(out)
    return {"Out": [out.reshape(xs[:n] + [w.shape[1]])]}


def _fmt(a, key="data_format", default="NCHW"):
    f = a.get(key) or default
    return "NCHW" if f in ("AnyLayout", "NCHW") else f


def _conv_pad(a):
    alg = a.get("padding_algorithm", "EXPLICIT")
    if alg in ("SAME", "VALID"):
        return alg
    p = list(a.get("paddings", [0, 0]))
    return p if len(p) != 4 else [[0, 0], [0, 0], [p[0], p[1]], [p[2], p[3]]] if _fmt(a) == "NCHW" else \
        [[0, 0], [p[0], p[1]], [p[2], p[3]], [0, 0]]


def _conv2d(ins, a):
    out = _F().conv2d(ins["Input"][0], ins["Filter"][0], bias=None, stride=a.get("strides", [1, 1]),
                      padding=_conv_pad(a), dilation=a.get("dilations", [1, 1]), groups=a.get("groups", 1) or 1,
                      data_format=_fmt(a))
    return {"Output": [out]}


def _conv2d_t(ins, a):
    out = _F().conv2d_transpose(ins["Input"][0], ins["Filter"][0], bias=None, stride=a.get("strides", [1, 1]),
                                padding=_conv_pad(a), output_padding=a.get("output_padding") or 0,
                                dilation=a.get("dilations", [1, 1]), groups=a.get("groups", 1) or 1,
                                data_format=_fmt(a))
    return {"Output": [out]}


def _batch_norm(ins, a):
    y = _F().batch_norm(ins["X"][0], ins["Mean"][0], ins["Variance"][0], weight=ins["Scale"][0],
                        bias=ins["Bias"][0], training=False, epsilon=a.get("epsilon", 1e-5),
                        data_format=_fmt(a, "data_layout"))
    return {"Y": [y]}


def _layer_norm(ins, a):
    x = ins["X"][0]
    b = a.get("begin_norm_axis", 1)
    shape = list(x.shape)[b:]
    w = ins["Scale"][0].reshape(shape) if ins.get("Scale") else None
    bias = ins["Bias"][0].reshape(shape) if ins.get("Bias") else None
    return {"Y": [_F().layer_norm(x, shape, weight=w, bias=bias, epsilon=a.get("epsilon", 1e-5))]}


def _pool2d(ins, a):
    F = _F()
    x = ins["X"][0]
    fmt = _fmt(a)
    typ = a.get("pooling_type", "max")
    if a.get("global_pooling") or (a.get("adaptive") and list(a.get("ksize")) == [1, 1]):
        fn = F.adaptive_max_pool2d if typ == "max" else F.adaptive_avg_pool2d
        return {"Out": [fn(x, 1, data_format=fmt) if typ != "max" else fn(x, 1)]}
    if a.get("adaptive"):
        fn = F.adaptive_max_pool2d if typ == "max" else F.adaptive_avg_pool2d
        return {"Out": [fn(x, a["ksize"]) if typ == "max" else fn(x, a["ksize"], data_format=fmt)]}
    pad = _conv_pad(a)
    if typ == "max":
        out = F.max_pool2d(x, a["ksize"], stride=a.get("strides"), padding=pad, ceil_mode=bool(a.get("ceil_mode")),
                           data_format=fmt)
    else:
        out = F.avg_pool2d(x, a["ksize"], stride=a.get("strides"), padding=pad, ceil_mode=bool(a.get("ceil_mode")),
                           exclusive=a.get("exclusive", True), data_format=fmt)
    return {"Out": [out]}


def _reshape2(ins, a):
    x = ins["X"][0]
    if ins.get("ShapeTensor"):
        shape = [int(t.item()) for t in ins["ShapeTensor"]]
    elif ins.get("Shape"):
        shape = [int(v) for v in ins["Shape"][0].numpy().tolist()]
    else:
        shape = list(a.get("shape", []))
    shape = [x.shape[i] if s == 0 else s for i, s in enumerate(shape)]
    return {"Out": [x.reshape(shape)]}


def _flatten(ins, a):
    return {"Out": [_P().flatten(ins["X"][0], a.get("start_axis", 1), a.get("stop_axis", -1))]}


def _slice(ins, a):
    x = ins["Input"][0]
    idx = [slice(None)] * x.ndim
    for ax, s, e in zip(a["axes"], a["starts"], a["ends"]):
        idx[ax] = slice(s, min(e, x.shape[ax]) if e > 0 else e)
    out = x[tuple(idx)]
    dec = a.get("decrease_axis") or []
    if dec:
        out = out.reshape([d for i, d in enumerate(out.shape) if i not in dec])
    return {"Out": [out]}


def _split(ins, a):
    P = _P()
    x = ins["X"][0]
    secs = a.get("sections") or []
    return {"Out": list(P.split(x, secs if secs else a.get("num", 1), axis=a.get("axis", 0)))}


def _scale(ins, a):
    x = ins["X"][0]
    s = float(ins["ScaleTensor"][0].item()) if ins.get("ScaleTensor") else a.get("scale", 1.0)
    b = a.get("bias", 0.0)
    return {"Out": [x * s + b if a.get("bias_after_scale", True) else (x + b) * s]}


def _dropout(ins, a):
    x = ins["X"][0]
    p = a.get("dropout_prob", 0.5)
    keep = a.get("dropout_implementation", "downgrade_in_infer") == "upscale_in_train"
    return {"Out": [x if keep else x * (1.0 - p)]}


def _fill_constant(ins, a):
    P = _P()
    dt = _FROM_PROTO.get(a.get("dtype", 5), torch.float32)
    v = a.get("str_value")
    v = float(v) if v not in (None, "") else a.get("value", 0.0)
    return {"Out": [P.Tensor(torch.full(list(a.get("shape", [])), v, dtype=dt, device=_dev()))]}


def _cast(ins, a):
    dt = _FROM_PROTO[a["out_dtype"]]
    from .dtype import from_torch_dtype
    return {"Out": [ins["X"][0].astype(from_torch_dtype(dt))]}


def _reduce(name):
    def run(ins, a):
        P = _P()
        x = ins["X"][0]
        ax = None if a.get("reduce_all") else a.get("dim")
        return {"Out": [getattr(P, name)(x, axis=ax, keepdim=bool(a.get("keep_dim")))]}
    return run


def _interp(mode):
    def run(ins, a):
        x = ins["X"][0]
        fmt = _fmt(a, "data_layout")
        size = None
        if a.get("out_h", -1) and a.get("out_h", -1) > 0:
            size = [a["out_h"], a["out_w"]]
        sc = a.get("scale") or None
        out = _F().interpolate(x, size=size, scale_factor=None if size else sc, mode=mode,
                               align_corners=bool(a.get("align_corners")), align_mode=a.get("align_mode", 1),
                               data_format=fmt)
        return {"Out": [out]}
    return run


def _dev():
    from .place import _get_torch_device
    return _get_torch_device()


def _act(name, **kw):
    return _unary(lambda x, a: getattr(_F(), name)(x, **{k: a.get(v, d) for k, (v, d) in kw.items()}))


OPS = {
    "matmul_v2": _matmul_v2, "matmul": _matmul_v1, "mul": _mul, "fc": _fc,
    "elementwise_add": _ew(lambda x, y: x + y), "elementwise_sub": _ew(lambda x, y: x - y),
    "elementwise_mul": _ew(lambda x, y: x * y), "elementwise_div": _ew(lambda x, y: x / y),
    "elementwise_pow": _ew(lambda x, y: x ** y), "elementwise_max": _ew(lambda x, y: _P().maximum(x, y)),
    "elementwise_min": _ew(lambda x, y: _P().minimum(x, y)),
    "relu": _act("relu"), "sigmoid": _act("sigmoid"), "tanh": _unary(lambda x, a: _P().tanh(x)),
    "gelu": _unary(lambda x, a: _F().gelu(x, approximate=bool(a.get("approximate")))),
    "silu": _act("silu"), "swish": _act("silu"), "relu6": _act("relu6"),
    "leaky_relu": _unary(lambda x, a: _F().leaky_relu(x, a.get("alpha", 0.02))),
    "hard_swish": _act("hardswish"), "hard_sigmoid": _unary(
        lambda x, a: _F().hardsigmoid(x, slope=a.get("slope", 0.1666667), offset=a.get("offset", 0.5))),
    "softplus": _act("softplus"), "elu": _unary(lambda x, a: _F().elu(x, a.get("alpha", 1.0))),
    "exp": _unary(lambda x, a: _P().exp(x)), "sqrt": _unary(lambda x, a: _P().sqrt(x)),
    "rsqrt": _unary(lambda x, a: _P().rsqrt(x)), "abs": _unary(lambda x, a: _P().abs(x)),
    "log": _unary(lambda x, a: _P().log(x)), "square": _unary(lambda x, a: x * x),
    "softmax": _unary(lambda x, a: _F().softmax(x, axis=a.get("axis", -1))),
    "log_softmax": _unary(lambda x, a: _F().log_softmax(x, axis=a.get("axis", -1))),
    "conv2d": _conv2d, "depthwise_conv2d": _conv2d, "conv2d_transpose": _conv2d_t,
    "batch_norm": _batch_norm, "layer_norm": _layer_norm, "pool2d": _pool2d,
    "reshape2": _reshape2, "reshape": _reshape2,
    "transpose2": lambda ins, a: {"Out": [_P().transpose(ins["X"][0], list(a["axis"]))]},
    "transpose": lambda ins, a: {"Out": [_P().transpose(ins["X"][0], list(a["axis"]))]},
    "flatten_contiguous_range": _flatten,
    "squeeze2": lambda ins, a: {"Out": [_P().squeeze(ins["X"][0], axis=list(a.get("axes") or []) or None)]},
    "unsqueeze2": lambda ins, a: {"Out": [_P().unsqueeze(ins["X"][0], axis=list(a.get("axes") or []))]},
    "concat": lambda ins, a: {"Out": [_P().concat(ins["X"], axis=a.get("axis", 0))]},
    "stack": lambda ins, a: {"Y": [_P().stack(ins["X"], axis=a.get("axis", 0))]},
    "split": _split, "slice": _slice, "scale": _scale, "dropout": _dropout,
    "sum": lambda ins, a: {"Out": [_P().add_n(ins["X"])]},
    "assign": lambda ins, a: {"Out": [ins["X"][0]]},
    "lookup_table_v2": lambda ins, a: {"Out": [_F().embedding(ins["Ids"][0], ins["W"][0])]},
    "flash_attn_qkvpacked": lambda ins, a: {"out": [_qkvpacked(ins["qkv"][0], a)]},
    "fill_constant": _fill_constant, "cast": _cast,
    "shape": lambda ins, a: {"Out": [_P().to_tensor(list(ins["Input"][0].shape), dtype="int32")]},
    "reduce_mean": _reduce("mean"), "reduce_sum": _reduce("sum"), "reduce_max": _reduce("max"),
    "reduce_min": _reduce("min"),
    "arg_max": lambda ins, a: {"Out": [_P().argmax(ins["X"][0], axis=None if a.get("flatten") else a.get("axis"),
                                                    keepdim=bool(a.get("keepdims")))]},
    "clip": lambda ins, a: {"Out": [_P().clip(ins["X"][0], a.get("min"), a.get("max"))]},
    "gather": lambda ins, a: {"Out": [_P().gather(ins["X"][0], ins["Index"][0], axis=a.get("axis", 0))]},
    "expand_v2": lambda ins, a: {"Out": [_P().expand(ins["X"][0], list(a["shape"]))]},
    "tile": lambda ins, a: {"Out": [_P().tile(ins["X"][0], list(a["repeat_times"]))]},
    "where": lambda ins, a: {"Out": [_P().where(ins["Condition"][0], ins["X"][0], ins["Y"][0])]},
    "bilinear_interp_v2": _interp("bilinear"), "nearest_interp_v2": _interp("nearest"),
}


def _qkvpacked(qkv, a):
    """Reference flash_attn_qkvpacked: qkv [B, S, G + 2, Hk, D] (query groups, then K and V) -> [B, S, G*Hk, D]."""
    from ..framework.tensor import _wrap
    from ..ops import attention as _att
    t = qkv._t
    g = t.shape[2] - 2
    q = t[:, :, :g].transpose(2, 3).flatten(2, 3) if g > 1 else t[:, :, 0]
    return _wrap(_att.flash_attention(q, t[:, :, g], t[:, :, g + 1], causal=bool(a.get("causal", False)),
                                      dropout=0.0, training=False))


class ProgramDescRunner:
    """Runs block 0 of a reference program over this framework's ops (inference: no autograd recording)."""

    def __init__(self, program, params):
        self.program = program
        self.params = params  # name -> Tensor
        missing = sorted({o["type"] for o in program.ops} - set(OPS) - {"feed", "fetch"})
        if missing:
            raise NotImplementedError(f"reference program uses operators without a mapping: {missing}")

    def run(self, feeds):
        from . import grad_mode
        P = _P()
        env = dict(self.params)
        for i, name in enumerate(self.program.feed_names):
            v = feeds[name] if isinstance(feeds, dict) else feeds[i]
            env[name] = v if isinstance(v, P.Tensor) else P.to_tensor(np.asarray(v))
        with grad_mode.no_grad():
            for op in self.program.ops:
                if op["type"] in ("feed", "fetch"):
                    continue
                ins = {k: [env[n] for n in names if n in env] for k, names in op["inputs"].items()}
                outs = OPS[op["type"]](ins, op["attrs"])
                for k, names in op["outputs"].items():
                    vals = outs.get(k)
                    if vals is None:
                        continue  # auxiliary outputs (XShape, Mean/Variance of inference BN, ...)
                    for n, v in zip(names, vals):
                        env[n] = v
        return [env[n] for n in self.program.fetch_names]


def load(path_prefix, device=None):
    """Load a reference ``.pdmodel`` ProgramDesc + ``.pdiparams`` pair; returns a ProgramDescRunner."""
    from .combine_io import read_combined
    from .tensor import Tensor
    base = path_prefix[:-len(".pdmodel")] if path_prefix.endswith(".pdmodel") else path_prefix
    with open(base + ".pdmodel", "rb") as f:
        prog = parse(f.read())
    names = prog.persistable_names()
    tensors = read_combined(base + ".pdiparams") if names else []
    if len(tensors) != len(names):
        raise ValueError(f"{base}.pdiparams holds {len(tensors)} tensors, the program lists {len(names)} persistables")
    dev = device or _dev()
    params = {n: Tensor(t.to(dev)) for n, t in zip(names, tensors)}
    return ProgramDescRunner(prog, params)


# ------------------------------------------------------------------------------------------------- builder
def _attr(name, v):
    if isinstance(v, bool):
        return {"name": name, "type": BOOLEAN, "b": int(v)}
    if isinstance(v, int):
        return {"name": name, "type": INT, "i": v} if -2**31 <= v < 2**31 else {"name": name, "type": LONG, "l": v}
    if isinstance(v, float):
        return {"name": name, "type": FLOAT, "f": v}
    if isinstance(v, str):
        return {"name": name, "type": STRING, "s": v}
    v = list(v)
    if all(isinstance(x, bool) for x in v) and v:
        return {"name": name, "type": BOOLEANS, "bools": [int(x) for x in v]}
    if all(isinstance(x, int) for x in v):
        return {"name": name, "type": INTS, "ints": v}
    if all(isinstance(x, (int, float)) for x in v):
        return {"name": name, "type": FLOATS, "floats": [float(x) for x in v]}
    return {"name": name, "type": STRINGS, "strings": [str(x) for x in v]}


class ProgramDescBuilder:
    """Assemble a block-0 ProgramDesc (feed -> ops -> fetch) and write ``.pdmodel`` + ``.pdiparams``."""

    def __init__(self):
        self.vars = {}
        self.ops = []
        self.params = {}
        self._nfeed = self._nfetch = 0
        self._var("feed", None, [], ty=FEED_MINIBATCH, persistable=True)
        self._var("fetch", None, [], ty=FETCH_LIST, persistable=True)

    def _var(self, name, dtype, shape, ty=DENSE_TENSOR, persistable=False):
        vt = {"type": ty}
        if ty == DENSE_TENSOR:
            vt["dense_tensor"] = {"tensor": {"data_type": _PROTO[dtype], "dims": [int(s) for s in shape]}}
        self.vars[name] = {"name": name, "type": vt, "persistable": int(persistable)}

    def feed(self, name, shape, dtype=torch.float32):
        self._var(name, dtype, shape)
        self.ops.append(self._op("feed", {"X": ["feed"]}, {"Out": [name]}, {"col": self._nfeed}))
        self._nfeed += 1
        return name

    def param(self, name, value):
        t = value if isinstance(value, torch.Tensor) else torch.as_tensor(np.asarray(value))
        self._var(name, t.dtype, t.shape, persistable=True)
        self.params[name] = t.detach().cpu()
        return name

    def var(self, name, shape=(), dtype=torch.float32):
        self._var(name, dtype, shape)
        return name

    @staticmethod
    def _op(ty, inputs, outputs, attrs):
        return {"type": ty, "inputs": [{"parameter": k, "arguments": list(v)} for k, v in inputs.items()],
                "outputs": [{"parameter": k, "arguments": list(v)} for k, v in outputs.items()],
                "attrs": [_attr(k, v) for k, v in attrs.items()]}

    def op(self, ty, inputs, outputs, **attrs):
        for names in outputs.values():
            for n in names:
                if n not in self.vars:
                    self._var(n, torch.float32, [])
        self.ops.append(self._op(ty, inputs, outputs, attrs))
        return outputs

    def fetch(self, name):
        self.ops.append(self._op("fetch", {"X": [name]}, {"Out": ["fetch"]}, {"col": self._nfetch}))
        self._nfetch += 1

    def to_bytes(self):
        blk = {"idx": 0, "parent_idx": -1, "vars": list(self.vars.values()), "ops": self.ops}
        return encode({"blocks": [blk], "version": {"version": 0}})

    def save(self, path_prefix):
        import os
        from .combine_io import write_combined
        d = os.path.dirname(path_prefix)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(path_prefix + ".pdmodel", "wb") as f:
            f.write(self.to_bytes())
        names = sorted(self.params)
        write_combined(path_prefix + ".pdiparams", [self.params[n] for n in names])


# ------------------------------------------------------------------------------------------------ exporter
class _Exporter:
    """Lowers this framework's recorded static Program (static/program.py OpNodes) to reference operators."""

    def __init__(self, prog, const_names):
        self.prog, self.cn = prog, const_names
        self.b = ProgramDescBuilder()
        self.n_tmp = 0
        self.alias = {}  # slot -> feed name

    def name(self, a):
        from ..static import program as P
        if isinstance(a, P._Ref):
            return self.alias.get(a.i, f"t{a.i}")
        if isinstance(a, P._Const):
            n = self.cn[a.idx]
            if n not in self.b.params:
                self.b.param(n, self.prog._consts[a.idx])
            return n
        return None

    def ndim(self, a):
        from ..static import program as P
        if isinstance(a, P._Ref):
            return len(self.prog._metas[a.i].shape)
        return self.prog._consts[a.idx].dim()

    def tmp(self, like=None):
        """A temporary; ``like``: an already declared variable whose dtype / shape it shares (the intermediate
        of a lowered op chain, e.g. the conv output before its bias add)."""
        self.n_tmp += 1
        name = f"tmp_{self.n_tmp}"
        if like is not None and like in self.b.vars:
            self.b.vars[name] = dict(self.b.vars[like], name=name)
        return name

    def declare(self, slot):
        slot = getattr(slot, "i", slot)
        m = self.prog._metas[slot]
        name = self.alias.get(slot, f"t{slot}")
        self.b.var(name, list(m.shape), m.dtype)
        return name

    def emit(self, node):
        outs = node.outs if isinstance(node.outs, (list, tuple)) else [node.outs]
        out = [self.declare(s) for s in outs]
        key = node.name.split(":")[-1]
        fn = getattr(self, "op_" + key, None)
        if fn is None:
            raise NotImplementedError(f"no reference operator lowering for recorded op {node.name!r}")
        fn(out, list(node.args), dict(node.kwargs))

    def op(self, ty, ins, outs, **attrs):
        self.b.op(ty, ins, outs, **attrs)

    # --- lowerings (reference operator definitions: paddle/phi/ops/yaml/op_compat.yaml names / attributes)
    def op_fused_linear(self, out, a, k):
        x, w, bias, act = (a + [None, None])[:4]
        act = act or k.get("act")
        cur = out[0] if bias is None and act is None else self.tmp(like=out[0])
        self.op("matmul_v2", {"X": [self.name(x)], "Y": [self.name(w)]}, {"Out": [cur]}, trans_x=False, trans_y=False)
        if bias is not None:
            nxt = out[0] if act is None else self.tmp(like=out[0])
            self.op("elementwise_add", {"X": [cur], "Y": [self.name(bias)]}, {"Out": [nxt]}, axis=-1)
            cur = nxt
        if act is not None:
            if act.startswith("gelu"):
                self.op("gelu", {"X": [cur]}, {"Out": [out[0]]}, approximate=act != "gelu")
            else:
                self.op({"swish": "silu"}.get(act, act), {"X": [cur]}, {"Out": [out[0]]})

    def op_layer_norm(self, out, a, k):
        x, w, b, eps = a[:4]
        ins = {"X": [self.name(x)]}
        if w is not None:
            ins["Scale"] = [self.name(w)]
        if b is not None:
            ins["Bias"] = [self.name(b)]
        nd = self.ndim(w) if w is not None else 1
        self.op("layer_norm", ins, {"Y": [out[0]], "Mean": [self.tmp()], "Variance": [self.tmp()]},
                epsilon=float(eps), begin_norm_axis=self.ndim(x) - nd)

    def op_gelu(self, out, a, k):
        approx = a[1] if len(a) > 1 else k.get("approximate", False)
        self.op("gelu", {"X": [self.name(a[0])]}, {"Out": out},
                approximate=bool(approx) and approx != "none")

    def _unary(ty):
        return lambda self, out, a, k: self.op(ty, {"X": [self.name(a[0])]}, {"Out": out})
    op_relu = _unary("relu")
    op_sigmoid = _unary("sigmoid")
    op_tanh = _unary("tanh")
    op_silu = _unary("silu")
    op_exp = _unary("exp")
    op_sqrt = _unary("sqrt")
    op_rsqrt = _unary("rsqrt")
    op_abs = _unary("abs")
    op_log = _unary("log")

    def op_softmax(self, out, a, k):
        axis = a[1] if len(a) > 1 else k.get("dim", k.get("axis", -1))
        self.op("softmax", {"X": [self.name(a[0])]}, {"Out": out}, axis=int(axis))

    def _binary(ty, scale_of):
        def run(self, out, a, k):
            x, y = a[0], a[1]
            if isinstance(y, (int, float)):
                s, bias = scale_of(float(y))
                self.op("scale", {"X": [self.name(x)]}, {"Out": out}, scale=s, bias=bias, bias_after_scale=True)
            else:
                self.op(ty, {"X": [self.name(x)], "Y": [self.name(y)]}, {"Out": out}, axis=-1)
        return run
    op_add = _binary("elementwise_add", lambda v: (1.0, v))
    op_sub = _binary("elementwise_sub", lambda v: (1.0, -v))
    op_mul = _binary("elementwise_mul", lambda v: (v, 0.0))
    op_div = _binary("elementwise_div", lambda v: (1.0 / v, 0.0))
    op_true_divide = op_div

    def op_matmul(self, out, a, k):
        self.op("matmul_v2", {"X": [self.name(a[0])], "Y": [self.name(a[1])]}, {"Out": out}, trans_x=False,
                trans_y=False)

    def op_unsqueeze(self, out, a, k):
        d = a[1] if len(a) > 1 else k["dim"]
        self.op("unsqueeze2", {"X": [self.name(a[0])]}, {"Out": out, "XShape": [self.tmp()]},
                axes=[int(v) for v in (d if isinstance(d, (list, tuple)) else [d])])

    def op_permute(self, out, a, k):
        perm = list(a[1]) if len(a) == 2 and isinstance(a[1], (list, tuple)) else [int(v) for v in a[1:]]
        self.op("transpose2", {"X": [self.name(a[0])]}, {"Out": out, "XShape": [self.tmp()]}, axis=perm)

    def op_transpose(self, out, a, k):
        nd = self.ndim(a[0])
        d0, d1 = a[1] % nd, a[2] % nd
        perm = list(range(nd))
        perm[d0], perm[d1] = perm[d1], perm[d0]
        self.op("transpose2", {"X": [self.name(a[0])]}, {"Out": out, "XShape": [self.tmp()]}, axis=perm)

    def op_reshape(self, out, a, k):
        shape = list(a[1]) if len(a) == 2 and isinstance(a[1], (list, tuple)) else [int(v) for v in a[1:]]
        self.op("reshape2", {"X": [self.name(a[0])]}, {"Out": out, "XShape": [self.tmp()]},
                shape=[int(v) for v in shape])
    op_view = op_reshape

    def op_to(self, out, a, k):
        dt = next((v for v in list(a[1:]) + list(k.values()) if isinstance(v, torch.dtype)), None)
        src = self.name(a[0])
        if dt is None or src == out[0]:
            if src != out[0]:
                self.op("assign", {"X": [src]}, {"Out": out})
            if dt is None or self.prog._metas[a[0].i].dtype == dt:
                return
        self.op("cast", {"X": [src]}, {"Out": out}, in_dtype=_PROTO[self.prog._metas[a[0].i].dtype],
                out_dtype=_PROTO[dt])

    def op_cat(self, out, a, k):
        axis = a[1] if len(a) > 1 else k.get("dim", 0)
        self.op("concat", {"X": [self.name(t) for t in a[0]]}, {"Out": out}, axis=int(axis))

    def op_batch_norm(self, out, a, k):
        x, mean, var = a[:3]
        self.op("batch_norm", {"X": [self.name(x)], "Scale": [self.name(k["weight"])], "Bias": [self.name(k["bias"])],
                               "Mean": [self.name(mean)], "Variance": [self.name(var)]},
                {"Y": out}, epsilon=float(k.get("eps", 1e-5)), is_test=True, data_layout="NCHW")

    @staticmethod
    def _pair(v):
        return [int(v), int(v)] if isinstance(v, int) else [int(x) for x in v]

    def op_avg_pool2d(self, out, a, k):
        x, ks = a[0], a[1]
        stride = a[2] if len(a) > 2 and a[2] is not None else ks
        pad = a[3] if len(a) > 3 else 0
        ceil = bool(a[4]) if len(a) > 4 else False
        incl = bool(a[5]) if len(a) > 5 else True
        self.op("pool2d", {"X": [self.name(x)]}, {"Out": out}, pooling_type="avg", ksize=self._pair(ks),
                strides=self._pair(stride), paddings=self._pair(pad), global_pooling=False, adaptive=False,
                ceil_mode=ceil, exclusive=not incl, data_format="NCHW", padding_algorithm="EXPLICIT")

    def op_max_pool2d(self, out, a, k):
        x, ks = a[0], a[1]
        stride = k.get("stride", a[2] if len(a) > 2 else None) or ks
        pad = k.get("padding", a[3] if len(a) > 3 else 0)
        self.op("pool2d", {"X": [self.name(x)]}, {"Out": out}, pooling_type="max", ksize=self._pair(ks),
                strides=self._pair(stride), paddings=self._pair(pad), global_pooling=False, adaptive=False,
                ceil_mode=bool(k.get("ceil_mode", False)), exclusive=True, data_format="NCHW",
                padding_algorithm="EXPLICIT")

    def op_mean(self, out, a, k):
        dims = a[1] if len(a) > 1 else k.get("dim")
        keep = bool(k.get("keepdim", a[2] if len(a) > 2 else False))
        if dims is None:
            self.op("reduce_mean", {"X": [self.name(a[0])]}, {"Out": out}, dim=[0], keep_dim=keep, reduce_all=True)
        else:
            dims = [int(d) for d in (dims if isinstance(dims, (list, tuple)) else [dims])]
            self.op("reduce_mean", {"X": [self.name(a[0])]}, {"Out": out}, dim=dims, keep_dim=keep,
                    reduce_all=False)

    def op_conv2d(self, out, a, k):
        x, w, b = a[0], a[1], (a[2] if len(a) > 2 else None)
        stride, pad, dil, groups = (list(a[3:7]) + [1, 0, 1, 1][len(a[3:7]):])
        cur = out[0] if b is None else self.tmp(like=out[0])
        self.op("conv2d", {"Input": [self.name(x)], "Filter": [self.name(w)]}, {"Output": [cur]},
                strides=self._pair(stride), paddings=self._pair(pad), dilations=self._pair(dil), groups=int(groups),
                padding_algorithm="EXPLICIT", data_format="NCHW")
        if b is not None:
            self.op("elementwise_add", {"X": [cur], "Y": [self.name(b)]}, {"Out": out}, axis=1)

    def op_embedding(self, out, a, k):
        if k.get("max_norm") is not None:
            raise NotImplementedError("embedding with max_norm has no reference operator")
        pad = k.get("padding_idx")
        self.op("lookup_table_v2", {"Ids": [self.name(a[0])], "W": [self.name(a[1])]}, {"Out": out},
                padding_idx=-1 if pad is None else int(pad), is_sparse=bool(k.get("sparse", False)))

    def op_dropout_add(self, out, a, k):
        x, res = a[0], (a[1] if len(a) > 1 else None)
        p = float(a[2]) if len(a) > 2 else 0.0
        training = bool(a[3]) if len(a) > 3 else False
        if training and p > 0:
            raise NotImplementedError("a training-mode dropout_add cannot be exported (inference programs only)")
        if res is None:
            self.op("assign", {"X": [self.name(x)]}, {"Out": out})
        else:
            self.op("elementwise_add", {"X": [self.name(x)], "Y": [self.name(res)]}, {"Out": out}, axis=-1)

    def op_flash_attention_qkvpacked(self, out, a, k):
        """Our packing is [B, S, H, 3, D]; the reference op takes [B, S, G + 2, Hk, D] (G = H / Hk = 1 here)."""
        if k.get("training") and float(k.get("dropout", 0.0)) > 0:
            raise NotImplementedError("attention dropout cannot be exported (inference programs only)")
        x = self.name(a[0])
        t = self.tmp()
        m = self.prog._metas[a[0].i]
        B, S, H, _, D = m.shape
        self.b.var(t, [B, S, 3, H, D], m.dtype)
        self.op("transpose2", {"X": [x]}, {"Out": [t], "XShape": [self.tmp()]}, axis=[0, 1, 3, 2, 4])
        self.op("flash_attn_qkvpacked", {"qkv": [t]},
                {"out": out, "softmax": [self.tmp()], "softmax_lse": [self.tmp()], "seed_offset": [self.tmp()]},
                dropout=0.0, causal=bool(k.get("causal", a[1] if len(a) > 1 else True)), return_softmax=False,
                is_test=True, rng_name="")

    def op_linear_nt(self, out, a, k):
        self.op("matmul_v2", {"X": [self.name(a[0])], "Y": [self.name(a[1])]}, {"Out": out}, trans_x=False,
                trans_y=True)

    def op_arange(self, out, a, k):
        """A shape-only value (positions of a fixed-length program): a persistable constant."""
        vals = torch.arange(*[int(v) for v in a if isinstance(v, (int, float))])
        n = f"__arange_{'_'.join(str(int(v)) for v in a if isinstance(v, (int, float)))}"
        if n not in self.b.params:
            self.b.param(n, vals)
        self.op("assign", {"X": [n]}, {"Out": out})

    def op_flatten(self, out, a, k):
        s = a[1] if len(a) > 1 else k.get("start_dim", 0)
        e = a[2] if len(a) > 2 else k.get("end_dim", -1)
        self.op("flatten_contiguous_range", {"X": [self.name(a[0])]}, {"Out": out, "XShape": [self.tmp()]},
                start_axis=int(s), stop_axis=int(e))


def export(prog, fetch_slots, feed_names, const_names):
    """A recorded static Program (pruned to the fetch targets) as a reference ProgramDescBuilder."""
    ex = _Exporter(prog, const_names)
    b = ex.b
    for name in feed_names:
        slot, shape, dtype = prog.feeds[name]
        ex.alias[slot] = name
        b.feed(name, list(shape), getattr(torch, dtype))
    for n in prog.nodes:
        ex.emit(n)
    for s in fetch_slots:
        b.fetch(ex.alias.get(s, f"t{s}"))
    return b
