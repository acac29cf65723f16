"""PIR program JSON: the program format of Paddle 3.x inference / jit models (``<prefix>.json`` next to the
``<prefix>.pdiparams`` parameters).

Reference schema (re-implemented, nothing imported):
  paddle/fluid/pir/serialize_deserialize/include/schema.h   key strings ("#", "%", "I", "O", "A", "OA", "TT",
                                                            "N", "AT", "D", "VD", "p", ...)
  .../src/interface.cc      file = {"base_code": {"magic": "pir", "version": N, "trainable": b}, "program": ...}
  .../src/ir_serialize.cc   program -> regions -> blocks -> ops; value ids count up from 1, block args down
                            from -1; builtin.parameter is compressed to {"#": "p", "O": value, "A": [is_distributed,
                            is_parameter, need_clip, name], "OA": [persistable, stop_gradient, trainable]}
  .../src/schema.cc         dialect ids: builtin "0", pd_op "1", cf "2", custom_op "3", pd_dist "4"
  .../include/serialize_utils.h  types {"#": "0.t_dtensor", "D": [dtype type, dims, layout, lod, offset]},
                            attributes {"#": "<dialect>.a_<kind>", "D": data} (+ "VD" for nan / inf floats)
  python/paddle/static/pir_io.py:743  save_inference_model_pir: params in save_combine layout, sorted by name
Operand layout of each pd_op operation: its tensor arguments in ops.yaml order, then its mutable attributes
(IntArray / Scalar arguments that op_compat.yaml marks support_tensor / tensor_name) as operands produced by
pd_op.full_int_array / pd_op.full — the table _MUTABLE below.

Writing lowers the legacy-operator stream of program_desc.ProgramDescBuilder (this framework's static Program
export) to pd_op operations. Reading runs block 0 of the program over this framework's ops (PirRunner).
"""
from __future__ import annotations

import json
import math
import os

import numpy as np
import torch

MAGIC = "pir"
VERSION = 1  # save_inference_model_pir writes pir_version 1

_DT_NAME = {torch.float32: "float32", torch.float16: "float16", torch.bfloat16: "bfloat16", torch.float64: "float64",
            torch.int8: "int8", torch.uint8: "uint8", torch.int16: "int16", torch.int32: "int32",
            torch.int64: "int64", torch.bool: "bool", torch.complex64: "complex64", torch.complex128: "complex128"}
_FROM_DT_NAME = {v: k for k, v in _DT_NAME.items()}
_TYPE_OF = {"float32": "t_f32", "float16": "t_f16", "bfloat16": "t_bf16", "float64": "t_f64", "int8": "t_i8",
            "uint8": "t_ui8", "int16": "t_i16", "int32": "t_i32", "int64": "t_i64", "bool": "t_bool",
            "complex64": "t_c64", "complex128": "t_c128", "float8_e4m3fn": "t_f8e4m3fn", "float8_e5m2": "t_f8e5m2"}
_DT_OF_TYPE = {v: k for k, v in _TYPE_OF.items()}

# ops.yaml tensor arguments (operand order) and mutable attributes (extra operands, after the tensors)
_MUTABLE = {"scale": ["scale"], "reshape": ["shape"], "pool2d": ["kernel_size"], "concat": ["axis"],
            "unsqueeze": ["axis"], "squeeze": ["axis"], "split": ["sections", "axis"], "slice": ["starts", "ends"],
            "sum": ["axis"], "max": ["axis"], "min": ["axis"], "expand": ["shape"], "tile": ["repeat_times"],
            "split_with_num": ["axis"], "gather": ["axis"], "clip": ["min", "max"], "argmax": ["axis"],
            "full_like": ["value"], "dropout": ["p"], "prod": ["axis"], "cumsum": ["axis"]}


# ------------------------------------------------------------------------------------------- type / attribute codec
def dtensor(dtype, shape, layout="NCHW"):
    dt = dtype if isinstance(dtype, str) else _DT_NAME[dtype]
    return {"#": "0.t_dtensor", "D": [{"#": "0." + _TYPE_OF[dt]}, [int(s) for s in shape], layout, [], 0]}


def vec_type(types):
    return {"#": "0.t_vec", "D": list(types)}


def _float_attr(kind, v):
    v = float(v)
    if math.isnan(v):
        return {"#": kind, "VD": "NaN"}
    if math.isinf(v):
        return {"#": kind, "VD": "INF" if v > 0 else "-INF"}
    return {"#": kind, "D": v}


def a_bool(v):
    return {"#": "0.a_bool", "D": bool(v)}


def a_i32(v):
    return {"#": "0.a_i32", "D": int(v)}


def a_i64(v):
    return {"#": "0.a_i64", "D": int(v)}


def a_f32(v):
    return _float_attr("0.a_f32", v)


def a_f64(v):
    return _float_attr("0.a_f64", v)


def a_str(v):
    return {"#": "0.a_str", "D": str(v)}


def a_array(items):
    return {"#": "0.a_array", "D": list(items)}


def a_intarray(v):
    return {"#": "1.a_intarray", "D": [int(x) for x in v]}


def a_dtype(dt):
    return {"#": "1.a_dtype", "D": dt if isinstance(dt, str) else _DT_NAME[dt]}


def a_place(kind=0, dev_id=0, dev_type=""):
    # phi::AllocationType: 0 UNDEFINED, 1 CPU, 2 GPU, 3 GPUPINNED ...; UNDEFINED = "use the executor's place"
    return {"#": "1.a_place", "D": [int(kind), int(dev_id), dev_type]}


def a_scalar(v, dt="float32"):
    return {"#": "1.a_scalar", "D": [dt, v]}


def decode_attr(a):
    """pir attribute json -> python value."""
    if a is None:
        return None
    kind = a.get("#", "")
    tag = kind.split(".", 1)[-1]
    if "VD" in a:
        return {"NaN": float("nan"), "INF": float("inf"), "-INF": float("-inf")}[a["VD"]]
    d = a.get("D")
    if tag == "a_array":
        return [decode_attr(x) for x in d]
    if tag == "a_scalar":
        return d[1] if len(d) == 2 else complex(d[1], d[2])
    if tag in ("a_c64", "a_c128"):
        return complex(d[0], d[1])
    if tag == "a_dtype":
        return d
    if tag == "a_type":
        return d
    return d


def decode_type(t):
    """pir type json -> (dtype name, shape) for dense tensors, [..] for vectors, None otherwise."""
    if t is None or t.get("#") == "NULL":
        return None
    tag = t["#"].split(".", 1)[-1]
    if tag == "t_dtensor":
        d = t["D"]
        return _DT_OF_TYPE.get(d[0]["#"].split(".", 1)[-1], "float32"), list(d[1])
    if tag == "t_vec":
        return [decode_type(x) for x in t["D"]]
    if tag in _DT_OF_TYPE:
        return _DT_OF_TYPE[tag], []
    return None


# ------------------------------------------------------------------------------------------- writer
class PirWriter:
    """Builds one PIR program (a single region / block) in the reference JSON schema."""

    def __init__(self, trainable=False):
        self.ops = []
        self.next_id = 1
        self.trainable = trainable
        self.types = {}   # value id -> type json
        self.params = {}  # name -> tensor (written to .pdiparams sorted by name)

    def _value(self, ty):
        vid = self.next_id
        self.next_id += 1
        self.types[vid] = ty
        return vid

    def op(self, name, operands, attrs, out_types):
        """Append ``1.<name>`` (or a full "<dialect>.<name>") with operand value ids, attrs {name: attr json}
        and output types; returns the output value ids."""
        full = name if "." in name else "1." + name
        outs = [self._value(t) for t in out_types]
        op = {"#": full, "I": [{"%": (0 if v is None else v)} for v in operands],
              "O": [{"%": v, "TT": self.types[v]} for v in outs],
              "A": [{"N": k, "AT": v} for k, v in attrs.items()]}
        if self.trainable:
            op["OA"] = [{"N": "stop_gradient", "AT": a_array([a_bool(True) for _ in outs])}]
        self.ops.append(op)
        return outs

    def parameter(self, name, tensor):
        self.params[name] = tensor.detach().cpu()
        vid = self._value(dtensor(tensor.dtype, tensor.shape))
        op = {"#": "p", "O": {"%": vid, "TT": self.types[vid]}, "A": [0, 1, 0, name], "DA": [], "QA": []}
        if self.trainable:
            op["OA"] = [1, 1, 1]
        self.ops.append(op)
        return vid

    def data(self, name, shape, dtype):
        return self.op("data", [], {"name": a_str(name), "shape": a_intarray(shape), "dtype": a_dtype(dtype),
                                    "place": a_place()}, [dtensor(dtype, shape)])[0]

    def fetch(self, vid, name, col):
        return self.op("fetch", [vid], {"name": a_str(name), "col": a_i32(col), "persistable": a_array([a_bool(True)])},
                       [self.types[vid]])[0]

    def full_int_array(self, values, dtype="int64"):
        return self.op("full_int_array", [], {"value": a_array([a_i64(v) for v in values]), "dtype": a_dtype(dtype),
                                              "place": a_place(1)}, [dtensor(dtype, [len(values)])])[0]

    def full(self, shape, value, dtype="float32"):
        return self.op("full", [], {"shape": a_intarray(shape), "value": a_f64(value), "dtype": a_dtype(dtype),
                                    "place": a_place(1)}, [dtensor(dtype, shape)])[0]

    def block(self, args_types=()):
        """Open a sub-block (for if_ / while_): ops appended until the matching end_block() go into it; its
        arguments (block-argument ids count down from -1) are returned."""
        if not hasattr(self, "_stack"):
            self._stack, self._next_arg = [], -1
        args = []
        for ty in args_types:
            args.append(self._next_arg)
            self.types[self._next_arg] = ty
            self._next_arg -= 1
        self._stack.append((self.ops, args))
        self.ops = []
        return args

    def end_block(self, yields):
        self.op("2.yield", list(yields), {}, [])
        ops, (outer, args) = self.ops, self._stack.pop()
        self.ops = outer
        return {"#": f"block_{len(self._stack)}", "args": [{"#": a, "TT": self.types[a]} for a in args], "ops": ops}

    def if_(self, cond, true_block, false_block, out_types):
        """pd_op.if with two closed blocks (from end_block); returns the result ids."""
        outs = self.op("if", [cond], {}, out_types)
        self.ops[-1]["regions"] = [{"#": "region_t", "blocks": [true_block]}, {"#": "region_f", "blocks": [false_block]}]
        return outs

    def while_(self, cond, vids, body_block):
        """pd_op.while over loop values ``vids`` (body args = their values per iteration, body yields the next
        condition then the next values); returns the result ids."""
        outs = self.op("while", [cond] + list(vids), {}, [self.types[v] for v in vids])
        self.ops[-1]["regions"] = [{"#": "region_w", "blocks": [body_block]}]
        return outs

    def combine(self, vids):
        return self.op("0.combine", list(vids), {}, [vec_type([self.types[v] for v in vids])])[0]

    def to_json(self):
        return {"base_code": {"magic": MAGIC, "version": VERSION, "trainable": bool(self.trainable)},
                "program": {"regions": [{"#": "region_0", "blocks": [{"#": "block_0", "args": [],
                                                                      "ops": self.ops}]}]}}

    def save(self, path_prefix):
        from .combine_io import write_combined
        d = os.path.dirname(path_prefix)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(path_prefix + ".json", "w") as f:
            json.dump(self.to_json(), f)
        names = sorted(self.params)
        write_combined(path_prefix + ".pdiparams", [self.params[n] for n in names])


def _la(op):
    """legacy op dict (program_desc builder form) -> (inputs {slot: [names]}, outputs, attrs {name: value})."""
    ins = {e["parameter"]: list(e["arguments"]) for e in op["inputs"]}
    outs = {e["parameter"]: list(e["arguments"]) for e in op["outputs"]}
    attrs = {}
    for a in op["attrs"]:
        v = None
        for k in ("b", "i", "l", "f", "s", "ints", "floats", "strings", "bools"):
            if k in a:
                v = a[k]
                break
        if "b" in a:
            v = bool(a["b"])
        if "bools" in a:
            v = [bool(x) for x in a["bools"]]
        attrs[a["name"]] = v
    return ins, outs, attrs


def from_builder(b, trainable=False):
    """Lower a program_desc.ProgramDescBuilder (block 0: feed -> legacy ops -> fetch) to a PirWriter."""
    from . import program_desc as PD
    w = PirWriter(trainable)
    env = {}
    meta = {}
    for name, v in b.vars.items():
        vt = v["type"]
        if vt.get("type") == PD.DENSE_TENSOR:
            td = vt["dense_tensor"]["tensor"]
            meta[name] = (_DT_NAME[PD._FROM_PROTO[td["data_type"]]], list(td.get("dims", [])))
    for name in sorted(b.params):
        env[name] = w.parameter(name, b.params[name])

    def ty(name):
        dt, shape = meta.get(name, ("float32", []))
        return dtensor(dt, shape)

    def put(names, vids):
        for n, v in zip(names, vids):
            env[n] = v

    for op in b.ops:
        t = op["type"]
        ins, outs, at = _la(op)
        X = lambda k="X", i=0: env[ins[k][i]]  # noqa: E731
        o = outs.get("Out", [None])
        if t == "feed":
            dt, shape = meta[o[0]]
            env[o[0]] = w.data(o[0], shape, dt)
        elif t == "fetch":
            w.fetch(env[ins["X"][0]], ins["X"][0], at.get("col", 0))
        elif t == "matmul_v2":
            put(o, w.op("matmul", [X(), X("Y")], {"transpose_x": a_bool(at.get("trans_x", False)),
                                                   "transpose_y": a_bool(at.get("trans_y", False))}, [ty(o[0])]))
        elif t in ("elementwise_add", "elementwise_sub", "elementwise_mul", "elementwise_div"):
            y = X("Y")
            axis = at.get("axis", -1)
            xs = meta.get(ins["X"][0], (None, []))[1]
            ys = meta.get(ins["Y"][0], (None, []))[1]
            if axis not in (-1, None) and len(ys) < len(xs) and axis + len(ys) < len(xs):
                # legacy broadcast from `axis`: reshape Y to line up with X
                shape = [1] * axis + list(ys) + [1] * (len(xs) - axis - len(ys))
                y = w.op("reshape", [y, w.full_int_array(shape)], {}, [dtensor(meta[ins["Y"][0]][0], shape)])[0]
            name = {"elementwise_add": "add", "elementwise_sub": "subtract", "elementwise_mul": "multiply",
                    "elementwise_div": "divide"}[t]
            put(o, w.op(name, [X(), y], {}, [ty(o[0])]))
        elif t in ("relu", "sigmoid", "tanh", "silu", "exp", "sqrt", "rsqrt", "abs", "log", "assign"):
            put(o, w.op(t, [X()], {}, [ty(o[0])]))
        elif t == "gelu":
            put(o, w.op("gelu", [X()], {"approximate": a_bool(at.get("approximate", False))}, [ty(o[0])]))
        elif t == "softmax":
            put(o, w.op("softmax", [X()], {"axis": a_i32(at.get("axis", -1))}, [ty(o[0])]))
        elif t == "layer_norm":
            y = outs["Y"]
            ops_ = [X(), env[ins["Scale"][0]] if "Scale" in ins else None, env[ins["Bias"][0]] if "Bias" in ins else None]
            r = w.op("layer_norm", ops_, {"epsilon": a_f32(at.get("epsilon", 1e-5)),
                                          "begin_norm_axis": a_i32(at.get("begin_norm_axis", 1))},
                     [ty(y[0]), dtensor("float32", []), dtensor("float32", [])])
            env[y[0]] = r[0]
        elif t == "scale":
            s = w.full([1], at.get("scale", 1.0))
            put(o, w.op("scale", [X(), s], {"bias": a_f32(at.get("bias", 0.0)),
                                            "bias_after_scale": a_bool(at.get("bias_after_scale", True))}, [ty(o[0])]))
        elif t == "reshape2":
            put(o, w.op("reshape", [X(), w.full_int_array(at["shape"])], {}, [ty(o[0])]))
        elif t == "transpose2":
            put(o, w.op("transpose", [X()], {"perm": a_array([a_i32(v) for v in at["axis"]])}, [ty(o[0])]))
        elif t in ("unsqueeze2", "squeeze2"):
            put(o, w.op(t[:-1], [X(), w.full_int_array(at.get("axes") or [])], {}, [ty(o[0])]))
        elif t == "flatten_contiguous_range":
            put(o, w.op("flatten", [X()], {"start_axis": a_i32(at["start_axis"]), "stop_axis": a_i32(at["stop_axis"])},
                        [ty(o[0])]))
        elif t == "concat":
            c = w.combine([env[n] for n in ins["X"]])
            put(o, w.op("concat", [c, w.full([1], at.get("axis", 0), "int32")], {}, [ty(o[0])]))
        elif t == "cast":
            from .combine_io import _FROM_PROTO
            put(o, w.op("cast", [X()], {"dtype": a_dtype(_DT_NAME[_FROM_PROTO[at["out_dtype"]]])}, [ty(o[0])]))
        elif t == "conv2d":
            out = outs["Output"]
            put(out, w.op("conv2d", [env[ins["Input"][0]], env[ins["Filter"][0]]],
                          {"strides": a_array([a_i32(v) for v in at["strides"]]),
                           "paddings": a_array([a_i32(v) for v in at["paddings"]]),
                           "padding_algorithm": a_str(at.get("padding_algorithm", "EXPLICIT")),
                           "dilations": a_array([a_i32(v) for v in at["dilations"]]),
                           "groups": a_i32(at.get("groups", 1)), "data_format": a_str(at.get("data_format", "NCHW"))},
                          [ty(out[0])]))
        elif t == "batch_norm":
            y = outs["Y"]
            f32 = dtensor("float32", [])
            r = w.op("batch_norm_", [X(), env[ins["Mean"][0]], env[ins["Variance"][0]], env[ins["Scale"][0]],
                                     env[ins["Bias"][0]]],
                     {"is_test": a_bool(True), "momentum": a_f32(0.9), "epsilon": a_f32(at.get("epsilon", 1e-5)),
                      "data_format": a_str(at.get("data_layout", "NCHW")), "use_global_stats": a_bool(False),
                      "trainable_statistics": a_bool(False)}, [ty(y[0])] + [f32] * 5)
            env[y[0]] = r[0]
        elif t == "pool2d":
            put(o, w.op("pool2d", [X(), w.full_int_array(at["ksize"])],
                        {"strides": a_array([a_i32(v) for v in at["strides"]]),
                         "paddings": a_array([a_i32(v) for v in at["paddings"]]),
                         "ceil_mode": a_bool(at.get("ceil_mode", False)), "exclusive": a_bool(at.get("exclusive", True)),
                         "data_format": a_str(at.get("data_format", "NCHW")), "pooling_type": a_str(at["pooling_type"]),
                         "global_pooling": a_bool(at.get("global_pooling", False)),
                         "adaptive": a_bool(at.get("adaptive", False)),
                         "padding_algorithm": a_str(at.get("padding_algorithm", "EXPLICIT"))}, [ty(o[0])]))
        elif t == "lookup_table_v2":
            put(o, w.op("embedding", [X("Ids"), X("W")], {"padding_idx": a_i64(at.get("padding_idx", -1)),
                                                           "sparse": a_bool(at.get("is_sparse", False))}, [ty(o[0])]))
        elif t == "flash_attn_qkvpacked":
            res = outs["out"]
            f32 = dtensor("float32", [])
            r = w.op("flash_attn_qkvpacked", [X("qkv"), None, None],
                     {"dropout": a_f32(at.get("dropout", 0.0)), "causal": a_bool(at.get("causal", False)),
                      "return_softmax": a_bool(False), "is_test": a_bool(True), "rng_name": a_str("")},
                     [ty(res[0]), f32, f32, dtensor("int64", [2])])
            env[res[0]] = r[0]
        elif t == "reduce_mean":
            axis = [] if at.get("reduce_all") else list(at.get("dim") or [])
            put(o, w.op("mean", [X()], {"axis": a_intarray(axis), "keepdim": a_bool(at.get("keep_dim", False))},
                        [ty(o[0])]))
        else:
            raise NotImplementedError(f"no PIR lowering for legacy operator {t!r}")
    return w


# ------------------------------------------------------------------------------------------- reader / runner
class PirOp(tuple):
    """(name, operand ids, result ids, attrs, result types) — plus ``regions``: the op's sub-blocks (pd_op.if:
    true / false block; pd_op.while: body block), each a PirBlock."""

    def __new__(cls, name, operands, results, attrs, types, regions=()):
        o = super().__new__(cls, (name, operands, results, attrs, types))
        o.regions = list(regions)
        return o


class PirBlock:
    """One block: argument value ids (block arguments count down from -1) and its ops."""

    def __init__(self, args, ops):
        self.args, self.ops = args, ops

    def yields(self):
        """Operand ids of the block's terminating cf.yield ([] when it has none)."""
        return list(self.ops[-1][1]) if self.ops and self.ops[-1][0] == "cf.yield" else []


_DIALECTS = {"0": "builtin", "1": "pd_op", "2": "cf", "3": "custom_op", "4": "pd_dist"}


class PirProgram:
    """Block 0 of a PIR JSON program: ops as (name, operand ids, result ids, attrs, result types); control-flow ops
    (pd_op.if / pd_op.while) carry their sub-blocks (reference ir_serialize.cc WriteOp: an op's "regions")."""

    def __init__(self, data):
        if not (isinstance(data, dict) and data.get("base_code", {}).get("magic") == MAGIC):
            raise ValueError("not a PIR program (base_code.magic != 'pir')")
        self.version = data["base_code"].get("version")
        self.trainable = bool(data["base_code"].get("trainable", False))
        self.params = []  # (name, value id, (dtype, shape)) in program order
        self.feed_names, self.fetch = [], []
        self.ops = self._block(data["program"]["regions"][0]["blocks"][0], top=True).ops

    def _block(self, bj, top=False):
        ops = []
        for op in bj["ops"]:
            name = op["#"]
            if name == "p":
                res = op["O"]
                pname = op["A"][3]
                self.params.append((pname, res["%"], decode_type(res.get("TT"))))
                ops.append(PirOp("builtin.parameter", [], [res["%"]], {"parameter_name": pname}, [res.get("TT")]))
                continue
            dialect, _, short = name.partition(".")
            full = _DIALECTS.get(dialect, dialect) + "." + short
            operands = [x["%"] for x in op.get("I", [])]
            results = [x["%"] for x in op.get("O", [])]
            attrs = {a["N"]: decode_attr(a["AT"]) for a in op.get("A", [])}
            regions = [self._block(r["blocks"][0]) for r in op.get("regions", []) if r.get("blocks")]
            ops.append(PirOp(full, operands, results, attrs, [x.get("TT") for x in op.get("O", [])], regions))
            if not top:
                continue
            if full in ("pd_op.data", "pd_op.feed"):
                self.feed_names.append(attrs["name"])
            elif full == "pd_op.fetch":
                self.fetch.append((attrs.get("name", f"fetch{len(self.fetch)}"), operands[0]))
        return PirBlock([a["#"] for a in bj.get("args", [])], ops)

    def all_ops(self):
        """Every op of the program, sub-blocks included (depth first)."""
        def walk(ops):
            for o in ops:
                yield o
                for b in getattr(o, "regions", ()):
                    yield from walk(b.ops)
        return list(walk(self.ops))

    @property
    def fetch_names(self):
        return [n for n, _ in self.fetch]

    def param_names_sorted(self):
        return sorted(n for n, _, _ in self.params)


def is_pir_json(path):
    try:
        with open(path, "rb") as f:
            head = f.read(4096)
        return b'"base_code"' in head and b'"pir"' in head
    except OSError:
        return False


def _F():
    from ..nn import functional as F
    return F


def _P():
    import paddlepaddle_amd as paddle
    return paddle


def _ints(v):
    if v is None:
        return []
    if hasattr(v, "numpy"):
        return [int(x) for x in np.asarray(v.numpy()).reshape(-1)]
    return [int(x) for x in (v if isinstance(v, (list, tuple)) else [v])]


def _scalar(v):
    if hasattr(v, "numpy"):
        return np.asarray(v.numpy()).reshape(-1)[0].item()
    return v


def _pool2d(x, ks, a):
    F = _F()
    ks = _ints(ks)
    fmt = a.get("data_format", "NCHW")
    if a.get("global_pooling") or (a.get("adaptive") and ks == [1, 1]):
        return (F.adaptive_avg_pool2d if a.get("pooling_type") == "avg" else F.adaptive_max_pool2d)(
            x, 1, data_format=fmt) if fmt == "NCHW" or a.get("pooling_type") == "avg" else F.adaptive_max_pool2d(x, 1)
    if a.get("adaptive"):
        return (F.adaptive_avg_pool2d if a.get("pooling_type") == "avg" else F.adaptive_max_pool2d)(x, ks)
    pads = list(a.get("paddings") or [0, 0])
    pad = pads[:2] if len(pads) == 4 and pads[0] == pads[1] and pads[2] == pads[3] else pads
    if len(pads) == 4 and pads[0] == pads[1] and pads[2] == pads[3]:
        pad = [pads[0], pads[2]]
    if a.get("pooling_type") == "max":
        return F.max_pool2d(x, ks, stride=list(a.get("strides")), padding=pad, ceil_mode=a.get("ceil_mode", False),
                            data_format=fmt)
    return F.avg_pool2d(x, ks, stride=list(a.get("strides")), padding=pad, ceil_mode=a.get("ceil_mode", False),
                        exclusive=a.get("exclusive", True), data_format=fmt)


def _bn(ins, a):
    x, mean, var, scale, bias = ins[:5]
    return [_F().batch_norm(x, mean, var, weight=scale, bias=bias, training=False, epsilon=a.get("epsilon", 1e-5),
                            data_format=a.get("data_format", "NCHW"))]


def _ln(ins, a):
    x, w, b = (ins + [None, None])[:3]
    axis = a.get("begin_norm_axis", 1)
    shape = x.shape[axis:]
    return [_F().layer_norm(x, shape, weight=w, bias=b, epsilon=a.get("epsilon", 1e-5))]


def _full(ins, a):
    dt = a.get("dtype", "float32")
    return [_P().full(list(a.get("shape") or []), a.get("value", 0.0), dtype=dt)]


def _full_int_array(ins, a):
    return [_P().to_tensor(np.asarray([int(v) for v in a.get("value") or []], dtype=a.get("dtype", "int64")))]


def _slice(ins, a):
    x, starts, ends = ins[0], _ints(ins[1]), _ints(ins[2])
    out = _P().slice(x, list(a.get("axes") or []), starts, ends)
    dec = list(a.get("decrease_axis") or [])
    if dec:
        out = _P().squeeze(out, axis=dec)
    return [out]


def _split(ins, a):
    return list(_P().split(ins[0], _ints(ins[1]), axis=int(_scalar(ins[2]))))


def _interp(mode):
    def run(ins, a):
        x = ins[0]
        size = [int(a.get("out_h", -1)), int(a.get("out_w", -1))]
        scale = a.get("scale") or None
        kw = {"data_format": a.get("data_format", "NCHW"), "mode": mode,
              "align_corners": bool(a.get("align_corners", False))}
        if size[0] > 0:
            return [_F().interpolate(x, size=size, **kw)]
        return [_F().interpolate(x, scale_factor=list(scale), **kw)]
    return run


def _un(fn):
    return lambda ins, a: [fn(ins[0])]


def _flash_attn(ins, a):
    from .program_desc import _qkvpacked
    from ..ops import attention as _att
    from .tensor import _wrap
    mask = ins[4]._t if len(ins) > 4 and ins[4] is not None else None  # additive / boolean [B|1, H|1, Sq, Sk]
    q, k, v = ins[0], ins[1], ins[2]
    return [_wrap(_att.flash_attention(q._t, k._t, v._t, causal=bool(a.get("causal", False)), mask=mask,
                                       dropout=0.0, training=False))]


_RUN = {
    "pd_op.embedding": lambda ins, a: [_F().embedding(ins[0], ins[1])],
    "pd_op.flash_attn": _flash_attn,
    "pd_op.flash_attn_qkvpacked": lambda ins, a: [__import__(
        "paddlepaddle_amd.framework.program_desc", fromlist=["_qkvpacked"])._qkvpacked(ins[0], a)],
    "pd_op.full": _full, "pd_op.full_int_array": _full_int_array,
    "pd_op.full_like": lambda ins, a: [_P().full_like(ins[0], _scalar(ins[1]), dtype=a.get("dtype") or None)],
    "pd_op.assign": lambda ins, a: [ins[0]],
    "pd_op.less_than": lambda ins, a: [_P().less_than(ins[0], ins[1])],
    "pd_op.less_equal": lambda ins, a: [_P().less_equal(ins[0], ins[1])],
    "pd_op.greater_than": lambda ins, a: [_P().greater_than(ins[0], ins[1])],
    "pd_op.greater_equal": lambda ins, a: [_P().greater_equal(ins[0], ins[1])],
    "pd_op.equal": lambda ins, a: [_P().equal(ins[0], ins[1])],
    "pd_op.not_equal": lambda ins, a: [_P().not_equal(ins[0], ins[1])],
    "pd_op.logical_and": lambda ins, a: [_P().logical_and(ins[0], ins[1])],
    "pd_op.logical_or": lambda ins, a: [_P().logical_or(ins[0], ins[1])],
    "pd_op.logical_not": lambda ins, a: [_P().logical_not(ins[0])],
    # increment_ runs out of place: the result is a new value (no aliasing of the loop's input)
    "pd_op.increment": lambda ins, a: [ins[0] + a.get("value", 1.0)],
    "pd_op.increment_": lambda ins, a: [ins[0] + a.get("value", 1.0)],
    "pd_op.matmul": lambda ins, a: [_P().matmul(ins[0], ins[1], transpose_x=a.get("transpose_x", False),
                                                transpose_y=a.get("transpose_y", False))],
    "pd_op.add": lambda ins, a: [ins[0] + ins[1]], "pd_op.subtract": lambda ins, a: [ins[0] - ins[1]],
    "pd_op.multiply": lambda ins, a: [ins[0] * ins[1]], "pd_op.divide": lambda ins, a: [ins[0] / ins[1]],
    "pd_op.maximum": lambda ins, a: [_P().maximum(ins[0], ins[1])],
    "pd_op.minimum": lambda ins, a: [_P().minimum(ins[0], ins[1])],
    "pd_op.elementwise_pow": lambda ins, a: [ins[0] ** ins[1]],
    "pd_op.pow": lambda ins, a: [ins[0] ** a.get("y", 1.0)],
    "pd_op.relu": _un(lambda x: _F().relu(x)), "pd_op.relu6": _un(lambda x: _F().relu6(x)),
    "pd_op.sigmoid": _un(lambda x: _F().sigmoid(x)), "pd_op.tanh": _un(lambda x: _P().tanh(x)),
    "pd_op.silu": _un(lambda x: _F().silu(x)), "pd_op.swish": _un(lambda x: _F().silu(x)),
    "pd_op.exp": _un(lambda x: _P().exp(x)), "pd_op.sqrt": _un(lambda x: _P().sqrt(x)),
    "pd_op.rsqrt": _un(lambda x: _P().rsqrt(x)), "pd_op.abs": _un(lambda x: _P().abs(x)),
    "pd_op.log": _un(lambda x: _P().log(x)), "pd_op.square": _un(lambda x: x * x),
    "pd_op.hardswish": _un(lambda x: _F().hardswish(x)), "pd_op.hardsigmoid": lambda ins, a: [
        _F().hardsigmoid(ins[0], a.get("slope", 0.1666667), a.get("offset", 0.5))],
    "pd_op.leaky_relu": lambda ins, a: [_F().leaky_relu(ins[0], a.get("negative_slope", 0.02))],
    "pd_op.elu": lambda ins, a: [_F().elu(ins[0], a.get("alpha", 1.0))],
    "pd_op.gelu": lambda ins, a: [_F().gelu(ins[0], approximate=bool(a.get("approximate", False)))],
    "pd_op.softmax": lambda ins, a: [_F().softmax(ins[0], axis=a.get("axis", -1))],
    "pd_op.log_softmax": lambda ins, a: [_F().log_softmax(ins[0], axis=a.get("axis", -1))],
    "pd_op.layer_norm": _ln, "pd_op.batch_norm": _bn, "pd_op.batch_norm_": _bn,
    "pd_op.rms_norm": lambda ins, a: [_P().incubate.nn.functional.fused_rms_norm(
        ins[0], ins[3] if len(ins) > 3 else None, None, a.get("epsilon", 1e-6), a.get("begin_norm_axis", 1))[0]],
    "pd_op.scale": lambda ins, a: [_P().scale(ins[0], float(_scalar(ins[1])) if len(ins) > 1 else a.get("scale", 1.0),
                                              bias=a.get("bias", 0.0),
                                              bias_after_scale=a.get("bias_after_scale", True))],
    "pd_op.reshape": lambda ins, a: [_P().reshape(ins[0], _ints(ins[1]) if len(ins) > 1 else list(a["shape"]))],
    "pd_op.transpose": lambda ins, a: [_P().transpose(ins[0], list(a["perm"]))],
    "pd_op.unsqueeze": lambda ins, a: [_P().unsqueeze(ins[0], _ints(ins[1]) if len(ins) > 1 else a.get("axis"))],
    "pd_op.squeeze": lambda ins, a: [_P().squeeze(ins[0], _ints(ins[1]) if len(ins) > 1 else (a.get("axis") or None))],
    "pd_op.flatten": lambda ins, a: [_P().flatten(ins[0], a.get("start_axis", 1), a.get("stop_axis", 1))],
    "pd_op.concat": lambda ins, a: [_P().concat(ins[0], axis=int(_scalar(ins[1])) if len(ins) > 1 else 0)],
    "pd_op.stack": lambda ins, a: [_P().stack(ins[0], axis=a.get("axis", 0))],
    "pd_op.split": _split,
    "pd_op.split_with_num": lambda ins, a: list(_P().split(ins[0], a["num"], axis=int(_scalar(ins[1])))),
    "pd_op.slice": _slice,
    "pd_op.cast": lambda ins, a: [_P().cast(ins[0], a["dtype"])],
    "pd_op.conv2d": lambda ins, a: [_F().conv2d(
        ins[0], ins[1], stride=list(a.get("strides", [1, 1])), padding=list(a.get("paddings", [0, 0])),
        dilation=list(a.get("dilations", [1, 1])), groups=a.get("groups", 1), data_format=a.get("data_format", "NCHW"))],
    "pd_op.depthwise_conv2d": lambda ins, a: [_F().conv2d(
        ins[0], ins[1], stride=list(a.get("strides", [1, 1])), padding=list(a.get("paddings", [0, 0])),
        dilation=list(a.get("dilations", [1, 1])), groups=a.get("groups", 1), data_format=a.get("data_format", "NCHW"))],
    "pd_op.pool2d": lambda ins, a: [_pool2d(ins[0], ins[1], a)],
    "pd_op.mean": lambda ins, a: [_P().mean(ins[0], axis=list(a.get("axis") or []) or None,
                                            keepdim=a.get("keepdim", False))],
    "pd_op.sum": lambda ins, a: [_P().sum(ins[0], axis=_ints(ins[1]) or None if len(ins) > 1 else None,
                                          keepdim=a.get("keepdim", False))],
    "pd_op.max": lambda ins, a: [_P().max(ins[0], axis=_ints(ins[1]) or None, keepdim=a.get("keepdim", False))],
    "pd_op.min": lambda ins, a: [_P().min(ins[0], axis=_ints(ins[1]) or None, keepdim=a.get("keepdim", False))],
    "pd_op.argmax": lambda ins, a: [_P().argmax(ins[0], axis=None if a.get("flatten") else int(_scalar(ins[1])),
                                                keepdim=a.get("keepdims", False))],
    "pd_op.embedding": lambda ins, a: [_F().embedding(ins[0], ins[1])],
    "pd_op.gather": lambda ins, a: [_P().gather(ins[0], ins[1], axis=int(_scalar(ins[2])) if len(ins) > 2 else 0)],
    "pd_op.expand": lambda ins, a: [_P().expand(ins[0], _ints(ins[1]))],
    "pd_op.tile": lambda ins, a: [_P().tile(ins[0], _ints(ins[1]))],
    "pd_op.where": lambda ins, a: [_P().where(ins[0], ins[1], ins[2])],
    "pd_op.clip": lambda ins, a: [_P().clip(ins[0], _scalar(ins[1]), _scalar(ins[2]))],
    "pd_op.dropout": lambda ins, a: [ins[0], None],
    "pd_op.bilinear_interp": _interp("bilinear"), "pd_op.nearest_interp": _interp("nearest"),
    "pd_op.shape": lambda ins, a: [_P().to_tensor(list(ins[0].shape), dtype="int32")],
}


class PirRunner:
    """Executes block 0 of a PIR program over this framework's ops (inference: no autograd recording)."""

    def __init__(self, program, params):
        self.program = program
        self.params = params  # name -> Tensor
        known = set(_RUN) | {"pd_op.data", "pd_op.feed", "pd_op.fetch", "builtin.parameter", "builtin.combine",
                             "builtin.split", "builtin.shadow_output", "builtin.constant", "pd_op.if",
                             "pd_op.while", "cf.yield"}
        missing = sorted({o[0] for o in program.all_ops()} - known)
        if missing:
            raise NotImplementedError(f"PIR program uses operations without a mapping: {missing}")

    @property
    def feed_names(self):
        return self.program.feed_names

    @property
    def fetch_names(self):
        return self.program.fetch_names

    def run(self, feeds):
        from . import grad_mode
        env = {}
        self._fi = 0
        with grad_mode.no_grad():
            self._block(self.program.ops, env, feeds)
        return [env[v] for _, v in self.program.fetch]

    def _block(self, ops, env, feeds):
        """Runs ``ops`` in ``env``; returns the operands of a terminating cf.yield (sub-blocks)."""
        P = _P()
        for op in ops:
            name, operands, results, attrs, types = op
            ins = [env.get(v) if v != 0 else None for v in operands]
            if name == "cf.yield":
                return ins
            if name == "builtin.parameter":
                env[results[0]] = self.params[attrs["parameter_name"]]
                continue
            if name in ("pd_op.data", "pd_op.feed"):
                key = attrs.get("name")
                v = feeds[key] if isinstance(feeds, dict) else feeds[self._fi]
                self._fi += 1
                env[results[0]] = v if isinstance(v, P.Tensor) else P.to_tensor(np.asarray(v))
                continue
            if name in ("pd_op.fetch", "builtin.shadow_output"):
                continue
            if name == "builtin.combine":
                env[results[0]] = list(ins)
                continue
            if name == "builtin.split":
                for r, v in zip(results, ins[0]):
                    env[r] = v
                continue
            if name == "pd_op.if":  # reference IfOp: true / false block, each ending in cf.yield
                blk = op.regions[0] if bool(_scalar(ins[0])) else op.regions[1]
                outs = self._block(blk.ops, env, feeds) or []
            elif name == "pd_op.while":  # reference WhileOp: operands (cond, vars), body yields (cond, vars)
                body = op.regions[0]
                cond, vals = ins[0], list(ins[1:])
                while bool(_scalar(cond)):
                    for a, v in zip(body.args, vals):
                        env[a] = v
                    y = self._block(body.ops, env, feeds)
                    cond, vals = y[0], list(y[1:])
                outs = vals
            else:
                outs = _RUN[name](ins, attrs)
            for r, v in zip(results, outs):
                env[r] = v
        return None


def load(path_prefix, device=None):
    """``<prefix>.json`` (PIR) + ``<prefix>.pdiparams`` (save_combine, params sorted by name) -> PirRunner."""
    from .combine_io import read_combined
    from .tensor import Tensor
    base = path_prefix[:-len(".json")] if path_prefix.endswith(".json") else path_prefix
    with open(base + ".json") as f:
        prog = PirProgram(json.load(f))
    names = prog.param_names_sorted()
    tensors = read_combined(base + ".pdiparams") if names and os.path.exists(base + ".pdiparams") else []
    if len(tensors) != len(names):
        raise ValueError(f"{base}.pdiparams holds {len(tensors)} tensors, the program lists {len(names)} parameters")
    if device is None:
        from .place import _get_torch_device
        device = _get_torch_device()
    params = {n: Tensor(t.to(device)) for n, t in zip(names, tensors)}
    from ..framework.flags import flag
    if flag("FLAGS_pir_native_interpreter", True):
        from .native_interp import compile_program
        native = compile_program(prog, params, device if isinstance(device, torch.device) else
                                 torch.device(device))
        if native is not None:
            return native
    return PirRunner(prog, params)
