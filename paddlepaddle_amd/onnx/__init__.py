"""paddle.onnx.export (reference: python/paddle/onnx/export.py — a front for paddle2onnx, which converts the
saved static program into an ONNX ModelProto).

Here the Layer is traced into our static Program (jit.trace_program over the InputSpecs: one node per op, the
hand-written HIP ops as whole nodes) and every node is lowered to ONNX operators by the table below; the model is
serialised by onnx/proto.py (protobuf wire format, no onnx package needed). Parameters become initializers
(their names), shapes are static except a leading batch dimension given as None / -1 in the InputSpec, which is
exported symbolically ("N") and kept through Reshape by ONNX's copy-dim 0. Default opset 17 (LayerNormalization).

``onnx/runtime.py`` is a small numpy executor of the emitted operator set; the tests check the exported graph
against eager execution with it (no onnxruntime in this image: parity with a real ONNX runtime is unpinned).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import proto as PB

__all__ = ["export"]

_ONNX_DT = {torch.float32: PB.FLOAT, torch.float16: PB.FLOAT16, torch.bfloat16: PB.BFLOAT16, torch.float64: PB.DOUBLE,
            torch.int64: PB.INT64, torch.int32: PB.INT32, torch.bool: PB.BOOL, torch.uint8: PB.UINT8,
            torch.int8: PB.INT8}


class _Ctx:
    def __init__(self, prog, dyn_batch):
        from ..static import program as P
        self.P = P
        self.prog = prog
        self.nodes, self.inits = [], []
        self.const_names = {}
        self.n_tmp = 0
        self.dyn_batch = dyn_batch

    # ---------------------------------------------------------------- values
    def meta(self, t):
        if isinstance(t, self.P._Ref):
            return self.prog._metas[t.i]
        if isinstance(t, self.P._Const):
            return t.t
        return None

    def shape(self, t):
        return list(self.meta(t).shape)

    def dtype(self, t):
        m = self.meta(t)
        return m.dtype if m is not None else None

    def name(self, t, like=None):
        P = self.P
        if isinstance(t, P._Ref):
            return f"v{t.i}"
        if isinstance(t, P._Const):
            key = ("c", t.idx)
            if key not in self.const_names:
                prm = self.prog._params.get(t.idx)
                nm = getattr(prm, "name", None) or f"const_{t.idx}"
                self.const_names[key] = nm
                self._init(nm, t.t.detach())
            return self.const_names[key]
        if isinstance(t, (bool, int, float)):  # Python scalar operand: typed like the tensor it meets
            dt = self.dtype(like) if like is not None else torch.float32
            if dt is None or (isinstance(t, float) and not dt.is_floating_point):
                dt = torch.float32
            return self.const(torch.tensor(t, dtype=dt))
        raise NotImplementedError(f"ONNX export: operand {t!r}")

    def _init(self, name, tt):
        tt = tt.detach().cpu().contiguous()
        code = _ONNX_DT.get(tt.dtype)
        if code is None:
            raise NotImplementedError(f"ONNX export: initializer dtype {tt.dtype}")
        raw = tt.view(torch.int16).numpy().tobytes() if tt.dtype == torch.bfloat16 else tt.numpy().tobytes()
        b = (PB.f_packed_int(1, tt.shape) if tt.dim() else b"") + PB.f_int(2, code) + PB.f_bytes(8, name) + \
            PB.f_bytes(9, raw)
        self.inits.append(b)

    def const(self, value, name=None):
        t = value if isinstance(value, torch.Tensor) else torch.as_tensor(np.asarray(value))
        nm = name or self.tmp("k")
        self._init(nm, t)
        return nm

    def ints(self, vals):
        return self.const(torch.tensor(list(vals), dtype=torch.int64))

    def tmp(self, p="t"):
        self.n_tmp += 1
        return f"{p}{self.n_tmp}"

    def emit(self, op, ins, outs=None, **attrs):
        outs = outs or [self.tmp()]
        self.nodes.append(PB.node(op, ins, outs, f"{op}_{len(self.nodes)}", **attrs))
        return outs[0] if len(outs) == 1 else outs

    def out(self, node):
        return f"v{node.outs.i}"

    def target_shape(self, node):
        """The output's static shape for Reshape (dim 0 copied from the input when the batch is dynamic)."""
        s = list(self.prog._metas[node.outs.i].shape)
        if self.dyn_batch and s:
            s[0] = 0
        return s


def _arg(a, kw, i, name, default=None):
    if len(a) > i:
        return a[i]
    return kw.get(name, default)


def _act(c, x, act, out, dt=torch.float32):
    if act is None:
        return c.emit("Identity", [x], [out])
    if act == "relu":
        return c.emit("Relu", [x], [out])
    if act in ("gelu", "gelu_tanh", "gelu_approximate"):
        return _gelu(c, x, True, out, dt)
    if act == "gelu_erf":
        return _gelu(c, x, False, out, dt)
    raise NotImplementedError(f"ONNX export: activation {act}")


def _gelu(c, x, approx, out, dt=torch.float32):
    def k(v):
        return c.const(torch.tensor(v, dtype=dt))
    half, one = k(0.5), k(1.0)
    if approx:  # 0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3)))
        inner = c.emit("Mul", [k(0.7978845608028654),
                               c.emit("Add", [x, c.emit("Mul", [k(0.044715), c.emit("Pow", [x, k(3.0)])])])])
        t = c.emit("Tanh", [inner])
    else:  # 0.5 x (1 + erf(x / sqrt 2))
        t = c.emit("Erf", [c.emit("Div", [x, k(1.4142135623730951)])])
    return c.emit("Mul", [c.emit("Mul", [half, x]), c.emit("Add", [one, t])], [out])


def _binary(op, rev=False):
    def h(c, n, a, kw):
        x, y = a[0], a[1]
        alpha = kw.get("alpha", 1)
        xn, yn = c.name(x, like=y if not isinstance(y, (int, float, bool)) else x), \
            c.name(y, like=x if not isinstance(x, (int, float, bool)) else y)
        if alpha != 1:
            yn = c.emit("Mul", [yn, c.name(alpha, like=y)])
        ins = [yn, xn] if rev else [xn, yn]
        return c.emit(op, ins, [c.out(n)])
    return h


def _unary(op):
    def h(c, n, a, kw):
        return c.emit(op, [c.name(a[0])], [c.out(n)])
    return h


def _matmul(c, n, a, kw):
    return c.emit("MatMul", [c.name(a[0]), c.name(a[1])], [c.out(n)])


def _fused_linear(c, n, a, kw):
    x, w = a[0], a[1]
    b = _arg(a, kw, 2, "b")
    act = _arg(a, kw, 3, "act")
    y = c.emit("MatMul", [c.name(x), c.name(w)])
    if b is not None:
        y = c.emit("Add", [y, c.name(b)])
    return _act(c, y, act, c.out(n), c.dtype(x))


def _linear_nt(c, n, a, kw):
    wt = c.emit("Transpose", [c.name(a[1])], perm=[1, 0])
    return c.emit("MatMul", [c.name(a[0]), wt], [c.out(n)])


def _f_linear(c, n, a, kw):
    wt = c.emit("Transpose", [c.name(a[1])], perm=[1, 0])
    y = c.emit("MatMul", [c.name(a[0]), wt])
    b = _arg(a, kw, 2, "bias")
    return c.emit("Add", [y, c.name(b)], [c.out(n)]) if b is not None else c.emit("Identity", [y], [c.out(n)])


def _gelu_h(c, n, a, kw):
    approx = _arg(a, kw, 1, "approximate", False)
    if isinstance(approx, str):
        approx = approx == "tanh"
    return _gelu(c, c.name(a[0]), bool(approx), c.out(n), c.dtype(a[0]))


def _silu(c, n, a, kw):
    x = c.name(a[0])
    return c.emit("Mul", [x, c.emit("Sigmoid", [x])], [c.out(n)])


def _rsqrt(c, n, a, kw):
    return c.emit("Reciprocal", [c.emit("Sqrt", [c.name(a[0])])], [c.out(n)])


def _softmax(op):
    def h(c, n, a, kw):
        ax = _arg(a, kw, 1, "axis", _arg(a, kw, 1, "dim", -1))
        ax = kw.get("dim", ax)
        return c.emit(op, [c.name(a[0])], [c.out(n)], axis=int(ax))
    return h


def _layer_norm_ops(c, n, a, kw):  # ops.norm.layer_norm(x, w, b, eps)
    x, w, b, eps = a[0], a[1], a[2], _arg(a, kw, 3, "eps", 1e-5)
    ins = [c.name(x)]
    C = c.shape(x)[-1]
    ins.append(c.name(w) if w is not None else c.const(torch.ones(C, dtype=c.dtype(x))))
    ins.append(c.name(b) if b is not None else c.const(torch.zeros(C, dtype=c.dtype(x))))
    return c.emit("LayerNormalization", ins, [c.out(n)], axis=-1, epsilon=float(eps))


def _layer_norm_f(c, n, a, kw):  # F.layer_norm(x, shape, weight, bias, eps)
    x, shp = a[0], a[1]
    w, b = _arg(a, kw, 2, "weight"), _arg(a, kw, 3, "bias")
    eps = _arg(a, kw, 4, "eps", 1e-5)
    k = len(shp)
    ins = [c.name(x)]
    ins.append(c.name(w) if w is not None else c.const(torch.ones(list(shp), dtype=c.dtype(x))))
    ins.append(c.name(b) if b is not None else c.const(torch.zeros(list(shp), dtype=c.dtype(x))))
    return c.emit("LayerNormalization", ins, [c.out(n)], axis=-k, epsilon=float(eps))


def _rms_norm(c, n, a, kw):  # ops.norm.rms_norm(x, w, eps)
    x, w, eps = c.name(a[0]), a[1], _arg(a, kw, 2, "eps", 1e-6)
    ms = c.emit("ReduceMean", [c.emit("Mul", [x, x])], axes=[-1], keepdims=1)
    r = c.emit("Reciprocal", [c.emit("Sqrt", [c.emit("Add", [ms, c.name(float(eps), like=a[0])])])])
    y = c.emit("Mul", [x, r])
    return c.emit("Mul", [y, c.name(w)], [c.out(n)]) if w is not None else c.emit("Identity", [y], [c.out(n)])


def _batch_norm(c, n, a, kw):  # F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    x, rm, rv = a[0], a[1], a[2]
    w, b = _arg(a, kw, 3, "weight"), _arg(a, kw, 4, "bias")
    if _arg(a, kw, 5, "training", False):
        raise NotImplementedError("ONNX export: batch_norm in training mode (export an eval() model)")
    eps = _arg(a, kw, 7, "eps", 1e-5)
    C = c.shape(x)[1]
    ins = [c.name(x), c.name(w) if w is not None else c.const(torch.ones(C)),
           c.name(b) if b is not None else c.const(torch.zeros(C)), c.name(rm), c.name(rv)]
    return c.emit("BatchNormalization", ins, [c.out(n)], epsilon=float(eps))


def _pair(v, k=2):
    return list(v) if isinstance(v, (list, tuple)) else [int(v)] * k


def _conv2d(c, n, a, kw):  # torch conv2d(x, w, b, stride, padding, dilation, groups)
    x, w = a[0], a[1]
    b = _arg(a, kw, 2, "bias")
    stride, pad, dil = _pair(_arg(a, kw, 3, "stride", 1)), _arg(a, kw, 4, "padding", 0), \
        _pair(_arg(a, kw, 5, "dilation", 1))
    groups = int(_arg(a, kw, 6, "groups", 1))
    kshape = c.shape(w)[2:]
    if isinstance(pad, str):
        pads = [((k - 1) * d) // 2 for k, d in zip(kshape, dil)] * 2 if pad == "same" else [0, 0, 0, 0]
    else:
        p = _pair(pad)
        pads = p + p
    ins = [c.name(x), c.name(w)] + ([c.name(b)] if b is not None else [])
    return c.emit("Conv", ins, [c.out(n)], strides=stride, pads=pads, dilations=dil, group=groups,
                  kernel_shape=kshape)


def _pool(op):
    def h(c, n, a, kw):
        k = _pair(_arg(a, kw, 1, "kernel_size"))
        s = _arg(a, kw, 2, "stride", None)
        s = k if s is None or s == [] else _pair(s)
        p = _pair(_arg(a, kw, 3, "padding", 0))
        attrs = dict(kernel_shape=k, strides=s, pads=p + p)
        if op == "MaxPool":
            attrs["ceil_mode"] = int(bool(kw.get("ceil_mode", False)))
            if _pair(kw.get("dilation", 1)) != [1, 1]:
                attrs["dilations"] = _pair(kw.get("dilation", 1))
        else:
            attrs["ceil_mode"] = int(bool(_arg(a, kw, 4, "ceil_mode", False)))
            attrs["count_include_pad"] = int(bool(_arg(a, kw, 5, "count_include_pad", True)))
        return c.emit(op, [c.name(a[0])], [c.out(n)], **attrs)
    return h


def _adaptive_avg(c, n, a, kw):
    osz = _pair(a[1])
    if osz != [1, 1]:
        raise NotImplementedError("ONNX export: adaptive_avg_pool2d to a size other than 1")
    return c.emit("GlobalAveragePool", [c.name(a[0])], [c.out(n)])


def _reduce(op):
    def h(c, n, a, kw):
        x = a[0]
        dims = _arg(a, kw, 1, "dim", None)
        keep = int(bool(kw.get("keepdim", _arg(a, kw, 2, "keepdim", False))))
        nd = len(c.shape(x))
        if dims is None:
            dims = list(range(nd))
        dims = [int(d) for d in (dims if isinstance(dims, (list, tuple)) else [dims])]
        if op == "ReduceSum":  # axes are an input from opset 13
            return c.emit(op, [c.name(x), c.ints(dims)], [c.out(n)], keepdims=keep)
        return c.emit(op, [c.name(x)], [c.out(n)], axes=dims, keepdims=keep)
    return h


def _reshape(c, n, a, kw):
    return c.emit("Reshape", [c.name(a[0]), c.ints(c.target_shape(n))], [c.out(n)])


def _permute(c, n, a, kw):
    dims = a[1:] if len(a) > 2 else a[1]
    dims = list(dims) if isinstance(dims, (list, tuple)) else [dims]
    nd = len(c.shape(a[0]))
    return c.emit("Transpose", [c.name(a[0])], [c.out(n)], perm=[int(d) % nd for d in dims])


def _transpose(c, n, a, kw):
    nd = len(c.shape(a[0]))
    d0, d1 = int(a[1]) % nd, int(a[2]) % nd
    perm = list(range(nd))
    perm[d0], perm[d1] = perm[d1], perm[d0]
    return c.emit("Transpose", [c.name(a[0])], [c.out(n)], perm=perm)


def _t(c, n, a, kw):
    return c.emit("Transpose", [c.name(a[0])], [c.out(n)], perm=[1, 0])


def _cat(c, n, a, kw):
    ts = a[0]
    ax = _arg(a, kw, 1, "dim", 0)
    return c.emit("Concat", [c.name(t) for t in ts], [c.out(n)], axis=int(ax))


def _identity(c, n, a, kw):
    return c.emit("Identity", [c.name(a[0])], [c.out(n)])


def _dropout(c, n, a, kw):
    if _arg(a, kw, 2, "training", False):
        raise NotImplementedError("ONNX export: dropout in training mode (export an eval() model)")
    return _identity(c, n, a, kw)


_CAST = {torch.float32: PB.FLOAT, torch.float16: PB.FLOAT16, torch.bfloat16: PB.BFLOAT16, torch.int64: PB.INT64,
         torch.int32: PB.INT32, torch.bool: PB.BOOL, torch.float64: PB.DOUBLE}


def _to(c, n, a, kw):
    dt = c.prog._metas[n.outs.i].dtype
    return c.emit("Cast", [c.name(a[0])], [c.out(n)], to=_CAST[dt])


def _embedding(c, n, a, kw):  # F.embedding(ids, weight, ...)
    return c.emit("Gather", [c.name(a[1]), c.name(a[0])], [c.out(n)], axis=0)


def _pow(c, n, a, kw):
    return c.emit("Pow", [c.name(a[0]), c.name(a[1], like=a[0])], [c.out(n)])


def _clamp(c, n, a, kw):
    lo, hi = _arg(a, kw, 1, "min"), _arg(a, kw, 2, "max")
    ins = [c.name(a[0]), c.name(lo, like=a[0]) if lo is not None else "",
           c.name(hi, like=a[0]) if hi is not None else ""]
    return c.emit("Clip", ins, [c.out(n)])


def _getitem(c, n, a, kw):
    x, idx = a[0], a[1]
    idx = idx if isinstance(idx, tuple) else (idx,)
    shape = c.shape(x)
    starts, ends, axes, steps, squeeze = [], [], [], [], []
    ax = 0
    for it in idx:
        if it is Ellipsis:
            ax = len(shape) - (len(idx) - 1 - idx.index(Ellipsis))  # the items after it index the last dims
            continue
        if isinstance(it, slice):
            if it != slice(None):
                st, en, sp = it.indices(shape[ax])
                starts.append(st), ends.append(en), axes.append(ax), steps.append(sp)
        elif isinstance(it, int):
            i = it % shape[ax]
            starts.append(i), ends.append(i + 1), axes.append(ax), steps.append(1)
            squeeze.append(ax)
        else:
            raise NotImplementedError(f"ONNX export: index {it!r}")
        ax += 1
    y = c.name(x)
    if axes:
        y = c.emit("Slice", [y, c.ints(starts), c.ints(ends), c.ints(axes), c.ints(steps)])
    if squeeze:
        y = c.emit("Squeeze", [y, c.ints(squeeze)])
    return c.emit("Identity", [y], [c.out(n)])


def _split(c, n, a, kw):  # torch.split(x, size_or_sections, dim) -> several outputs
    x = a[0]
    sz = _arg(a, kw, 1, "split_size_or_sections")
    dim = int(_arg(a, kw, 2, "dim", 0))
    L = c.shape(x)[dim]
    sizes = list(sz) if isinstance(sz, (list, tuple)) else [min(sz, L - i) for i in range(0, L, sz)]
    outs = [f"v{r.i}" for r in n.outs]
    return c.emit("Split", [c.name(x), c.ints(sizes)], outs, axis=dim)


def _chunk(c, n, a, kw):  # Tensor.chunk(k, dim)
    x = a[0]
    k = int(_arg(a, kw, 1, "chunks"))
    dim = int(_arg(a, kw, 2, "dim", 0))
    L = c.shape(x)[dim]
    step = -(-L // k)
    sizes = [min(step, L - i) for i in range(0, L, step)]
    outs = [f"v{r.i}" for r in n.outs]
    return c.emit("Split", [c.name(x), c.ints(sizes)], outs, axis=dim)


def _where(c, n, a, kw):
    return c.emit("Where", [c.name(a[0]), c.name(a[1], like=a[2]), c.name(a[2], like=a[1])], [c.out(n)])


def _maxmin(op):
    def h(c, n, a, kw):
        return c.emit(op, [c.name(a[0], like=a[1]), c.name(a[1], like=a[0])], [c.out(n)])
    return h


_T = {}
for k in ("f:torch:matmul", "m:matmul", "m:__matmul__", "f:torch:mm", "m:mm", "f:torch:bmm", "m:bmm"):
    _T[k] = _matmul
for nm, op in (("add", "Add"), ("sub", "Sub"), ("mul", "Mul"), ("div", "Div"), ("true_divide", "Div")):
    _T[f"m:{nm}"] = _T[f"f:torch:{nm}"] = _T[f"m:__{nm}__"] = _binary(op)
_T["m:__truediv__"] = _binary("Div")
_T["m:__radd__"], _T["m:__rmul__"] = _binary("Add", True), _binary("Mul", True)
_T["m:__rsub__"], _T["m:__rtruediv__"] = _binary("Sub", True), _binary("Div", True)
for nm, op in (("relu", "Relu"), ("sigmoid", "Sigmoid"), ("tanh", "Tanh"), ("exp", "Exp"), ("log", "Log"),
               ("sqrt", "Sqrt"), ("abs", "Abs"), ("neg", "Neg"), ("erf", "Erf"), ("floor", "Floor"),
               ("ceil", "Ceil"), ("reciprocal", "Reciprocal"), ("sin", "Sin"), ("cos", "Cos")):
    _T[f"m:{nm}"] = _T[f"f:torch:{nm}"] = _T[f"f:torch.nn.functional:{nm}"] = _unary(op)
_T["m:__neg__"] = _unary("Neg")
_T.update({
    "o:paddlepaddle_amd.ops.linear:fused_linear": _fused_linear, "o:paddlepaddle_amd.ops.linear:linear_nt": _linear_nt,
    "f:torch.nn.functional:linear": _f_linear,
    "o:paddlepaddle_amd.ops.activation:gelu": _gelu_h, "f:torch.nn.functional:gelu": _gelu_h,
    "o:paddlepaddle_amd.ops.activation:silu": _silu, "f:torch.nn.functional:silu": _silu,
    "m:rsqrt": _rsqrt, "f:torch:rsqrt": _rsqrt,
    "o:paddlepaddle_amd.ops.activation:softmax": _softmax("Softmax"), "f:torch:softmax": _softmax("Softmax"),
    "m:softmax": _softmax("Softmax"), "f:torch.nn.functional:softmax": _softmax("Softmax"),
    "f:torch.nn.functional:log_softmax": _softmax("LogSoftmax"), "m:log_softmax": _softmax("LogSoftmax"),
    "o:paddlepaddle_amd.ops.norm:layer_norm": _layer_norm_ops, "f:torch.nn.functional:layer_norm": _layer_norm_f,
    "o:paddlepaddle_amd.ops.norm:rms_norm": _rms_norm,
    "f:torch.nn.functional:batch_norm": _batch_norm,
    "f:torch:conv2d": _conv2d, "f:torch.nn.functional:conv2d": _conv2d,
    "f:torch.nn.functional:max_pool2d": _pool("MaxPool"), "f:torch.nn.functional:avg_pool2d": _pool("AveragePool"),
    "f:torch.nn.functional:adaptive_avg_pool2d": _adaptive_avg,
    "m:mean": _reduce("ReduceMean"), "f:torch:mean": _reduce("ReduceMean"),
    "m:sum": _reduce("ReduceSum"), "f:torch:sum": _reduce("ReduceSum"),
    "m:amax": _reduce("ReduceMax"), "f:torch:amax": _reduce("ReduceMax"),
    "m:reshape": _reshape, "f:torch:reshape": _reshape, "m:view": _reshape, "f:torch:flatten": _reshape,
    "m:flatten": _reshape, "m:squeeze": _reshape, "f:torch:squeeze": _reshape, "m:unsqueeze": _reshape,
    "f:torch:unsqueeze": _reshape, "m:expand_as": None,
    "m:permute": _permute, "f:torch:permute": _permute, "m:transpose": _transpose, "f:torch:transpose": _transpose,
    "m:t": _t, "f:torch:cat": _cat, "f:torch:concat": _cat,
    "m:contiguous": _identity, "m:clone": _identity, "m:detach": _identity, "f:torch:clone": _identity,
    "f:torch.nn.functional:dropout": _dropout,
    "m:to": _to, "m:float": _to, "m:half": _to, "m:bfloat16": _to, "m:type": _to,
    "f:torch.nn.functional:embedding": _embedding,
    "m:pow": _pow, "f:torch:pow": _pow, "m:__pow__": _pow,
    "m:clamp": _clamp, "f:torch:clamp": _clamp, "m:clip": _clamp,
    "m:__getitem__": _getitem, "f:torch:where": _where,
    "f:torch.functional:split": _split, "f:torch:split": _split, "m:split": _split,
    "m:chunk": _chunk, "f:torch:chunk": _chunk,
    "f:torch:maximum": _maxmin("Max"), "f:torch:minimum": _maxmin("Min"),
})
_T = {k: v for k, v in _T.items() if v is not None}


def export_program(prog, feed_slots, fetch_slots, input_names, dyn_batch=False, opset=17, name="paddle_model"):
    """Lower a traced Program to ONNX bytes."""
    c = _Ctx(prog, dyn_batch)
    for nd in prog.nodes:
        if nd.kind == "guard":
            raise NotImplementedError("ONNX export: the program has data-dependent guards")
        nm = nd.name.replace("f:torch._C._nn:", "f:torch.nn.functional:")
        h = _T.get(nm)
        if h is None:
            raise NotImplementedError(f"ONNX export: no ONNX lowering for op '{nd.name}'")
        multi = h in (_split, _chunk)
        if nd.outs is None or (not isinstance(nd.outs, c.P._Ref) and not multi):
            raise NotImplementedError(f"ONNX export: op '{nd.name}' with multiple / no outputs")
        h(c, nd, list(nd.args), dict(nd.kwargs))
    ins, outs = [], []
    for s, nm in zip(feed_slots, input_names):
        m = prog._metas[s]
        shape = list(m.shape)
        if dyn_batch and shape:
            shape[0] = "N"
        c.nodes.insert(0, PB.node("Identity", [nm], [f"v{s}"], f"input_{nm}"))
        ins.append(PB.value_info(nm, _ONNX_DT[m.dtype], shape))
    for i, s in enumerate(fetch_slots):
        m = prog._metas[s]
        shape = list(m.shape)
        if dyn_batch and shape:
            shape[0] = "N"
        nm = f"output_{i}"
        c.nodes.append(PB.node("Identity", [f"v{s}"], [nm], f"output_{i}"))
        outs.append(PB.value_info(nm, _ONNX_DT[m.dtype], shape))
    return PB.model(c.nodes, name, c.inits, ins, outs, opset=opset)


def export(layer, path, input_spec=None, opset_version=17, **configs):
    """Export ``layer`` (eval mode) to ``path + '.onnx'`` (reference: paddle.onnx.export). ``input_spec``: list of
    InputSpec / example Tensors; a None / -1 leading dim is exported as a symbolic batch dimension."""
    from ..jit import trace_program
    from ..static.executor import InputSpec
    from ..framework.tensor import Tensor
    if input_spec is None:
        raise ValueError("paddle.onnx.export needs input_spec")
    specs, dyn = [], False
    for s in input_spec:
        if isinstance(s, Tensor):
            s = InputSpec(list(s.shape), str(s.dtype).replace("paddle.", ""), None)
        shape = list(s.shape)
        if shape and (shape[0] is None or shape[0] < 0):
            dyn = True
            shape[0] = 2  # traced at a concrete batch; exported with a symbolic one
        if any(d is None or d < 0 for d in shape[1:]):
            raise NotImplementedError("ONNX export: only the leading dimension may be dynamic")
        specs.append(InputSpec(shape, s.dtype, s.name))
    was_training = getattr(layer, "training", False)
    if hasattr(layer, "eval"):
        layer.eval()
    try:
        prog, feeds, tmpl, fetch = trace_program(layer, tuple(specs), {})
    finally:
        if was_training and hasattr(layer, "train"):
            layer.train()
    names = [s.name or f"x{i}" for i, s in enumerate(specs)]
    data = export_program(prog, feeds, fetch, names, dyn, int(opset_version), type(layer).__name__)
    out = path if path.endswith(".onnx") else path + ".onnx"
    d = os.path.dirname(out)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(out, "wb") as f:
        f.write(data)
    return out
