"""A small numpy executor for the ONNX operator subset the exporter emits (reads the ModelProto with onnx/proto.py).
Used by the tests to check exported graphs against eager execution; semantics follow the ONNX operator spec."""
from __future__ import annotations

import math

import numpy as np

from . import proto as PB


def _conv(x, w, b, strides, pads, dil, group):
    N, C, H, W = x.shape
    O, Cg, KH, KW = w.shape
    xp = np.pad(x, ((0, 0), (0, 0), (pads[0], pads[2]), (pads[1], pads[3])))
    Ho = (xp.shape[2] - dil[0] * (KH - 1) - 1) // strides[0] + 1
    Wo = (xp.shape[3] - dil[1] * (KW - 1) - 1) // strides[1] + 1
    out = np.zeros((N, O, Ho, Wo), dtype=np.float64)
    og = O // group
    for g in range(group):
        xs = xp[:, g * Cg:(g + 1) * Cg]
        for kh in range(KH):
            for kw in range(KW):
                patch = xs[:, :, kh * dil[0]:kh * dil[0] + strides[0] * Ho:strides[0],
                           kw * dil[1]:kw * dil[1] + strides[1] * Wo:strides[1]]
                out[:, g * og:(g + 1) * og] += np.einsum("nchw,oc->nohw", patch, w[g * og:(g + 1) * og, :, kh, kw])
    if b is not None:
        out += b.reshape(1, -1, 1, 1)
    return out.astype(x.dtype)


def _pool(x, k, s, pads, mode, count_include_pad=1):
    fill = -np.inf if mode == "max" else 0.0
    xp = np.pad(x, ((0, 0), (0, 0), (pads[0], pads[2]), (pads[1], pads[3])), constant_values=fill)
    ones = np.pad(np.ones_like(x), ((0, 0), (0, 0), (pads[0], pads[2]), (pads[1], pads[3])))
    Ho = (xp.shape[2] - k[0]) // s[0] + 1
    Wo = (xp.shape[3] - k[1]) // s[1] + 1
    acc = np.full(x.shape[:2] + (Ho, Wo), fill, dtype=np.float64)
    cnt = np.zeros_like(acc)
    for i in range(k[0]):
        for j in range(k[1]):
            v = xp[:, :, i:i + s[0] * Ho:s[0], j:j + s[1] * Wo:s[1]]
            if mode == "max":
                acc = np.maximum(acc, v)
            else:
                acc = acc + v
                cnt = cnt + ones[:, :, i:i + s[0] * Ho:s[0], j:j + s[1] * Wo:s[1]]
    if mode == "avg":
        acc = acc / (k[0] * k[1] if count_include_pad else cnt)
    return acc.astype(x.dtype)


def _ln(x, w, b, axis, eps):
    axes = tuple(range(axis % x.ndim, x.ndim))
    m = x.mean(axes, keepdims=True)
    v = ((x - m) ** 2).mean(axes, keepdims=True)
    return ((x - m) / np.sqrt(v + eps) * w + b).astype(x.dtype)


def _softmax(x, axis):
    e = np.exp(x - x.max(axis, keepdims=True))
    return e / e.sum(axis, keepdims=True)


_ERF = np.vectorize(math.erf)


def run(model_bytes, feeds):
    m = PB.read_model(model_bytes)
    env = dict(m["initializers"])
    env.update({k: np.asarray(v) for k, v in feeds.items()})
    for op, ins, outs, at in m["nodes"]:
        a = [env[i] if i else None for i in ins]
        if op == "Identity":
            r = a[0]
        elif op in ("Add", "Sub", "Mul", "Div", "Pow", "Max", "Min"):
            f = {"Add": np.add, "Sub": np.subtract, "Mul": np.multiply, "Div": np.divide, "Pow": np.power,
                 "Max": np.maximum, "Min": np.minimum}[op]
            r = f(a[0], a[1]).astype(np.result_type(a[0], a[1]))
        elif op == "MatMul":
            r = np.matmul(a[0], a[1])
        elif op in ("Relu", "Sigmoid", "Tanh", "Exp", "Log", "Sqrt", "Abs", "Neg", "Erf", "Floor", "Ceil",
                    "Reciprocal", "Sin", "Cos"):
            x = a[0]
            r = {"Relu": lambda: np.maximum(x, 0), "Sigmoid": lambda: 1 / (1 + np.exp(-x)), "Tanh": lambda: np.tanh(x),
                 "Exp": lambda: np.exp(x), "Log": lambda: np.log(x), "Sqrt": lambda: np.sqrt(x),
                 "Abs": lambda: np.abs(x), "Neg": lambda: -x, "Erf": lambda: _ERF(x),
                 "Floor": lambda: np.floor(x), "Ceil": lambda: np.ceil(x), "Reciprocal": lambda: 1 / x,
                 "Sin": lambda: np.sin(x), "Cos": lambda: np.cos(x)}[op]().astype(x.dtype)
        elif op == "Softmax":
            r = _softmax(a[0], at.get("axis", -1)).astype(a[0].dtype)
        elif op == "LogSoftmax":
            r = np.log(_softmax(a[0], at.get("axis", -1))).astype(a[0].dtype)
        elif op == "LayerNormalization":
            r = _ln(a[0], a[1], a[2], at.get("axis", -1), at.get("epsilon", 1e-5))
        elif op == "BatchNormalization":
            x, w, b, mu, var = a
            sh = (1, -1) + (1,) * (x.ndim - 2)
            r = ((x - mu.reshape(sh)) / np.sqrt(var.reshape(sh) + at.get("epsilon", 1e-5)) * w.reshape(sh)
                 + b.reshape(sh)).astype(x.dtype)
        elif op == "Conv":
            r = _conv(a[0], a[1], a[2] if len(a) > 2 else None, at.get("strides", [1, 1]), at.get("pads", [0] * 4),
                      at.get("dilations", [1, 1]), at.get("group", 1))
        elif op in ("MaxPool", "AveragePool"):
            r = _pool(a[0], at["kernel_shape"], at.get("strides", at["kernel_shape"]), at.get("pads", [0] * 4),
                      "max" if op == "MaxPool" else "avg", at.get("count_include_pad", 0))
        elif op == "GlobalAveragePool":
            r = a[0].mean((2, 3), keepdims=True)
        elif op in ("ReduceMean", "ReduceMax"):
            f = np.mean if op == "ReduceMean" else np.max
            r = f(a[0], axis=tuple(at["axes"]), keepdims=bool(at.get("keepdims", 1))).astype(a[0].dtype)
        elif op == "ReduceSum":
            r = a[0].sum(axis=tuple(a[1].tolist()), keepdims=bool(at.get("keepdims", 1))).astype(a[0].dtype)
        elif op == "Reshape":
            shp = [a[0].shape[i] if d == 0 else d for i, d in enumerate(a[1].tolist())]
            r = a[0].reshape(shp)
        elif op == "Transpose":
            r = np.transpose(a[0], at.get("perm"))
        elif op == "Concat":
            r = np.concatenate(a, axis=at["axis"])
        elif op == "Cast":
            r = a[0].astype(PB.ONNX2NP[at["to"]])
        elif op == "Gather":
            r = np.take(a[0], a[1].astype(np.int64), axis=at.get("axis", 0))
        elif op == "Clip":
            lo = a[1] if len(a) > 1 and a[1] is not None else -np.inf
            hi = a[2] if len(a) > 2 and a[2] is not None else np.inf
            r = np.clip(a[0], lo, hi).astype(a[0].dtype)
        elif op == "Slice":
            x, st, en, ax, sp = a
            sl = [slice(None)] * x.ndim
            for s0, e0, a0, p0 in zip(st.tolist(), en.tolist(), ax.tolist(), sp.tolist()):
                sl[a0] = slice(s0, e0, p0)
            r = x[tuple(sl)]
        elif op == "Squeeze":
            r = np.squeeze(a[0], axis=tuple(a[1].tolist()))
        elif op == "Where":
            r = np.where(a[0], a[1], a[2])
        elif op == "Split":
            idx = np.cumsum(a[1].tolist())[:-1]
            for o, part in zip(outs, np.split(a[0], idx, axis=at.get("axis", 0))):
                env[o] = part
            continue
        else:
            raise NotImplementedError(f"onnx runtime: {op}")
        env[outs[0]] = r
    return [env[o] for o in m["outputs"]]
