"""paddle.summary and paddle.flops. Reference: python/paddle/hapi/model_summary.py (summary),
hapi/dynamic_flops.py (flops: per-layer multiply-accumulate counting via forward hooks)."""
from __future__ import annotations

import numpy as np
import torch

from ..framework.tensor import Tensor, _wrap
from ..framework import dtype as _dt


def _make_inputs(input_size, dtypes, input):
    if input is not None:
        return input if isinstance(input, (list, tuple)) else [input]
    sizes = input_size if isinstance(input_size, list) and input_size and isinstance(input_size[0], (list, tuple)) \
        else [input_size]
    dts = dtypes if isinstance(dtypes, (list, tuple)) else [dtypes] * len(sizes)
    from ..tensor.creation import zeros
    out = []
    for s, d in zip(sizes, dts):
        shape = [1 if (v is None or v < 0) else int(v) for v in s]
        out.append(zeros(shape, d or _dt.get_default_dtype()))
    return out


def _is_leaf(layer):
    return len(list(layer.children())) == 0


def _shape_of(o):
    if isinstance(o, Tensor):
        return list(o.shape)
    if isinstance(o, (list, tuple)):
        return [_shape_of(v) for v in o]
    return []


def summary(net, input_size=None, dtypes=None, input=None):
    rows = []
    hooks = []

    def make_hook(name, layer):
        def hook(l, inp, out):
            n_params = sum(int(np.prod(p.shape)) for p in l.parameters(include_sublayers=False))
            trainable = sum(int(np.prod(p.shape)) for p in l.parameters(include_sublayers=False)
                            if not p.stop_gradient)
            rows.append((f"{type(l).__name__}-{len(rows) + 1}", _shape_of(inp[0]) if inp else [], _shape_of(out),
                         n_params, trainable))
        return hook

    for name, layer in net.named_sublayers():
        if _is_leaf(layer):
            hooks.append(layer.register_forward_post_hook(make_hook(name, layer)))
    was_training = net.training
    net.eval()
    from ..framework.grad_mode import no_grad
    try:
        with no_grad():
            net(*_make_inputs(input_size, dtypes, input))
    finally:
        for h in hooks:
            h.remove()
        if was_training:
            net.train()
    total = sum(int(np.prod(p.shape)) for p in net.parameters())
    trainable = sum(int(np.prod(p.shape)) for p in net.parameters() if not p.stop_gradient)
    w = 100
    lines = ["-" * w, f"{'Layer (type)':<28}{'Input Shape':<26}{'Output Shape':<26}{'Param #':>14}", "=" * w]
    for name, i, o, n, _ in rows:
        lines.append(f"{name:<28}{str(i):<26}{str(o):<26}{n:>14,}")
    lines += ["=" * w, f"Total params: {total:,}", f"Trainable params: {trainable:,}",
              f"Non-trainable params: {total - trainable:,}", "-" * w]
    print("\n".join(lines))
    return {"total_params": total, "trainable_params": trainable}


def _numel(x):
    return int(np.prod(x.shape)) if isinstance(x, Tensor) else 0


def _count(layer, inp, out):
    from .. import nn
    x = inp[0] if inp else None
    o = out[0] if isinstance(out, (list, tuple)) else out
    n_out = _numel(o)
    if isinstance(layer, (nn.Conv1D, nn.Conv2D, nn.Conv3D, nn.Conv1DTranspose, nn.Conv2DTranspose,
                          nn.Conv3DTranspose)):
        w = layer.weight
        k = int(np.prod(w.shape[2:])) if not getattr(layer, "_channels_last_weight", False) \
            else int(np.prod(w.shape[1:-1]))
        cin_per_group = (w.shape[1] if not getattr(layer, "_channels_last_weight", False) else w.shape[-1])
        ops = k * cin_per_group + (1 if getattr(layer, "bias", None) is not None else 0)
        return ops * n_out
    if isinstance(layer, nn.Linear):
        return int(layer.weight.shape[0]) * n_out
    if isinstance(layer, (nn.BatchNorm, nn.BatchNorm1D, nn.BatchNorm2D, nn.BatchNorm3D, nn.LayerNorm,
                          nn.GroupNorm, nn.InstanceNorm2D, nn.SyncBatchNorm)):
        return 2 * _numel(x)
    if isinstance(layer, (nn.ReLU, nn.ReLU6, nn.LeakyReLU, nn.Sigmoid, nn.GELU, nn.Tanh, nn.Hardswish, nn.Silu)):
        return _numel(x)
    if isinstance(layer, (nn.AvgPool1D, nn.AvgPool2D, nn.AvgPool3D, nn.MaxPool1D, nn.MaxPool2D, nn.MaxPool3D)):
        ks = layer.ksize if hasattr(layer, "ksize") else getattr(layer, "kernel_size", 1)
        k = int(np.prod(ks)) if isinstance(ks, (list, tuple)) else int(ks) ** (x.ndim - 2 if x is not None else 2)
        return k * n_out
    if isinstance(layer, (nn.AdaptiveAvgPool1D, nn.AdaptiveAvgPool2D, nn.AdaptiveAvgPool3D)):
        return _numel(x)
    if isinstance(layer, nn.Upsample):
        return n_out
    return 0


def flops(net, input_size, custom_ops=None, print_detail=False):
    custom_ops = custom_ops or {}
    total = [0]
    detail = []
    hooks = []

    def make_hook(layer):
        def hook(l, inp, out):
            fn = custom_ops.get(type(l))
            if fn is not None:
                c = fn(l, inp, out)
            else:
                c = _count(l, inp, out)
            total[0] += int(c)
            detail.append((type(l).__name__, int(c)))
        return hook

    for _, layer in net.named_sublayers(include_self=True):
        if _is_leaf(layer):
            hooks.append(layer.register_forward_post_hook(make_hook(layer)))
    was_training = net.training
    net.eval()
    from ..framework.grad_mode import no_grad
    try:
        with no_grad():
            net(*_make_inputs(list(input_size), None, None))
    finally:
        for h in hooks:
            h.remove()
        if was_training:
            net.train()
    if print_detail:
        for n, c in detail:
            print(f"{n:<24}{c:>16,}")
    print(f"Total Flops: {total[0]}     Total Params: {sum(int(np.prod(p.shape)) for p in net.parameters())}")
    return total[0]
