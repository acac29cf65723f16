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


def _layer_key(layer, n_rows):
    """`<Class>-<k>`: k is the per-class instance counter of the layer's full name plus one, so the
    n-th Conv2D built in the process is Conv2D-n (reference model_summary.py numbering)."""
    try:
        idx = int(layer.full_name().split("_")[-1])
    except ValueError:
        idx = n_rows
    return f"{type(layer).__name__}-{idx + 1}"


def _input_mb(sizes):
    if isinstance(sizes, (list, tuple)) and all(isinstance(v, (int, np.integer)) for v in sizes):
        return abs(float(np.prod(sizes)) * 4.0 / 1024 ** 2)
    return sum(_input_mb(v) for v in sizes)


def _summary_table(rows, input_sizes):
    """The reference's text table: centred columns at least 15/20/20/15 wide (grown to fit), a rule
    at least 75 wide, then parameter totals and a float32 memory estimate."""
    w = {"layer": 15, "in": 20, "out": 20, "params": 15}
    for key, r in rows.items():
        w["layer"] = max(w["layer"], len(key))
        w["in"] = max(w["in"], len(str(r["input_shape"])))
        w["out"] = max(w["out"], len(str(r["output_shape"])))
        w["params"] = max(w["params"], len(str(r["nb_params"])))
    width = max(75, sum(w.values()) + 5)

    def line(a, b, c, d):
        return f"{a:^{w['layer']}} {b:^{w['in']}} {c:^{w['out']}} {d:^{w['params']}}"

    out = ["-" * width, line("Layer (type)", "Input Shape", "Output Shape", "Param #"), "=" * width]
    total = trainable = 0
    n_out = 0.0
    for key, r in rows.items():
        out.append(line(key, str(r["input_shape"]), str(r["output_shape"]), f"{r['nb_params']:,}"))
        total += r["nb_params"]
        trainable += r["trainable_params"]
        shp = r["output_shape"]
        if shp and isinstance(shp[0], list):
            n_out += sum(float(np.prod(o)) for o in shp if o and not isinstance(o[0], list))
        elif shp:
            n_out += float(np.prod(shp))
    in_mb = _input_mb(input_sizes)
    act_mb = abs(2.0 * n_out * 4.0 / 1024 ** 2)  # x2: activations and their gradients
    par_mb = abs(total * 4.0 / 1024 ** 2)
    out += ["=" * width, f"Total params: {total:,}", f"Trainable params: {trainable:,}",
            f"Non-trainable params: {total - trainable:,}", "-" * width,
            f"Input size (MB): {in_mb:0.2f}", f"Forward/backward pass size (MB): {act_mb:0.2f}",
            f"Params size (MB): {par_mb:0.2f}", f"Estimated Total Size (MB): {par_mb + act_mb + in_mb:0.2f}",
            "-" * width]
    return "\n".join(out) + "\n", total, trainable


def summary(net, input_size=None, dtypes=None, input=None):
    """Per-layer input/output shapes and parameter counts from one forward pass (reference
    hapi/model_summary.py:summary). Every sublayer except Sequential / LayerList containers is
    hooked; each row counts the layer's own parameters."""
    from .. import nn
    if input_size is None and input is None:
        raise ValueError("summary needs input_size or input")
    rows = {}
    hooks = []

    def hook(l, inp, out):
        own = [p for p in l._parameters.values() if p is not None]
        rows[_layer_key(l, len(rows))] = {
            "input_shape": _shape_of(list(inp)),
            "output_shape": _shape_of(out),
            "nb_params": sum(int(np.prod(p.shape)) for p in own),
            "trainable_params": sum(int(np.prod(p.shape)) for p in own
                                    if not p.stop_gradient and getattr(p, "trainable", True)),
        }

    subs = net.sublayers()
    for layer in net.sublayers(include_self=True):
        if isinstance(layer, (nn.Sequential, nn.LayerList)) or (layer is net and subs):
            continue
        hooks.append(layer.register_forward_post_hook(hook))
    if isinstance(input_size, tuple):
        input_size = [input_size]
    if input is not None:
        flat = list(input.values()) if isinstance(input, dict) else \
            (list(input) if isinstance(input, (list, tuple)) else [input])
        sizes = [list(t.shape) for t in flat if isinstance(t, Tensor)]
    else:
        inputs, sizes = _make_inputs(input_size, dtypes, None), input_size
    was_training = net.training
    net.eval()
    from ..framework.grad_mode import no_grad
    try:
        with no_grad():
            if input is not None:
                net(input)  # passed through as the single forward argument, as the reference does
            else:
                net(*inputs)
    finally:
        for h in hooks:
            h.remove()
        if was_training:
            net.train()
    text, total, trainable = _summary_table(rows, sizes)
    print(text)
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
