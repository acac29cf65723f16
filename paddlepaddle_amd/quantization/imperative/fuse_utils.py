"""Conv / Linear + BatchNorm folding before quantization. Reference: python/paddle/quantization/imperative/
fuse_utils.py (fuse_conv_bn, fuse_layers): the BN's inference transform is folded into the preceding layer's
weight and bias and the BN becomes an identity."""
from __future__ import annotations

import torch

from ... import nn


class Identity(nn.Layer):
    def __init__(self, *args, **kwargs):
        super().__init__()

    def forward(self, x):
        return x


def _fold(layer, bn, channel_axis):
    rm, rv = bn._mean._t.detach().float(), bn._variance._t.detach().float()
    g = bn.weight._t.detach().float() if bn.weight is not None else torch.ones_like(rm)
    b = bn.bias._t.detach().float() if bn.bias is not None else torch.zeros_like(rm)
    scale = g / torch.sqrt(rv + bn._epsilon)
    w = layer.weight._t
    shape = [1] * w.dim()
    shape[channel_axis] = -1
    with torch.no_grad():
        w.copy_((w.float() * scale.reshape(shape)).to(w.dtype))
        old_b = layer.bias._t.detach().float() if layer.bias is not None else torch.zeros_like(rm)
        new_b = (old_b - rm) * scale + b
        if layer.bias is None:
            from ...nn.layer.layers import create_parameter_tensor
            layer.bias = create_parameter_tensor([new_b.numel()], "float32", None, is_bias=True, device=w.device)
        layer.bias._t.copy_(new_b.to(layer.bias._t.dtype))
    return layer


def _fuse_pair(a, b):
    if isinstance(a, nn.Conv2D) and isinstance(b, (nn.BatchNorm2D, nn.BatchNorm)):
        return _fold(a, b, 0), Identity()
    if isinstance(a, nn.Linear) and isinstance(b, (nn.BatchNorm1D, nn.BatchNorm)):
        return _fold(a, b, 1), Identity()
    return None


def fuse_conv_bn(model):
    """Folds every BN that directly follows a Conv2D (or Linear) among a layer's children, in eval semantics."""
    kids = list(model.named_children())
    for (n1, a), (n2, b) in zip(kids, kids[1:]):
        r = _fuse_pair(a, b)
        if r is not None:
            model._sub_layers[n1], model._sub_layers[n2] = r
    for _, sub in model.named_children():
        fuse_conv_bn(sub)
    return model


def _get(model, dotted):
    obj = model
    for p in dotted.split("."):
        obj = obj._sub_layers[p]
    return obj


def _set(model, dotted, value):
    parts = dotted.split(".")
    obj = model
    for p in parts[:-1]:
        obj = obj._sub_layers[p]
    obj._sub_layers[parts[-1]] = value


def fuse_layers(model, layers_to_fuse, inplace=False):
    """layers_to_fuse: lists of two dotted sublayer names ([conv, bn] or [linear, bn])."""
    import copy
    m = model if inplace else copy.deepcopy(model)
    for names in layers_to_fuse:
        if len(names) != 2:
            raise ValueError("fuse_layers: each entry names a (conv|linear, bn) pair")
        r = _fuse_pair(_get(m, names[0]), _get(m, names[1]))
        if r is None:
            raise ValueError(f"fuse_layers: {names} is not a (Conv2D|Linear, BatchNorm) pair")
        _set(m, names[0], r[0])
        _set(m, names[1], r[1])
    return m
