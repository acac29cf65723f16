"""Automatic SParsity (n:m structured pruning, 2:4 by default).
Reference: python/paddle/incubate/asp/ (asp.py: decorate, prune_model, set_excluded_layers,
reset_excluded_layers; utils.py: calculate_density, check_mask_1d/2d, create_mask).
Masks are computed on the device per group of m consecutive input weights; decorate() makes the
optimizer re-apply them after every step so pruned weights stay zero."""
from __future__ import annotations

import torch

from ..framework.grad_mode import no_grad
from ..framework.tensor import Tensor

_excluded = set()
_masks = {}
# layer-type name -> pruning function (weight ndarray, m, n, mask_algo, param_name) -> (pruned, mask);
# None = the default n:m mask of create_mask (reference supported_layer_list.py)
_supported = {"linear": None, "conv2d": None}


def _snake(name):
    import re
    return re.sub(r"(?<!^)(?=[A-Z])", "_", name).lower()


def add_supported_layer(layer, pruning_func=None):
    """Register a layer type (name, class or instance) whose weights prune_model should sparsify, optionally with
    its own pruning function ``(weight, m, n, mask_algo, param_name) -> (pruned_weight, mask)``."""
    from ..nn import Layer
    if isinstance(layer, str):
        name = layer
    elif isinstance(layer, Layer):
        name = _snake(type(layer).__name__)
    elif isinstance(layer, type) and issubclass(layer, Layer):
        name = _snake(layer.__name__)
    else:
        raise TypeError(f"add_supported_layer expects a name, Layer subclass or instance, got {type(layer)}")
    _supported[name] = pruning_func


def calculate_density(x):
    t = x._t if isinstance(x, Tensor) else torch.as_tensor(x)
    return float((t != 0).sum()) / max(t.numel(), 1)


def create_mask(t, n=2, m=4):
    """Keep the n largest-|w| of every m consecutive weights along the input dimension (dim 0 of a
    paddle [in, out] Linear weight)."""
    w = t.detach().float()
    if w.dim() == 1 or w.shape[0] % m != 0:
        return torch.ones_like(w, dtype=torch.bool)
    x = w.t().reshape(w.shape[1], -1, m) if w.dim() == 2 else w.reshape(-1, m)
    idx = x.abs().topk(n, -1).indices
    mask = torch.zeros_like(x, dtype=torch.bool).scatter_(-1, idx, True)
    return mask.reshape(w.shape[1], -1).t().contiguous() if w.dim() == 2 else mask.reshape(w.shape)


def check_mask_1d(mat, n, m):
    t = mat._t if isinstance(mat, Tensor) else torch.as_tensor(mat)
    if t.shape[-1] % m:
        return False
    return bool(((t.reshape(-1, m) != 0).sum(-1) <= n).all())


def check_sparsity(mat, n=2, m=4, func_name=None):
    t = mat._t if isinstance(mat, Tensor) else torch.as_tensor(mat)
    if t.dim() == 2:
        t = t.t()
    return check_mask_1d(t, n, m)


def set_excluded_layers(param_names, main_program=None):
    _excluded.update(param_names)


def reset_excluded_layers(main_program=None):
    _excluded.clear()


def _prunable(layer):
    out = []
    for name, sub in layer.named_sublayers(include_self=True):
        kind = _snake(type(sub).__name__)
        w = getattr(sub, "weight", None)
        if kind in _supported and w is not None and w.name not in _excluded and name not in _excluded:
            out.append((w, _supported[kind]))
    return out


@no_grad()
def prune_model(model, n=2, m=4, mask_algo="mask_1d", with_mask=True):
    res = {}
    for w, fn in _prunable(model):
        t = w._t
        if fn is not None:  # user pruning function on the host copy
            import numpy as np
            pruned, mk = fn(t.detach().float().cpu().numpy(), m, n, mask_algo, w.name)
            t.copy_(torch.as_tensor(np.asarray(pruned), dtype=t.dtype, device=t.device))
            mk = torch.as_tensor(np.asarray(mk) != 0, device=t.device)
            if with_mask:
                _masks[id(w)] = (w, mk)
            res[w.name] = mk
            continue
        if t.dim() == 4:  # conv [out, in, kh, kw] -> group along in
            mk = create_mask(t.permute(1, 2, 3, 0).reshape(t.shape[1] * t.shape[2] * t.shape[3], t.shape[0]), n, m)
            mk = mk.reshape(t.shape[1], t.shape[2], t.shape[3], t.shape[0]).permute(3, 0, 1, 2)
        else:
            mk = create_mask(t, n, m)
        t.mul_(mk.to(t.dtype))
        if with_mask:
            _masks[id(w)] = (w, mk)
        res[w.name] = mk
    return res


def decorate(optimizer):
    inner_step = optimizer.step

    def step(*a, **k):
        out = inner_step(*a, **k)
        with torch.no_grad():
            for w, mk in _masks.values():
                w._t.mul_(mk.to(w._t.dtype))
        return out
    optimizer.step = step
    return optimizer
