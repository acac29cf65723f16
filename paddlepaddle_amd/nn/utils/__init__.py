"""paddle.nn.utils. Reference: python/paddle/nn/utils/*.py."""
from __future__ import annotations

import torch

from ...framework.tensor import Parameter, Tensor, _wrap
from ..clip import clip_grad_norm_, clip_grad_value_  # noqa: F401


def parameters_to_vector(parameters, name=None):
    return _wrap(torch.cat([p._t.reshape(-1) for p in parameters]))


def vector_to_parameters(vec, parameters, name=None):
    v = vec._t
    off = 0
    with torch.no_grad():
        for p in parameters:
            n = p._t.numel()
            p._t.copy_(v[off:off + n].view_as(p._t))
            off += n


def weight_norm(layer, name="weight", dim=0):
    w = getattr(layer, name)
    t = w._t.detach()
    if dim is None:
        g = t.norm()
    else:
        red = [i for i in range(t.dim()) if i != dim]
        g = t.norm(dim=red, keepdim=True) if red else t.abs()
    g_p = Parameter(g.clone())
    v_p = Parameter(t.clone())
    del layer._parameters[name]
    layer.add_parameter(name + "_g", g_p)
    layer.add_parameter(name + "_v", v_p)

    def _compute(l, inputs):
        v = l._parameters[name + "_v"]._t
        gg = l._parameters[name + "_g"]._t
        if dim is None:
            wv = v * (gg / v.norm())
        else:
            red = [i for i in range(v.dim()) if i != dim]
            wv = v * (gg / v.norm(dim=red, keepdim=True))
        object.__setattr__(l, name, _wrap(wv))
    h = layer.register_forward_pre_hook(_compute)
    layer.__dict__["_weight_norm_hook"] = (h, name, dim)
    _compute(layer, None)
    return layer


def remove_weight_norm(layer, name="weight"):
    h, name, dim = layer.__dict__.pop("_weight_norm_hook")
    h.remove()
    w = layer.__dict__.pop(name)
    del layer._parameters[name + "_g"]
    del layer._parameters[name + "_v"]
    layer.add_parameter(name, Parameter(w._t.detach().clone()))
    return layer


def spectral_norm(layer, name="weight", n_power_iterations=1, eps=1e-12, dim=None):
    from ..layer.norm import SpectralNorm
    w = getattr(layer, name)
    if dim is None:
        dim = 0
    sn = SpectralNorm(w.shape, dim, n_power_iterations, eps)
    orig = Parameter(w._t.detach().clone())
    del layer._parameters[name]
    layer.add_parameter(name + "_orig", orig)
    layer.add_sublayer(name + "_sn", sn)

    def _compute(l, inputs):
        object.__setattr__(l, name, sn(l._parameters[name + "_orig"]))
    layer.register_forward_pre_hook(_compute)
    _compute(layer, None)
    return layer
