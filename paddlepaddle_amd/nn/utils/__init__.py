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


def _norm_except(v, dim):
    """2-norm over every axis but ``dim`` (all axes when dim is None), shaped to broadcast against v."""
    if dim is None:
        return (v * v).sum().sqrt()
    red = [i for i in range(v.dim()) if i != dim]
    return (v * v).sum(dim=red, keepdim=True).sqrt() if red else v.abs()


def weight_norm(layer, name="weight", dim=0):
    """w = g * v / ||v|| (reference nn/utils/weight_norm_hook.py): weight_g has the shape of the kept axis
    (``[out]`` for dim 0), weight_v the weight's."""
    w = getattr(layer, name)
    t = w._t.detach()
    if dim is not None and dim < 0:
        dim += t.dim()
    n = _norm_except(t, dim)
    g = n.reshape(t.shape[dim]) if dim is not None else n.reshape([])
    g_p = Parameter(g.clone())
    v_p = Parameter(t.clone())
    del layer._parameters[name]
    layer.add_parameter(name + "_g", g_p)
    layer.add_parameter(name + "_v", v_p)

    def _compute(l, inputs):
        v = l._parameters[name + "_v"]._t
        gg = l._parameters[name + "_g"]._t
        nv = _norm_except(v, dim)
        wv = v * (gg.reshape(nv.shape) / nv)
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
