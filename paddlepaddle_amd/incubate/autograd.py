"""paddle.incubate.autograd (functional forward/reverse-mode AD). Reference:
python/paddle/incubate/autograd/functional.py (vjp, jvp, Jacobian, Hessian)."""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor, _wrap
from ..autograd import Jacobian, jacobian, hessian  # noqa: F401


def _fn(func):
    def f(*xs):
        out = func(*[_wrap(x) for x in xs])
        if isinstance(out, (list, tuple)):
            return tuple(o._t for o in out)
        return out._t
    return f


def _ts(x):
    return tuple(v._t for v in x) if isinstance(x, (list, tuple)) else (x._t,)


def vjp(func, xs, v=None):
    ys, g = torch.autograd.functional.vjp(_fn(func), _ts(xs), None if v is None else _ts(v))
    wrap = (lambda t: tuple(_wrap(a) for a in t) if isinstance(t, tuple) else _wrap(t))
    gs = wrap(g)
    return wrap(ys), (gs if isinstance(xs, (list, tuple)) else gs[0] if isinstance(gs, tuple) else gs)


def jvp(func, xs, v=None):
    ys, g = torch.autograd.functional.jvp(_fn(func), _ts(xs), None if v is None else _ts(v))
    wrap = (lambda t: tuple(_wrap(a) for a in t) if isinstance(t, tuple) else _wrap(t))
    return wrap(ys), wrap(g)


class Hessian:
    def __init__(self, func, xs, is_batched=False):
        self.func, self.xs = func, xs
        H = torch.autograd.functional.hessian(_fn(func), _ts(xs))
        self._t = H[0][0] if isinstance(H, tuple) else H

    def __getitem__(self, idx):
        return _wrap(self._t[idx])

    @property
    def shape(self):
        return list(self._t.shape)


def enable_prim():
    pass


def disable_prim():
    pass


def prim_enabled():
    return False


def grad(outputs, inputs, grad_outputs=None):
    """Reverse-mode gradients (reference incubate.autograd.grad over primitive ops)."""
    from ..autograd import grad as _grad
    single = not isinstance(inputs, (list, tuple))
    r = _grad(outputs, inputs, grad_outputs, create_graph=True, allow_unused=True)
    return r[0] if single and isinstance(r, (list, tuple)) else r


def forward_grad(outputs, inputs, grad_inputs=None):
    """Forward-mode directional derivative d outputs / d inputs . grad_inputs, computed as the transpose of
    a VJP (double-backward), which needs no separate forward-mode rules."""
    import torch
    outs = outputs if isinstance(outputs, (list, tuple)) else [outputs]
    ins = inputs if isinstance(inputs, (list, tuple)) else [inputs]
    if grad_inputs is None:
        gins = [torch.ones_like(i._t) for i in ins]
    else:
        gins = [g._t for g in (grad_inputs if isinstance(grad_inputs, (list, tuple)) else [grad_inputs])]
    us = [torch.zeros_like(o._t, requires_grad=True) for o in outs]
    vjp = torch.autograd.grad([o._t for o in outs], [i._t for i in ins], us, create_graph=True, allow_unused=True)
    pairs = [(v, g) for v, g in zip(vjp, gins) if v is not None]
    jv = torch.autograd.grad([v for v, _ in pairs], us, [g for _, g in pairs], create_graph=True, allow_unused=True)
    res = [_wrap(j if j is not None else torch.zeros_like(u)) for j, u in zip(jv, us)]
    return res if isinstance(outputs, (list, tuple)) else res[0]
