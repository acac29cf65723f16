"""paddle.autograd. Reference: python/paddle/autograd/{py_layer.py, backward_mode.py, autograd.py}.

PyLayer user code (paddle Tensors) runs inside a native autograd Function node; backward()/grad()
drive the native graph traversal of the HIP runtime's autograd engine."""
from __future__ import annotations

import contextlib

import torch

from ..framework.tensor import Tensor, _wrap


def _u(x):
    return x._t if isinstance(x, Tensor) else x


def _w(x):
    return _wrap(x) if isinstance(x, torch.Tensor) else x


class PyLayerContext:
    def __init__(self, tctx):
        object.__setattr__(self, "_tctx", tctx)
        object.__setattr__(self, "_saved", ())
        object.__setattr__(self, "_attrs", {})

    def save_for_backward(self, *tensors):
        object.__setattr__(self, "_saved", tensors)
        self._tctx.save_for_backward(*[_u(t) if isinstance(t, Tensor) else None for t in tensors])

    def saved_tensor(self):
        ts = self._tctx.saved_tensors
        return tuple(_w(t) if t is not None else s for t, s in zip(ts, self._saved))

    saved_tensors = property(saved_tensor)

    def mark_not_inplace(self, *args):
        pass

    def mark_non_differentiable(self, *args):
        self._tctx.mark_non_differentiable(*[_u(a) for a in args])

    def set_materialize_grads(self, value):
        self._tctx.set_materialize_grads(value)

    def __getattr__(self, k):
        try:
            return self._attrs[k]
        except KeyError:
            raise AttributeError(k)

    def __setattr__(self, k, v):
        self._attrs[k] = v


class _PyLayerMeta(type):
    def __init__(cls, name, bases, attrs):
        super().__init__(name, bases, attrs)
        cls._torch_fn = None


class PyLayer(metaclass=_PyLayerMeta):
    @staticmethod
    def forward(ctx, *args, **kwargs):
        raise NotImplementedError

    @staticmethod
    def backward(ctx, *args):
        raise NotImplementedError

    @classmethod
    def apply(cls, *args, **kwargs):
        user = cls

        class _Fn(torch.autograd.Function):
            @staticmethod
            def forward(tctx, *targs):
                ctx = PyLayerContext(tctx)
                tctx._pctx = ctx
                wargs = [_w(a) for a in targs]
                with torch.enable_grad() if False else contextlib.nullcontext():
                    out = user.forward(ctx, *wargs, **kwargs)
                tctx._tuple_out = isinstance(out, (tuple, list))
                outs = out if isinstance(out, (tuple, list)) else (out,)
                res = tuple(_u(o) for o in outs)
                # outputs must not alias inputs for the native engine
                ins = {id(a) for a in targs if isinstance(a, torch.Tensor)}
                res = tuple(r.view_as(r) if isinstance(r, torch.Tensor) and id(r) in ins else r for r in res)
                return res if tctx._tuple_out else res[0]

            @staticmethod
            def backward(tctx, *grads):
                ctx = tctx._pctx
                g = user.backward(ctx, *[_w(x) for x in grads])
                gs = g if isinstance(g, (tuple, list)) else (g,)
                gs = [_u(x) for x in gs]
                out = []
                it = iter(gs)
                for a in tctx._targs_mask:
                    out.append(next(it, None) if a else None)
                return tuple(out)

        targs = tuple(_u(a) for a in args)
        mask = [isinstance(a, torch.Tensor) for a in targs]
        orig_fwd = _Fn.forward

        def fwd(tctx, *ta):
            tctx._targs_mask = mask
            return orig_fwd(tctx, *ta)
        _Fn.forward = staticmethod(fwd)
        out = _Fn.apply(*targs)
        if isinstance(out, tuple):
            return tuple(_w(o) for o in out)
        return _w(out)


LegacyPyLayer = PyLayer
EagerPyLayer = PyLayer
EagerPyLayerContext = PyLayerContext


def backward(tensors, grad_tensors=None, retain_graph=False):
    """paddle.autograd.backward: a missing (None) gradient of any output — scalar or not — is ones_like(output).
    Reference: python/paddle/autograd/backward_mode.py backward."""
    ts = [tensors] if isinstance(tensors, Tensor) else list(tensors)
    gs = [None] * len(ts)
    if grad_tensors is not None:
        gl = [grad_tensors] if isinstance(grad_tensors, Tensor) else list(grad_tensors)
        if len(gl) != len(ts):
            raise ValueError("The length of grad_tensors must be equal to the length of tensors")
        gs = [None if g is None else _u(g) for g in gl]
    gs = [torch.ones_like(t._t) if g is None else g for t, g in zip(ts, gs)]
    from . import engine as _eng
    if _eng.use_native():
        _eng.backward([t._t for t in ts], gs, retain_graph=retain_graph)
        return
    torch.autograd.backward([t._t for t in ts], gs, retain_graph=retain_graph)


def grad(outputs, inputs, grad_outputs=None, retain_graph=None, create_graph=False, only_inputs=True,
         allow_unused=False, no_grad_vars=None):
    outs = [outputs] if isinstance(outputs, Tensor) else list(outputs)
    ins = [inputs] if isinstance(inputs, Tensor) else list(inputs)
    gos = None
    if grad_outputs is not None:
        gos = [grad_outputs] if isinstance(grad_outputs, Tensor) else list(grad_outputs)
        gos = [None if g is None else _u(g) for g in gos]
    rg = create_graph if retain_graph is None else retain_graph
    from . import engine as _eng
    if _eng.use_native():
        gl = [torch.ones_like(o._t) if (gos is None or gos[k] is None) else gos[k] for k, o in enumerate(outs)]
        res = _eng.grad([o._t for o in outs], [i._t for i in ins], gl, create_graph=create_graph,
                        allow_unused=allow_unused)
        return [None if r is None else _wrap(r) for r in res]
    res = torch.autograd.grad([o._t for o in outs], [i._t for i in ins], gos, retain_graph=rg,
                              create_graph=create_graph, allow_unused=allow_unused)
    return [None if r is None else _wrap(r) for r in res]


def _as_fn(func):
    def f(*ts):
        r = func(*[_wrap(t) for t in ts])
        if isinstance(r, (tuple, list)):
            return tuple(_u(x) for x in r)
        return _u(r)
    return f


class Jacobian:
    def __init__(self, j):
        self._j = j

    def __getitem__(self, idx):
        return _wrap(self._j[idx])

    @property
    def shape(self):
        return list(self._j.shape)

    def numpy(self):
        return self._j.detach().cpu().numpy()


def jacobian(ys, xs, batch_axis=None):
    """paddle.autograd.jacobian(ys, xs): J[i, j] = d ys_i / d xs_j (flattened)."""
    single_x = isinstance(xs, Tensor)
    xl = [xs] if single_x else list(xs)
    y = ys if isinstance(ys, Tensor) else ys[0]
    yf = y._t.reshape(-1)
    rows = []
    for i in range(yf.numel()):
        g = torch.autograd.grad(yf[i], [x._t for x in xl], retain_graph=True, allow_unused=True)
        rows.append([torch.zeros_like(x._t).reshape(-1) if gi is None else gi.reshape(-1) for gi, x in zip(g, xl)])
    js = [torch.stack([r[k] for r in rows]) for k in range(len(xl))]
    return Jacobian(js[0]) if single_x else [Jacobian(j) for j in js]


def hessian(ys, xs, batch_axis=None):
    single_x = isinstance(xs, Tensor)
    xl = [xs] if single_x else list(xs)
    g = torch.autograd.grad(ys._t, [x._t for x in xl], create_graph=True)
    gf = torch.cat([gi.reshape(-1) for gi in g])
    rows = []
    for i in range(gf.numel()):
        h = torch.autograd.grad(gf[i], [x._t for x in xl], retain_graph=True, allow_unused=True)
        rows.append(torch.cat([torch.zeros_like(x._t).reshape(-1) if hi is None else hi.reshape(-1)
                               for hi, x in zip(h, xl)]))
    return Jacobian(torch.stack(rows))


class saved_tensors_hooks:
    def __init__(self, pack_hook, unpack_hook):
        self._ctx = torch.autograd.graph.saved_tensors_hooks(
            lambda t: pack_hook(_wrap(t)), lambda p: _u(unpack_hook(p)))

    def __enter__(self):
        self._ctx.__enter__()
        return self

    def __exit__(self, *a):
        return self._ctx.__exit__(*a)


from ..framework.grad_mode import no_grad, enable_grad, set_grad_enabled, is_grad_enabled  # noqa: E402,F401
