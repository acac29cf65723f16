"""paddle.jit.sot.symbolic_translate and the SOT-backed StaticFunction (reference: python/paddle/jit/sot/
translate.py:31, opcode_translator/transform.py — the eval-frame callback that translates a frame's
bytecode and caches the result under guards).

``symbolic_translate(fn)`` returns a callable that, per call:
  1. binds the arguments to ``fn``'s signature; the tensor leaves form the input signature (shape, dtype,
     stop_gradient) together with the grad mode;
  2. tries the cached translations of that signature: the first whose guards (guards.py) hold replays its
     program — nodes in recorded order: tensor ops, dual-trace guards (data-dependent branches), replayed
     side effects and graph breaks (opcode_executor.py);
  3. otherwise translates the bytecode again (up to ``MAX_ENTRIES`` per signature), or falls back to the
     plain function when the translator meets a construct it does not model.
Statistics of the last translation (breaks, side effects, inlined frames, guards) are on ``.last_info``.
"""
from __future__ import annotations

import functools
import inspect
import warnings

import torch

from ...framework.tensor import Tensor
from ...static import program as P
from .. import _flatten, _Leaf, _out_template, _rebuild_out
from .guards import Source
from .opcode_executor import Unsupported, _wrap_tree, translate

__all__ = ["symbolic_translate", "SOTFunction"]

MAX_ENTRIES = 8


class _Entry:
    def __init__(self, key, guards, prog, feed_slots, out_tmpl, fetch, info, rt_out=None):
        self.key, self.guards, self.prog = key, guards, prog
        self.rt_out = rt_out  # the return value is a runtime Python value (computed after a graph break)
        self.feed_slots, self.out_tmpl, self.fetch, self.info = feed_slots, out_tmpl, fetch, info
        self.first = True

    def run(self, leaves, dev):
        env = {s: t._t for s, t in zip(self.feed_slots, leaves)}
        first, self.first = self.first, False
        for n in self.prog.nodes:
            if first and n.kind == "py" and not n.func.idempotent:
                # ran during the translation already; reuse its tensor results
                if n.outs is not None and (n.func.first is not None or n.func.mode == "rt"):
                    P._assign(n.outs, n.func.first, env)
                continue
            P._exec_node(n, env, None, dev, None)
        if self.rt_out is not None:
            return _wrap_tree(env[self.rt_out])
        return _rebuild_out(self.out_tmpl, [env[s] for s in self.fetch])


class SOTFunction:
    def __init__(self, fn, instance=None):
        self._fn = fn
        self._instance = instance
        self._sig = inspect.signature(fn)
        self._entries = {}
        self._eager = set()
        self.last_info = None
        functools.update_wrapper(self, fn)

    def __get__(self, instance, owner):
        if instance is None:
            return self
        key = "_sot_fn_" + self._fn.__name__
        bound = instance.__dict__.get(key)
        if bound is None:
            bound = SOTFunction(self._fn, instance)
            instance.__dict__[key] = bound
        return bound

    def _eager_call(self, args, kwargs):
        return self._fn(*args, **kwargs)

    def __call__(self, *args, **kwargs):
        from .. import _enabled
        if self._instance is not None:
            args = (self._instance,) + args
        if not _enabled or P._active_program():
            return self._eager_call(args, kwargs)
        bound = self._sig.bind(*args, **kwargs)
        bound.apply_defaults()
        arguments = dict(bound.arguments)
        leaves = []
        struct = _flatten(arguments, leaves)
        tensor_sig = tuple((tuple(t.shape), str(t._t.dtype), t._t.device.type, t.stop_gradient) for t in leaves)
        skey = (repr({k: v for k, v in struct.items() if _has_leaf(v)}), tensor_sig, torch.is_grad_enabled())
        if skey in self._eager:
            return self._eager_call(args, kwargs)
        dev = leaves[0]._t.device if leaves else torch.device("cpu")
        entries = self._entries.setdefault(skey, [])
        for i, e in enumerate(entries):
            if not e.guards.check(arguments, self._fn):
                continue
            try:
                out = e.run(leaves, dev)
            except P.GuardFailure:
                continue
            if i:
                entries.insert(0, entries.pop(i))
            self.last_info = e.info
            return out
        if len(entries) >= MAX_ENTRIES:
            warnings.warn(f"symbolic_translate: {self._fn.__qualname__} needed more than {MAX_ENTRIES} "
                          "translations for one input signature; running it eagerly")
            self._eager.add(skey)
            return self._eager_call(args, kwargs)
        try:
            e = self._translate(skey, arguments, struct, leaves)
        except Unsupported as ex:
            warnings.warn(f"symbolic_translate: {self._fn.__qualname__} runs eagerly ({ex})")
            self._eager.add(skey)
            return self._eager_call(args, kwargs)
        entries.insert(0, e)
        self.last_info = e.info
        return e.run(leaves, dev)

    def _translate(self, skey, arguments, struct, leaves):
        prog = P.Program()
        feed_slots = []
        ph = []
        for i, t in enumerate(leaves):
            v = P.placeholder(prog, f"x{i}", t.shape, t.dtype, need_grad=not t.stop_gradient)
            feed_slots.append(prog.feeds[v._name][0])
            ph.append(v)

        def fill(x):
            if isinstance(x, _Leaf):
                return ph[x.i]
            if isinstance(x, (list, tuple)) and not hasattr(x, "_fields"):
                return type(x)(fill(v) for v in x)
            if isinstance(x, dict):
                return {k: fill(v) for k, v in x.items()}
            return x
        arg_values = {}
        for name, v in struct.items():
            if _has_leaf(v):
                arg_values[name] = (fill(v), None)
            else:
                arg_values[name] = (arguments[name], Source("arg", name))
        prog._shadow = {s: t._t for s, t in zip(feed_slots, leaves)}
        prog._shadow_dev = leaves[0]._t.device if leaves else torch.device("cpu")
        try:
            outv, tr = translate(self._fn, (), {}, prog, arg_values)
        finally:
            prog._shadow = None
        fetch = []
        tmpl = _out_template(prog, outv.v, fetch) if outv.slot is None else None
        info = {"breaks": tr.breaks, "side_effects": tr.effects, "inlined_frames": tr.inlined,
                "guards": [repr(g) for g in tr.guards], "nodes": len(prog.nodes),
                "dual_guards": sum(1 for n in prog.nodes if n.kind == "guard")}
        return _Entry(skey, tr.guards, prog, feed_slots, tmpl, fetch, info, outv.slot)

    @property
    def translations(self):
        return [e for es in self._entries.values() for e in es]


def _has_leaf(x):
    if isinstance(x, _Leaf):
        return True
    if isinstance(x, (list, tuple)):
        return any(_has_leaf(v) for v in x)
    if isinstance(x, dict):
        return any(_has_leaf(v) for v in x.values())
    return False


def symbolic_translate(fn, training=True, **kwargs):
    """Translate ``fn`` (a function, or a Layer: its forward) through the bytecode executor."""
    from ...nn.layer.layers import Layer
    if isinstance(fn, Layer):
        sf = SOTFunction(type(fn).forward, instance=fn)
        fn.__dict__["forward"] = sf
        return fn
    return SOTFunction(fn)
