"""Minimal hook the hot ops use to take part in static-graph tracing (kept dependency-free so the
``ops`` package can import it before ``static`` exists). See static/program.py."""
from __future__ import annotations

import functools
import threading

import torch

_state = threading.local()


def _active_program():
    st = getattr(_state, "stack", None)
    return st[-1].program if st else None


def static_op(fn):
    """Decorator for hot ops in ``ops/``: while tracing, record the whole op as ONE node so the HIP
    kernel (not its decomposition) runs at replay; otherwise a plain call-through."""

    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        prog = _active_program()
        if prog is None or getattr(_state, "in_op", False) or not prog._any((args, kwargs), prog._is_traced):
            return fn(*args, **kwargs)
        from ..static.program import OpNode
        _state.in_op = True
        try:
            with torch._C.DisableTorchFunction():
                targs, tkw = prog._template(args), prog._template(kwargs)
                out = fn(*prog._to_meta(args), **prog._to_meta(kwargs))
        finally:
            _state.in_op = False
        node = OpNode(wrapper, targs, tkw, None, kind="op", name="o:" + fn.__module__ + ":" + fn.__name__)
        node.outs = prog._out_template(out)
        prog._append(node)
        return out

    wrapper.__wrapped_static__ = fn
    return wrapper
