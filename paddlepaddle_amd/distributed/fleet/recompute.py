"""Activation recompute. Reference: python/paddle/distributed/fleet/recompute/recompute.py:459
(recompute), recompute_sequential, recompute_hybrid.

Uses the native non-reentrant checkpoint machinery: only the block input is kept; the block is
re-run in backward under the saved RNG state (dropout masks identical)."""
from __future__ import annotations

import contextlib

import torch
import torch.utils.checkpoint as _ckpt

from ...framework.tensor import Tensor, _wrap


def _u(x):
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, (list, tuple)):
        return type(x)(_u(v) for v in x)
    return x


def _w(x):
    if isinstance(x, torch.Tensor):
        return _wrap(x)
    if isinstance(x, (list, tuple)):
        return type(x)(_w(v) for v in x)
    return x


def recompute(function, *args, **kwargs):
    preserve = kwargs.pop("preserve_rng_state", True)
    kwargs.pop("use_reentrant", None)
    kwargs.pop("offload_indices", None)
    from ...framework.trace_hook import _active_program
    prog = _active_program()
    if prog is not None:  # traced into a static program: the block becomes a recompute segment of the program
        with prog.recompute_scope():
            return function(*args, **kwargs)

    def f(*targs):
        return _u(function(*[_w(a) for a in targs], **kwargs))

    from ...ops import linear as LIN
    mode = LIN.capture_forward_mode()  # the recompute inside backward takes the forward's op routing
    out = _ckpt.checkpoint(f, *[_u(a) for a in args], use_reentrant=False, preserve_rng_state=preserve,
                           context_fn=lambda: (contextlib.nullcontext(), LIN.forward_mode(mode)))
    return _w(out)


def recompute_sequential(ctx, functions, *args, **kwargs):
    segments = ctx.get("segments", 1) if isinstance(ctx, dict) else 1
    layers = list(functions.children()) if hasattr(functions, "children") else list(functions)
    n = len(layers)
    seg = max(n // segments, 1)
    x = args[0] if len(args) == 1 else args

    def run(lo, hi):
        def f(inp):
            for l in layers[lo:hi]:
                inp = l(inp)
            return inp
        return f
    for lo in range(0, n, seg):
        x = recompute(run(lo, min(lo + seg, n)), x, **kwargs)
    return x


def recompute_hybrid(ctx, function, *args, **kwargs):
    return recompute(function, *args, **kwargs)
