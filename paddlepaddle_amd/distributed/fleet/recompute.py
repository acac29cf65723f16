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


def detach_variable(inputs):
    """Detached copies of the tensors in ``inputs`` (tensors or tuples of tensors; anything else passes through),
    each keeping its ``stop_gradient`` flag (reference recompute.py:62 — the helper PaddleNLP's own recompute
    wrappers import)."""
    def one(t):
        if not isinstance(t, Tensor):
            return t
        d = t.detach()
        d.stop_gradient = t.stop_gradient
        return d

    return tuple(tuple(one(i) for i in v) if type(v) is tuple else one(v) for v in inputs)


def check_recompute_necessary(inputs):
    """Warn when no tensor input of a recompute block needs a gradient (recompute.py:98): its backward never
    runs, so checkpointing it only costs a forward."""
    flags = []
    for v in inputs:
        for t in (v if type(v) is tuple else (v,)):
            if isinstance(t, Tensor):
                flags.append(t.stop_gradient)
    if flags and all(flags):
        import logging
        logging.getLogger(__name__).warning(
            "[Recompute]: none of the inputs of this recompute block needs a gradient; recomputing it in backward "
            "is unnecessary")


@contextlib.contextmanager
def switch_rng_state_tracker(rng_state, tracker):
    """Run a block under the given global RNG state and tensor-parallel RNG tracker states, restoring both after
    (recompute.py:116: a recomputed block redraws the forward's dropout masks)."""
    from ... import get_rng_state, set_rng_state
    from ...parallel.tensor_parallel import get_rng_state_tracker
    orig, orig_tracker = get_rng_state(), get_rng_state_tracker().get_states_tracker()
    set_rng_state(rng_state)
    get_rng_state_tracker().set_states_tracker(tracker)
    try:
        yield
    finally:
        set_rng_state(orig)
        get_rng_state_tracker().set_states_tracker(orig_tracker)


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
    """Split ``functions`` (a Sequential or a list of layers) into ``ctx["segments"]`` parts of len // segments
    layers; the first segments - 1 parts are checkpointed, the rest runs plainly (the reference's split,
    recompute.py:659 — with one segment nothing is recomputed). ``ctx["preserve_rng_state"]`` goes to each
    checkpoint."""
    ctx = ctx if isinstance(ctx, dict) else {}
    segments = int(ctx.get("segments", 1))
    kwargs.setdefault("preserve_rng_state", ctx.get("preserve_rng_state", True))
    layers = list(functions.children()) if hasattr(functions, "children") else list(functions)
    size = len(layers) // segments if segments > 0 else len(layers)

    def run(lo, hi):
        def f(*inp):
            x = inp[0] if len(inp) == 1 else inp
            for l in layers[lo:hi]:
                x = l(x)
            return x
        return f

    x = args[0] if len(args) == 1 else args
    end = 0
    for lo in range(0, size * (segments - 1), size):
        end = lo + size
        x = recompute(run(lo, end), *(x if isinstance(x, tuple) else (x,)), **kwargs)
    return run(end, len(layers))(*(x if isinstance(x, tuple) else (x,)))


def recompute_hybrid(ctx, function, *args, **kwargs):
    return recompute(function, *args, **kwargs)
