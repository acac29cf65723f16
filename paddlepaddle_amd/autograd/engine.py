"""Eager backward engine selection and the Python half of the native engine.

``FLAGS_eager_backward_engine``:
  * ``native`` — backward()/paddle.grad run through ``_C_autograd.run_backward``
    (csrc/autograd/autograd_exec.cpp: C++ over the Node interface, saved tensors released as nodes run; the
    pybind traversal csrc/runtime/autograd_engine.cpp when that extension is absent): in-degree map over the
    reachable grad-node graph, ready queue,
    per-slot gradient sums, gradient hooks applied to the summed slot, paddle.grad pruning + capture.
    Reference: paddle/fluid/eager/backward.cc:105 (RunBackward), general_grad.h (paddle.grad).
  * ``torch`` — PyTorch-ROCm's C++ autograd engine runs the same grad nodes (multi-threaded device queues).
``native`` is the default (same 13B throughput as torch's engine, faster when launch-bound:
profiles/r3_passes_costmodel.md).

Grad nodes are the per-op backward functions: the autograd functions of the hand-written HIP kernels
(ops/*.py) and ATen's derivative formulas. Gradient hooks registered with ``Tensor.register_hook`` go into a
table keyed by the tensor's gradient edge (node, slot) that this engine applies; tensors' post-accumulate hooks
(DataParallel / sharding grad-ready hooks) run inside the leaf accumulation node under both engines.
"""
from __future__ import annotations

import torch

from ..framework.flags import get_flags

_HOOKS: dict = {}     # (node, slot) -> [fn(torch grad) -> torch grad | None]
_FINAL: list = []     # callbacks queued during a native backward, run once it has finished
_ACTIVE = [0]         # depth of native backward passes in flight


def queue_callback(fn):
    """Run ``fn`` once the current backward pass has finished, under either engine (the gradient-ready
    hooks of DataParallel / sharding / segment parallel use it to flush their last bucket)."""
    if _ACTIVE[0]:
        _FINAL.append(fn)
    else:
        torch.autograd.Variable._execution_engine.queue_callback(fn)


def _drain():
    while _FINAL:
        _FINAL.pop(0)()


def engine_name():
    try:
        return str(get_flags("FLAGS_eager_backward_engine")["FLAGS_eager_backward_engine"])
    except Exception:  # pragma: no cover
        return "torch"


def use_native():
    if engine_name() != "native":
        return False
    from ..utils import native
    m = native.module()
    return m is not None and hasattr(m, "run_backward")


def _edge(t):
    e = torch.autograd.graph.get_gradient_edge(t)
    return e.node, e.output_nr


def add_hook(t, fn):
    """Register a gradient hook for ``t`` in the native engine's table; returns a remover."""
    key = _edge(t)
    lst = _HOOKS.setdefault(key, [])
    lst.append(fn)

    def remove():
        if fn in lst:
            lst.remove(fn)
        if not lst:
            _HOOKS.pop(key, None)
    return remove


def runs_tensor_hooks():
    """True when native backward runs torch's tensor hook lists itself (the C++ executor does, like torch's
    engine); the pybind fallback traversal applies only the (node, slot) table."""
    return _executor() is not None


def register_grad_hook(t, fn):
    """Gradient hook on a torch tensor under whichever engine will run its backward (torch's hook list, or
    this engine's (node, slot) table)."""
    if use_native() and not runs_tensor_hooks():
        # pybind fallback: both tables. It applies its own (node, slot) table; a backward that some code starts
        # through torch's engine directly (recompute / pipeline schedules) runs torch's hook list.
        rm = add_hook(t, fn)
        h = t.register_hook(fn)

        def remove():
            rm()
            h.remove()
        return remove
    h = t.register_hook(fn)
    return h.remove


def retain(t):
    """Tensor.retain_grads under the native engine: store the summed slot gradient into ``t.grad``."""
    import warnings
    import weakref
    if t.is_leaf:
        return
    ref = weakref.ref(t)

    def h(g):
        x = ref()
        if x is not None:
            with warnings.catch_warnings():  # reading .grad of a non-leaf without torch's retain flag warns
                warnings.simplefilter("ignore")
                cur = x.grad
            x.grad = g.detach() if cur is None else cur + g.detach()
        return None
    if runs_tensor_hooks():
        # a tensor pre-hook in registration order (Paddle: retain_grads is a gradient hook like any other, so
        # a hook registered after it does not change the retained value)
        t.register_hook(h)
        return
    t.retain_grad()  # marks .grad readable on the non-leaf; the value is written by the hook below
    key = _edge(t)
    _HOOKS.setdefault(key, []).insert(0, h)


def _zeros_for(node, slot):
    m = node._input_metadata[slot]
    return torch.zeros(tuple(m.shape), dtype=m.dtype, device=m.device)


def _fix(g, node, slot):
    """validate_outputs: a gradient flowing into a node's slot takes that slot's dtype and shape
    (sum over broadcast dims)."""
    try:
        m = node._input_metadata[slot]
    except (IndexError, AttributeError, RuntimeError):
        return g
    if g.dtype != m.dtype and (m.dtype.is_floating_point or m.dtype.is_complex):
        g = g.to(m.dtype)
    shp = tuple(m.shape)
    if tuple(g.shape) != shp and len(shp) <= g.dim():
        try:
            g = g.sum_to_size(shp)
        except RuntimeError:
            pass
    return g


def _is_py(node):
    return isinstance(node, torch.autograd.function.BackwardCFunction)


_HELPERS = (_zeros_for, _fix, _is_py)


_EXEC = []


def _executor():
    """``_C_autograd`` (csrc/autograd/autograd_exec.cpp): the executor over the C++ Node interface; None when the
    extension is not built (the pybind traversal in _C_runtime is used then)."""
    if not _EXEC:
        try:
            from .. import _C_autograd
            _EXEC.append(_C_autograd)
        except ImportError:
            _EXEC.append(None)
    return _EXEC[0]


def _run(outs, grads, ins, create_graph, retain_graph=None):
    from ..utils import native
    for t in outs:
        if not t.requires_grad:
            raise RuntimeError("backward: the output tensor has stop_gradient=True (no grad node to start from)")
    keep = create_graph if retain_graph is None else bool(retain_graph)
    ex = _executor()
    _ACTIVE[0] += 1
    ok = False
    try:
        if ex is not None:
            res = ex.run_backward(list(zip(outs, grads)), list(ins), _HOOKS, keep, create_graph)
        else:
            roots = [(*_edge(t), g) for t, g in zip(outs, grads)]
            with torch.set_grad_enabled(create_graph):
                res = native.module().run_backward(roots, [_edge(t) for t in ins], _HOOKS, _HELPERS)
        ok = True
    finally:
        _ACTIVE[0] -= 1
        if not _ACTIVE[0] and not ok:
            # a failed backward must not leave its flush callbacks (DataParallel / sharding finalizers) to fire
            # at the end of the next, unrelated backward; their owners may queue again on the next pass
            for fn in _FINAL:
                owner = getattr(fn, "__self__", None)
                if owner is not None and getattr(owner, "_queued", False):
                    owner._queued = False
            _FINAL.clear()
    if not _ACTIVE[0]:
        _drain()
    return res


def backward(outs, grads, retain_graph=False):
    """Run backward from ``outs`` (torch tensors) seeded with ``grads``; leaves accumulate into ``.grad``.
    Hooks of non-leaf tensors belong to this graph and are dropped afterwards unless ``retain_graph``."""
    _run(outs, grads, [], False, retain_graph)
    if not retain_graph:
        for k in [k for k in _HOOKS if not isinstance(k[0], _ACC)]:
            del _HOOKS[k]


_ACC = type(torch.autograd.graph.get_gradient_edge(torch.zeros(1, requires_grad=True)).node)


def grad(outs, ins, grads, create_graph=False, allow_unused=False, retain_graph=None):
    for t in ins:
        if not t.requires_grad:
            raise RuntimeError("paddle.grad: an input tensor has stop_gradient=True")
    res = _run(outs, grads, ins, create_graph, retain_graph)
    for r in res:
        if r is None and not allow_unused:
            raise RuntimeError("paddle.grad: one of the inputs is not reachable from the outputs; "
                               "set allow_unused=True to return None for it")
    if not create_graph:
        res = [None if r is None else r.detach() for r in res]
    return res
