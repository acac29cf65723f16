"""Recompute annotations for auto-parallel programs.

Reference: python/paddle/distributed/auto_parallel/interface.py:210 (``recompute(op)``: the ops it records carry a
recompute id that the static recompute pass, distributed/passes/auto_parallel_recompute.py, turns into segments whose
activations are rebuilt in backward) and :236 (``exclude_ops_in_recompute``).

Here the id is stamped on the traced program's nodes (static/program.py ``Program.recompute_scope``); the static
engine (static_engine.py) runs each contiguous run of one id as a checkpointed segment when
``strategy.recompute.enable`` is set. Eagerly (no program being traced) both wrappers are plain calls.
"""
from __future__ import annotations

import contextlib

from ...framework.trace_hook import _active_program


def _scope(enabled):
    prog = _active_program()
    return prog.recompute_scope(enabled) if prog is not None else contextlib.nullcontext()


class _RecomputeOperator:
    def __init__(self, op, enabled=True):
        self._op = op
        self._enabled = enabled

    def __call__(self, *args, **kwargs):
        with _scope(self._enabled):
            return self._op(*args, **kwargs)


def recompute(op):
    """Mark ``op`` (a layer or function): what it records while a program is traced forms a recompute segment."""
    return _RecomputeOperator(op, True)


def exclude_ops_in_recompute(run_function):
    """Ops recorded by ``run_function`` stay out of the enclosing recompute segment (their outputs are kept)."""
    return _RecomputeOperator(run_function, False)
