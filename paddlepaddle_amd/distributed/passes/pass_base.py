"""Program pass framework (reference: python/paddle/distributed/passes/pass_base.py:20-380).

A pass rewrites the node list of a traced static ``Program`` (static/program.py: OpNode records of torch /
HIP-op calls over value slots) or sets program attributes the Executor honours. ``new_pass(name, attrs)``
builds a registered pass; ``PassManager`` applies a list of them in a valid order.

Ordering / conflicts are declared, not searched: each pass class names the passes it must run after
(``_after``) and the ones it cannot be combined with (``_conflicts``). The manager drops passes whose
``_check_self`` fails or that conflict with an already-applied (or earlier kept) pass, then orders the rest
topologically by ``_after`` (stable with respect to the given order). The reference instead builds a
conflict matrix and searches the longest compatible path; with explicit declarations the order is
deterministic and explainable.
"""
from __future__ import annotations

from abc import ABC, abstractmethod

__all__ = ["PassContext", "PassType", "PassBase", "register_pass", "new_pass", "PassManager"]


class PassContext:
    """What has been applied so far plus free-form attributes passes share."""

    def __init__(self):
        self._applied = []
        self._attrs = {}

    def set_attr(self, key, value):
        self._attrs[key] = value

    def get_attr(self, key, default=None):
        return self._attrs.get(key, default)

    @property
    def passes(self):
        return self._applied

    def _add_pass(self, p):
        self._applied.append(p)

    def _pop_pass(self):
        return self._applied.pop()


class PassType:
    UNKNOWN = 0
    COMM_OPT = 1
    CALC_OPT = 2
    PARALLEL_OPT = 3
    FUSION_OPT = 4


class PassBase(ABC):
    _REGISTERED_PASSES: dict = {}
    name = None
    _after: tuple = ()        # names of passes that must run before this one when both are applied
    _conflicts: tuple = ()    # names of passes this one cannot be combined with

    def __init__(self):
        self._attrs = {}

    def set_attr(self, key, value):
        self._attrs[key] = value
        return self

    def get_attr(self, key, default=None):
        return self._attrs.get(key, default)

    def _check_self(self):
        return True

    def _check_conflict(self, other):
        return other.name not in self._conflicts and self.name not in getattr(other, "_conflicts", ())

    def _type(self):
        return PassType.UNKNOWN

    def apply(self, main_programs, startup_programs, context=None):
        context = PassContext() if context is None else context
        if not self._check_self() or not all(self._check_conflict(p) for p in context.passes):
            return context
        if not isinstance(main_programs, (list, tuple)):
            main_programs, startup_programs = [main_programs], [startup_programs]
        if len(main_programs) != len(startup_programs):
            raise ValueError("main_programs and startup_programs must pair up")
        for m, s in zip(main_programs, startup_programs):
            self._apply_single_impl(m, s, context)
            m._version += 1
            m._plans.clear()  # cached execution plans refer to the old node list
        context._add_pass(self)
        return context

    @abstractmethod
    def _apply_single_impl(self, main_program, startup_program, context):
        ...


def register_pass(name):
    def deco(cls):
        PassBase._REGISTERED_PASSES[name] = cls
        cls.name = name
        return cls
    return deco


def new_pass(name, pass_attrs=None):
    cls = PassBase._REGISTERED_PASSES.get(name)
    if cls is None:
        raise ValueError(f"pass '{name}' is not registered; known: {sorted(PassBase._REGISTERED_PASSES)}")
    p = cls()
    for k, v in (pass_attrs or {}).items():
        p.set_attr(k, v)
    return p


def _order(passes, context):
    kept = []
    for p in passes:
        if not p._check_self():
            continue
        if all(p._check_conflict(q) for q in list(context.passes) + kept):
            kept.append(p)
    names = {p.name for p in kept}
    out, placed = [], set()
    pending = list(kept)
    while pending:
        for i, p in enumerate(pending):  # first pass (in the given order) whose predecessors are placed
            if all(a not in names or a in placed for a in p._after):
                out.append(p)
                placed.add(p.name)
                pending.pop(i)
                break
        else:
            raise ValueError(f"cyclic pass ordering among {[p.name for p in pending]}")
    return out


class PassManager:
    def __init__(self, passes, context=None, auto_solve_conflict=True):
        self._context = PassContext() if context is None else context
        self._passes = _order(passes, self._context) if auto_solve_conflict else list(passes)

    def apply(self, main_programs, startup_programs):
        for p in self._passes:
            self._context = p.apply(main_programs, startup_programs, self._context)
        return self._context

    @property
    def context(self):
        return self._context

    @property
    def names(self):
        return [p.name for p in self._passes]

    @property
    def passes(self):
        return tuple(self._passes)
