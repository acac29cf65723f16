"""Bytecode-level translation of a Python function into a replayable static program (reference:
python/paddle/jit/sot/opcode_translator/executor/opcode_executor.py — an interpreter of CPython bytecode that
simulates each frame, builds the graph from the tensor operations it meets and breaks the graph where Python
needs something the graph cannot hold).

How this one works. ``translate(fn, args, kwargs)`` interprets ``fn``'s CPython 3.10 bytecode instruction by
instruction inside a dual trace (static/program.py: every tensor op is recorded as a Program node over meta
tensors AND executed on the real inputs as shadow values). The interpreter itself is what the plain trace
cannot be:

* every value read from outside the frame (arguments, module globals, closure cells, attributes / items of
  those) carries a Source; what the trace specialised on becomes a Guard (guards.py) checked at call time —
  a changed flag, layer attribute or global re-translates instead of replaying a stale program;
* mutations of objects that live outside the call (STORE_ATTR / STORE_SUBSCR / STORE_GLOBAL, list / dict /
  set mutator methods on sourced containers) are recorded as "py" nodes and replayed on every call, in
  program order, with the replayed tensors;
* calls that cannot live in a graph (print, logging, user functions marked ``not_to_static`` /
  ``graph_break``) are graph breaks: a "py" node that runs the real callable on the real values at that
  point of the replay; tensors it returns become new program values, Python values it returns are guarded;
* grad-mode context managers (``with paddle.no_grad():``) are replayed as grad-mode switches;
* user functions, bound methods and ``Layer.__call__`` of user layers are inlined frame by frame (the
  bytecode of ``forward``), so all of the above holds inside sub-layers too; library code (this framework,
  torch, numpy, builtins) runs natively under the trace.

Anything the interpreter does not model (generators, class bodies, pattern matching, an exception raised
inside the translated code) raises ``Unsupported`` and the caller falls back (StaticFunction's trace path
or eager), the way SOT falls back to dygraph.
"""
from __future__ import annotations

import builtins
import dis
import functools
import inspect
import logging
import operator
import types

import torch

from ...framework.tensor import Tensor, _wrap
from ...static import program as P
from .guards import GuardSet, Source, is_plain

__all__ = ["Unsupported", "translate", "graph_break"]

MAX_DEPTH = 24
_LIB_PREFIXES = ("paddlepaddle_amd", "torch", "numpy", "builtins", "functools", "operator", "collections",
                 "typing", "itertools", "math", "einops", "inspect", "abc", "enum", "copy", "contextlib",
                 "warnings", "logging", "re", "json", "os", "sys", "types", "weakref", "threading",
                 "dataclasses", "scipy", "_pytest", "pytest")
_MUTATORS = {list: {"append", "extend", "insert", "pop", "remove", "clear", "sort", "reverse", "__setitem__",
                    "__delitem__", "__iadd__"},
             dict: {"update", "pop", "popitem", "clear", "setdefault", "__setitem__", "__delitem__"},
             set: {"add", "discard", "remove", "pop", "clear", "update", "difference_update",
                   "intersection_update", "symmetric_difference_update"}}
_GEN_FLAGS = inspect.CO_GENERATOR | inspect.CO_COROUTINE | inspect.CO_ASYNC_GENERATOR | inspect.CO_ITERABLE_COROUTINE


class Unsupported(Exception):
    """The translator does not model this construct; the caller falls back."""


def graph_break(fn):
    """Mark ``fn`` as a graph break: inside a translated function it is called on real values at replay."""
    fn._sot_break = True
    return fn


_BREAK_FUNCS = {builtins.print, builtins.input}
_LOG_METHODS = {"debug", "info", "warning", "warn", "error", "critical", "exception", "log"}


def _is_break(f):
    if f in _BREAK_FUNCS or getattr(f, "_sot_break", False) or getattr(f, "_not_to_static", False):
        return True
    if isinstance(f, types.MethodType) and isinstance(f.__self__, logging.Logger) and f.__name__ in _LOG_METHODS:
        return True
    return getattr(f, "__module__", None) == "logging" and getattr(f, "__name__", "") in _LOG_METHODS


def _is_user_function(f):
    if not isinstance(f, types.FunctionType):
        return False
    mod = f.__module__ or ""
    if any(mod == p or mod.startswith(p + ".") for p in _LIB_PREFIXES):
        return False
    return supported(f.__code__)


class V:
    """A value on the simulated stack: the Python object, where it came from (Source or None) and, for a bound
    method produced by LOAD_METHOD, the receiver's V."""
    __slots__ = ("v", "src", "recv", "slot")

    def __init__(self, v, src=None, recv=None, slot=None):
        self.v, self.src, self.recv, self.slot = v, src, recv, slot  # slot: a runtime value (see Translator.rt)

    def __repr__(self):
        return f"V({type(self.v).__name__}, {self.src!r})"


_NULL = object()


class _PyCall:
    """Replay of a Python-level call recorded by the translator: torch tensors in the arguments are wrapped as
    framework Tensors, the callable runs, tensor leaves of the result are returned (in trace order) for the
    program's value slots and the Python leaves are compared with the traced ones (GuardFailure otherwise)."""

    def __init__(self, fn, label, expected=None, idempotent=True, first=None, mode="lift"):
        self.fn, self.label, self.expected = fn, label, expected
        self.idempotent = idempotent  # re-applied on the first replay too (setattr / setitem / grad mode)
        self.first = first            # trace-time result of a non-idempotent call, reused on the first replay
        self.mode = mode              # "lift": tensor leaves out, "rt": the whole Python value out
        self.__name__ = label

    def __call__(self, *args, **kwargs):
        a = [_wrap_tree(x) for x in args]
        k = {n: _wrap_tree(x) for n, x in kwargs.items()}
        out = self.fn(*a, **k)
        if self.mode == "rt":
            return out
        if self.expected is None:
            return None
        tensors, py = [], []
        _split_leaves(out, tensors, py)
        if py != self.expected:
            raise P.GuardFailure(f"graph break {self.label} returned {py!r}, traced {self.expected!r}")
        return tuple(t._t if isinstance(t, Tensor) else t for t in tensors)

    def __repr__(self):
        return f"<py {self.label}>"


def _wrap_tree(x):
    if isinstance(x, torch.Tensor):
        return _wrap(x)
    if isinstance(x, list):
        return [_wrap_tree(v) for v in x]
    if isinstance(x, tuple):
        return tuple(_wrap_tree(v) for v in x)
    if isinstance(x, dict):
        return {k: _wrap_tree(v) for k, v in x.items()}
    return x


def _split_leaves(x, tensors, py):
    if isinstance(x, (Tensor, torch.Tensor)):
        tensors.append(x)
    elif isinstance(x, (list, tuple)):
        for v in x:
            _split_leaves(v, tensors, py)
    elif isinstance(x, dict):
        for k in sorted(x, key=repr):
            py.append(k)
            _split_leaves(x[k], tensors, py)
    else:
        py.append(x if is_plain(x) else type(x).__name__)


def _has_tensor(x):
    if isinstance(x, (Tensor, torch.Tensor)):
        return True
    if isinstance(x, (list, tuple)):
        return any(_has_tensor(v) for v in x)
    if isinstance(x, dict):
        return any(_has_tensor(v) for v in x.values())
    return False


def _ident(x):
    return x


def _mk_tuple(*a):
    return a


def _mk_list(*a):
    return list(a)


def _mk_set(*a):
    return set(a)


def _mk_slice(*a):
    return slice(*a)


def _mk_str(*a):
    return "".join(a)


def _format(v, spec, conv):
    if conv == 1:
        v = str(v)
    elif conv == 2:
        v = repr(v)
    elif conv == 3:
        v = ascii(v)
    return format(v, spec)


_DATA_METHODS = {"numpy", "item", "tolist", "__array__", "__float__", "__int__", "__index__", "__bool__"}
_CONVERSIONS = {float, int, bool, complex}


def _set_grad(mode):
    torch.set_grad_enabled(mode)


class Translator:
    """State shared by the frames of one translation: the program, guards and statistics."""

    def __init__(self, prog, fn):
        self.prog = prog
        self.fn = fn
        self.guards = GuardSet()
        self.overlay = {}      # (id(obj), attr) -> V written during this translation
        self.keep = []         # objects whose ids appear in overlay keys (no id reuse)
        self.breaks = 0
        self.effects = 0
        self.inlined = 0

    # -------------------------------------------------------------- values <-> program
    def is_traced(self, x):
        t = x._t if isinstance(x, Tensor) else x
        return isinstance(t, torch.Tensor) and self.prog._is_traced(t)

    def real(self, x):
        """The real (shadow) value behind a traced tensor; structures are mapped, other values kept."""
        if isinstance(x, Tensor) and self.is_traced(x):
            r = _wrap(self.prog._shadow[self.prog._slot_of[id(x._t)]])
            r.stop_gradient = x.stop_gradient
            return r
        if isinstance(x, torch.Tensor) and self.prog._is_traced(x):
            return self.prog._shadow[self.prog._slot_of[id(x)]]
        if isinstance(x, list):
            return [self.real(v) for v in x]
        if isinstance(x, tuple) and not hasattr(x, "_fields"):
            return tuple(self.real(v) for v in x)
        if isinstance(x, dict):
            return {k: self.real(v) for k, v in x.items()}
        return x

    def lift(self, out, tensors_out):
        """Real tensors returned by a graph break become fresh traced values (shadow = the real value)."""
        if isinstance(out, (Tensor, torch.Tensor)):
            t = out._t if isinstance(out, Tensor) else out
            with torch._C.DisableTorchFunction():
                m = torch.empty(t.shape, dtype=t.dtype, device="meta")
            s = self.prog._new_slot(m)
            self.prog._shadow[s] = t
            tensors_out.append(P._Ref(s))
            w = _wrap(m)
            if isinstance(out, Tensor):
                w.stop_gradient = out.stop_gradient
            return w
        if isinstance(out, list):
            return [self.lift(v, tensors_out) for v in out]
        if isinstance(out, tuple) and not hasattr(out, "_fields"):
            return tuple(self.lift(v, tensors_out) for v in out)
        if isinstance(out, dict):
            return {k: self.lift(out[k], tensors_out) for k in sorted(out, key=repr)} if out else out
        return out

    def record_py(self, fn, args, kwargs, label, result=None, has_result=False, idempotent=True):
        """Append a "py" node calling ``fn`` at replay (``args`` are templated: traced tensors become value
        references; bind receivers into ``fn``). The call already ran during the translation, so a
        non-idempotent one is skipped on the first replay (its tensor results are reused). Returns the traced
        result (tensor leaves lifted to program values)."""
        prog = self.prog
        targs = [self.tmpl(a) for a in args]
        tkw = {k: self.tmpl(v) for k, v in kwargs.items()}
        outs = None
        expected = None
        lifted = None
        first = None
        if has_result and not _has_tensor(result):
            # a Python value computed at replay: later operations on it are replayed too (runtime value)
            s = self.rt_slot()
            node = P.OpNode(_PyCall(fn, label, None, idempotent, result, "rt"), tuple(targs), tkw,
                            P._Ref(s), "py", "py:" + label)
            self._append(node)
            return V(result, slot=s)
        if has_result:
            tensors_out = []
            lifted = self.lift(result, tensors_out)
            tensors, py = [], []
            _split_leaves(result, tensors, py)
            expected = py
            outs = tuple(tensors_out)
            first = tuple(t._t if isinstance(t, Tensor) else t for t in tensors)
        node = P.OpNode(_PyCall(fn, label, expected, idempotent, first), tuple(targs), tkw, outs, "py",
                        "py:" + label)
        self._append(node)
        return V(lifted) if has_result else None

    def _append(self, node):
        self.prog._cur.append(node)
        self.prog._version += 1
        self.prog._plans.clear()

    def rt_slot(self):
        with torch._C.DisableTorchFunction():
            return self.prog._new_slot(torch.empty(0, device="meta"))

    def tmpl(self, a):
        """Program template of a call argument: runtime values and traced tensors become value references."""
        if isinstance(a, V):
            if a.slot is not None:
                return P._Ref(a.slot)
            a = a.v
        return self.prog._template(a)

    def rt_call(self, fn, args, kwargs, label, idempotent=True):
        """``fn`` on runtime values: executed now on the real values (the translation goes on with the result)
        and recorded to run at replay; a tensor result is lifted into the program, any other value stays a
        runtime value."""
        res = fn(*[self.real_v(a) for a in args], **{k: self.real_v(v) for k, v in kwargs.items()})
        return self.record_py(fn, args, kwargs, label, res, has_result=True, idempotent=idempotent)

    def real_v(self, a):
        return a.v if a.slot is not None else self.real(a.v)

    def guard_rt(self, a, fn, expected):
        """Specialise on a runtime value (a branch on it, a loop over it): checked at replay."""
        self._append(P.GuardNode(fn, (P._Ref(a.slot),), {}, expected, "rt_guard"))

    def guard_value(self, src, v):
        self.guards.add_for_value(src, v)


class Frame:
    def __init__(self, tr, fn, code, local_vals, depth, cells=None):
        self.tr, self.fn, self.code, self.depth = tr, fn, code, depth
        self.globals = fn.__globals__
        self.locals = dict(local_vals)   # name -> V
        self.stack = []
        self.blocks = []
        self.with_exits = []
        n_cell = len(code.co_cellvars)
        self.cells = list(cells) if cells is not None else []
        if cells is None:
            for name in code.co_cellvars:
                c = types.CellType()
                if name in self.locals:  # an argument captured by a closure lives in its cell
                    c.cell_contents = self.locals[name].v
                self.cells.append(c)
            for i, c in enumerate(fn.__closure__ or ()):
                self.cells.append(c)
        self.n_cell = n_cell
        self.instrs = list(dis.get_instructions(code))
        self.index = {ins.offset: i for i, ins in enumerate(self.instrs)}

    # ------------------------------------------------------------------ stack helpers
    def push(self, v):
        self.stack.append(v if isinstance(v, V) else V(v))

    def pop(self):
        return self.stack.pop()

    def popn(self, n):
        if n == 0:
            return []
        out = self.stack[-n:]
        del self.stack[-n:]
        return out

    # ------------------------------------------------------------------ run
    def run(self):
        pc = 0
        instrs = self.instrs
        while True:
            ins = instrs[pc]
            op = ins.opname
            h = getattr(self, "op_" + op, None)
            if h is None:
                raise Unsupported(f"opcode {op} ({self.code.co_name}:{ins.starts_line})")
            r = h(ins)
            if r is None:
                pc += 1
            elif isinstance(r, tuple) and r[0] == "jump":
                pc = self.index[r[1]]
            else:  # ("return", V)
                return r[1]

    # ------------------------------------------------------------------ loads / stores
    def op_NOP(self, ins):
        return None

    def op_EXTENDED_ARG(self, ins):
        return None

    def op_LOAD_CONST(self, ins):
        self.push(V(ins.argval))

    def op_LOAD_FAST(self, ins):
        if ins.argval not in self.locals:
            raise UnboundLocalError(f"local variable '{ins.argval}' referenced before assignment")
        self.push(self.locals[ins.argval])

    def op_STORE_FAST(self, ins):
        self.locals[ins.argval] = self.pop()

    def op_DELETE_FAST(self, ins):
        self.locals.pop(ins.argval, None)

    def op_LOAD_GLOBAL(self, ins):
        name = ins.argval
        g = self.globals
        if name in g:
            v = g[name]
        else:
            b = g.get("__builtins__", builtins)
            try:
                v = b[name] if isinstance(b, dict) else getattr(b, name)
            except (KeyError, AttributeError):
                raise NameError(f"name '{name}' is not defined") from None
        src = Source("global", (g, name))
        self.tr.guard_value(src, v)
        self.push(V(v, src))

    def op_STORE_GLOBAL(self, ins):
        val = self.pop()
        self.tr.record_py(functools.partial(operator.setitem, self.globals, ins.argval), [val], {},
                          f"global {ins.argval}")
        self.tr.effects += 1
        self.globals[ins.argval] = self.tr.real_v(val)

    def op_LOAD_DEREF(self, ins):
        c = self.cells[ins.arg]
        try:
            v = c.cell_contents
        except ValueError:
            raise NameError(f"free variable '{ins.argval}' referenced before assignment") from None
        src = None
        if ins.arg >= self.n_cell and self.depth == 0:  # a closure cell of the translated function
            src = Source("cell", c)
            self.tr.guard_value(src, v)
        self.push(V(v, src))

    def op_STORE_DEREF(self, ins):
        self.cells[ins.arg].cell_contents = self.pop().v

    def op_LOAD_CLOSURE(self, ins):
        self.push(V(self.cells[ins.arg]))

    def op_LOAD_ATTR(self, ins):
        obj = self.pop()
        self.push(self._getattr(obj, ins.argval))

    def _getattr(self, obj, name):
        if obj.slot is not None:
            return self.tr.rt_call(getattr, [obj, V(name)], {}, "getattr")
        obj = _anchor(obj)
        o = obj.v
        ov = self.tr.overlay.get((id(o), name))
        if ov is not None:
            return ov
        val = getattr(o, name)
        src = None
        if obj.src is not None and not isinstance(o, (Tensor, torch.Tensor)):
            if isinstance(val, (types.MethodType, types.BuiltinMethodType, types.MethodWrapperType)):
                src = None
                if isinstance(val, types.MethodType):
                    self.tr.guard_value(obj.src.attr(name).attr("__func__"), val.__func__)
            elif isinstance(getattr(type(o), name, None), property):
                if is_plain(val):
                    src = obj.src.attr(name)
                    self.tr.guard_value(src, val)
            else:
                src = obj.src.attr(name)
                self.tr.guard_value(src, val)
        return V(val, src)

    def op_STORE_ATTR(self, ins):
        obj = _anchor(self.pop())
        val = self.pop()
        if obj.src is not None:  # an object that outlives the call: replay the write
            self.tr.record_py(functools.partial(setattr, obj.v, ins.argval), [val], {}, f"setattr {ins.argval}")
            self.tr.effects += 1
            self.tr.overlay[(id(obj.v), ins.argval)] = val
            self.tr.keep.append(obj.v)
            setattr(obj.v, ins.argval, self.tr.real_v(val))
        else:
            setattr(obj.v, ins.argval, val.v)

    def op_DELETE_ATTR(self, ins):
        obj = self.pop()
        if obj.src is not None:
            self.tr.record_py(functools.partial(delattr, obj.v, ins.argval), [], {}, f"delattr {ins.argval}",
                              idempotent=False)
            self.tr.effects += 1
        delattr(obj.v, ins.argval)

    def op_LOAD_METHOD(self, ins):
        obj = self.pop()
        m = self._getattr(obj, ins.argval)
        self.push(V(_NULL))
        self.push(V(m.v, m.src, obj))

    def op_BINARY_SUBSCR(self, ins):
        k = self.pop()
        c = self.pop()
        if c.slot is not None or k.slot is not None:
            self.push(self.tr.rt_call(operator.getitem, [c, k], {}, "getitem"))
            return
        val = c.v[k.v]
        src = None
        if c.src is not None and is_plain(k.v) and not isinstance(c.v, (Tensor, torch.Tensor)):
            src = c.src.item(k.v)
            self.tr.guard_value(src, val)
        self.push(V(val, src))

    def op_STORE_SUBSCR(self, ins):
        k = self.pop()
        c = self.pop()
        val = self.pop()
        if c.src is not None and not isinstance(c.v, (Tensor, torch.Tensor)):
            self.tr.record_py(functools.partial(operator.setitem, c.v), [k, val], {}, "setitem")
            self.tr.effects += 1
            c.v[k.v] = self.tr.real_v(val)
        else:
            c.v[k.v] = val.v

    def op_DELETE_SUBSCR(self, ins):
        k = self.pop()
        c = self.pop()
        if c.src is not None:
            self.tr.record_py(functools.partial(operator.delitem, c.v), [k], {}, "delitem", idempotent=False)
            self.tr.effects += 1
        del c.v[k.v]

    # ------------------------------------------------------------------ stack shuffles
    def op_POP_TOP(self, ins):
        self.pop()

    def op_ROT_TWO(self, ins):
        s = self.stack
        s[-1], s[-2] = s[-2], s[-1]

    def op_ROT_THREE(self, ins):
        s = self.stack
        s[-1], s[-2], s[-3] = s[-2], s[-3], s[-1]

    def op_ROT_FOUR(self, ins):
        s = self.stack
        s[-1], s[-2], s[-3], s[-4] = s[-2], s[-3], s[-4], s[-1]

    def op_ROT_N(self, ins):
        s = self.stack
        top = s.pop()
        s.insert(len(s) - ins.arg + 1, top)

    def op_DUP_TOP(self, ins):
        self.stack.append(self.stack[-1])

    def op_DUP_TOP_TWO(self, ins):
        self.stack.extend(self.stack[-2:])

    # ------------------------------------------------------------------ operators
    _BIN = {"BINARY_ADD": operator.add, "BINARY_SUBTRACT": operator.sub, "BINARY_MULTIPLY": operator.mul,
            "BINARY_TRUE_DIVIDE": operator.truediv, "BINARY_FLOOR_DIVIDE": operator.floordiv,
            "BINARY_MODULO": operator.mod, "BINARY_POWER": operator.pow, "BINARY_MATRIX_MULTIPLY": operator.matmul,
            "BINARY_LSHIFT": operator.lshift, "BINARY_RSHIFT": operator.rshift, "BINARY_AND": operator.and_,
            "BINARY_OR": operator.or_, "BINARY_XOR": operator.xor,
            "INPLACE_ADD": operator.iadd, "INPLACE_SUBTRACT": operator.isub, "INPLACE_MULTIPLY": operator.imul,
            "INPLACE_TRUE_DIVIDE": operator.itruediv, "INPLACE_FLOOR_DIVIDE": operator.ifloordiv,
            "INPLACE_MODULO": operator.imod, "INPLACE_POWER": operator.ipow,
            "INPLACE_MATRIX_MULTIPLY": operator.imatmul, "INPLACE_LSHIFT": operator.ilshift,
            "INPLACE_RSHIFT": operator.irshift, "INPLACE_AND": operator.iand, "INPLACE_OR": operator.ior,
            "INPLACE_XOR": operator.ixor}

    def _binary(self, ins):
        b = self.pop()
        a = self.pop()
        f = self._BIN[ins.opname]
        if ins.opname.startswith("INPLACE") and a.src is not None and isinstance(a.v, (list, dict, set)):
            # `self.items += [...]` mutates a container that outlives the call
            self.tr.record_py(functools.partial(f, a.v), [b], {}, ins.opname.lower(), idempotent=False)
            self.tr.effects += 1
            f(a.v, self.tr.real_v(b))
            self.push(a)
            return
        if a.slot is not None or b.slot is not None:
            self.push(self.tr.rt_call(f, [a, b], {}, ins.opname.lower()))
            return
        self.push(V(f(a.v, b.v)))

    _UN = {"UNARY_NEGATIVE": operator.neg, "UNARY_POSITIVE": operator.pos, "UNARY_INVERT": operator.invert,
           "UNARY_NOT": operator.not_}

    def _unary(self, ins):
        a = self.pop()
        f = self._UN[ins.opname]
        self.push(self.tr.rt_call(f, [a], {}, ins.opname.lower()) if a.slot is not None else V(f(a.v)))

    _CMP = {"<": operator.lt, "<=": operator.le, "==": operator.eq, "!=": operator.ne, ">": operator.gt,
            ">=": operator.ge}

    def _rt2(self, f, a, b, label):
        if a.slot is not None or b.slot is not None:
            return self.tr.rt_call(f, [a, b], {}, label)
        return V(f(a.v, b.v))

    def op_COMPARE_OP(self, ins):
        b = self.pop()
        a = self.pop()
        self.push(self._rt2(self._CMP[ins.argval], a, b, "cmp" + ins.argval))

    def op_IS_OP(self, ins):
        b = self.pop()
        a = self.pop()
        self.push(self._rt2(operator.is_not if ins.arg else operator.is_, a, b, "is"))

    def op_CONTAINS_OP(self, ins):
        b = self.pop()
        a = self.pop()
        f = (lambda x, y: x not in y) if ins.arg else (lambda x, y: x in y)
        self.push(self._rt2(f, a, b, "in"))

    # ------------------------------------------------------------------ control flow
    def _truth(self, v):
        if v.slot is not None:  # a runtime value: the branch is specialised and checked at replay
            r = bool(v.v)
            self.tr.guard_rt(v, bool, r)
            return r
        return bool(v.v)  # a traced tensor: a guard (dual trace) fixes the branch to the real value

    def op_POP_JUMP_IF_FALSE(self, ins):
        if not self._truth(self.pop()):
            return ("jump", ins.argval)

    def op_POP_JUMP_IF_TRUE(self, ins):
        if self._truth(self.pop()):
            return ("jump", ins.argval)

    def op_JUMP_IF_FALSE_OR_POP(self, ins):
        if not self._truth(self.stack[-1]):
            return ("jump", ins.argval)
        self.pop()

    def op_JUMP_IF_TRUE_OR_POP(self, ins):
        if self._truth(self.stack[-1]):
            return ("jump", ins.argval)
        self.pop()

    def op_JUMP_FORWARD(self, ins):
        return ("jump", ins.argval)

    def op_JUMP_ABSOLUTE(self, ins):
        return ("jump", ins.argval)

    def op_GET_ITER(self, ins):
        it = self.pop()
        o = it.v
        if it.slot is not None:  # iterating a runtime value: specialised on it (checked at replay)
            self.tr.guard_rt(it, _ident, o)
        if it.src is not None and isinstance(o, (list, tuple)):
            self.tr.guards.add(it.src, "len", len(o))
            items = [V(x, it.src.item(i)) for i, x in enumerate(o)]
            for v in items:
                self.tr.guard_value(v.src, v.v)
            self.push(V(iter(items), None, "src_iter"))
            return
        if it.src is not None and isinstance(o, dict):
            keys = list(o)
            self.tr.guards.add(it.src, "len", len(keys))
            self.push(V(iter([V(k) for k in keys]), None, "src_iter"))
            return
        if it.src is not None and hasattr(o, "__len__") and hasattr(o, "__getitem__") and \
                not isinstance(o, (Tensor, torch.Tensor, str, bytes, range)):
            n = len(o)
            self.tr.guards.add(it.src, "len", n)
            items = [V(x, it.src.item(i)) for i, x in enumerate(list(o))]
            for v in items:
                self.tr.guard_value(v.src, v.v)
            self.push(V(iter(items), None, "src_iter"))
            return
        self.push(V(iter(o)))

    def op_GET_YIELD_FROM_ITER(self, ins):
        raise Unsupported("yield from")

    def op_FOR_ITER(self, ins):
        top = self.stack[-1]
        try:
            nxt = next(top.v)
        except StopIteration:
            self.pop()
            return ("jump", ins.argval)
        self.push(nxt if top.recv == "src_iter" else V(nxt))

    def op_RETURN_VALUE(self, ins):
        return ("return", self.pop())

    # try / with: the handlers only run on an exception, which aborts the translation
    def op_SETUP_FINALLY(self, ins):
        self.blocks.append("finally")

    def op_POP_BLOCK(self, ins):
        self.blocks.pop()

    def op_SETUP_WITH(self, ins):
        ctx = self.pop()
        mgr = ctx.v
        exit_fn = type(mgr).__exit__
        before = torch.is_grad_enabled()
        res = type(mgr).__enter__(mgr)
        after = torch.is_grad_enabled()
        if after != before:  # grad-mode switch (no_grad / enable_grad / set_grad_enabled): replayed
            self.tr.record_py(_set_grad, [after], {}, "set_grad_enabled")
        self.blocks.append("with")

        def _exit(*a, _m=mgr, _f=exit_fn):
            b = torch.is_grad_enabled()
            r = _f(_m, *a)
            if torch.is_grad_enabled() != b:
                self.tr.record_py(_set_grad, [torch.is_grad_enabled()], {}, "set_grad_enabled")
            return r
        self.push(V(_exit))
        self.push(V(res))

    # exception-handler code: only reached after an exception, which already ends the translation
    def _handler_only(self, ins):
        raise Unsupported(f"exception handler opcode {ins.opname}")

    op_WITH_EXCEPT_START = op_RERAISE = op_POP_EXCEPT = op_JUMP_IF_NOT_EXC_MATCH = _handler_only

    def op_RAISE_VARARGS(self, ins):
        args = self.popn(ins.arg)
        if not args:
            raise Unsupported("bare raise")
        exc = args[0].v
        raise exc

    def op_LOAD_ASSERTION_ERROR(self, ins):
        self.push(V(AssertionError))

    # ------------------------------------------------------------------ builders
    def _build(self, items, mk, label):
        if any(v.slot is not None for v in items):
            return self.tr.rt_call(mk, items, {}, label)
        return V(mk(*[v.v for v in items]))

    def op_BUILD_TUPLE(self, ins):
        self.push(self._build(self.popn(ins.arg), _mk_tuple, "tuple"))

    def op_BUILD_LIST(self, ins):
        self.push(self._build(self.popn(ins.arg), _mk_list, "list"))

    def op_BUILD_SET(self, ins):
        self.push(self._build(self.popn(ins.arg), _mk_set, "set"))

    def op_BUILD_MAP(self, ins):
        items = self.popn(2 * ins.arg)
        self.push(V({items[i].v: items[i + 1].v for i in range(0, len(items), 2)}))

    def op_BUILD_CONST_KEY_MAP(self, ins):
        keys = self.pop().v
        vals = self.popn(ins.arg)
        self.push(V(dict(zip(keys, (v.v for v in vals)))))

    def op_BUILD_STRING(self, ins):
        self.push(self._build(self.popn(ins.arg), _mk_str, "str"))

    def op_BUILD_SLICE(self, ins):
        self.push(self._build(self.popn(ins.arg), _mk_slice, "slice"))

    def op_LIST_APPEND(self, ins):
        v = self.pop()
        self.stack[-ins.arg].v.append(v.v)

    def op_SET_ADD(self, ins):
        v = self.pop()
        self.stack[-ins.arg].v.add(v.v)

    def op_MAP_ADD(self, ins):
        v = self.pop()
        k = self.pop()
        self.stack[-ins.arg].v[k.v] = v.v

    def op_LIST_EXTEND(self, ins):
        v = self.pop()
        self.stack[-ins.arg].v.extend(v.v)

    def op_SET_UPDATE(self, ins):
        v = self.pop()
        self.stack[-ins.arg].v.update(v.v)

    def op_DICT_UPDATE(self, ins):
        v = self.pop()
        self.stack[-ins.arg].v.update(v.v)

    def op_DICT_MERGE(self, ins):
        v = self.pop()
        d = self.stack[-ins.arg].v
        for k in v.v:
            if k in d:
                raise TypeError(f"got multiple values for keyword argument '{k}'")
        d.update(v.v)

    def op_LIST_TO_TUPLE(self, ins):
        self.push(V(tuple(self.pop().v)))

    def op_UNPACK_SEQUENCE(self, ins):
        seq = self.pop()
        vals = list(seq.v)
        if len(vals) != ins.arg:
            raise ValueError(f"expected {ins.arg} values to unpack, got {len(vals)}")
        srcs = [seq.src.item(i) if seq.src is not None and isinstance(seq.v, (list, tuple)) else None
                for i in range(len(vals))]
        for v, s in reversed(list(zip(vals, srcs))):
            self.push(V(v, s))

    def op_UNPACK_EX(self, ins):
        vals = list(self.pop().v)
        before, after = ins.arg & 0xFF, ins.arg >> 8
        if len(vals) < before + after:
            raise ValueError("not enough values to unpack")
        mid = vals[before:len(vals) - after]
        out = vals[:before] + [mid] + vals[len(vals) - after:]
        for v in reversed(out):
            self.push(V(v))

    def op_FORMAT_VALUE(self, ins):
        spec = self.pop() if (ins.arg & 0x04) else V("")
        v = self.pop()
        conv = ins.arg & 0x03
        if v.slot is not None or spec.slot is not None or self.tr.is_traced(v.v):
            # formatting a runtime value or a tensor reads data: done at replay (a graph break)
            self.push(self.tr.rt_call(_format, [v, spec, V(conv)], {}, "format", idempotent=True))
            return
        self.push(V(_format(v.v, spec.v, conv)))

    def op_GET_LEN(self, ins):
        self.push(V(len(self.stack[-1].v)))

    def op_IMPORT_NAME(self, ins):
        fromlist = self.pop().v
        level = self.pop().v
        self.push(V(__import__(ins.argval, self.globals, None, fromlist, level)))

    def op_IMPORT_FROM(self, ins):
        self.push(V(getattr(self.stack[-1].v, ins.argval)))

    def op_MAKE_FUNCTION(self, ins):
        qualname = self.pop().v
        code = self.pop().v
        closure = self.pop().v if ins.arg & 0x08 else None
        if ins.arg & 0x04:
            self.pop()
        kwdefaults = self.pop().v if ins.arg & 0x02 else None
        defaults = self.pop().v if ins.arg & 0x01 else None
        f = types.FunctionType(code, self.globals, code.co_name, defaults, closure)
        f.__qualname__ = qualname
        if kwdefaults:
            f.__kwdefaults__ = kwdefaults
        self.push(V(f))

    # ------------------------------------------------------------------ calls
    def op_CALL_FUNCTION(self, ins):
        args = self.popn(ins.arg)
        f = self.pop()
        self.push(self.call(f, args, {}))

    def op_CALL_FUNCTION_KW(self, ins):
        names = self.pop().v
        vals = self.popn(ins.arg)
        f = self.pop()
        n = len(names)
        pos, kw = vals[:len(vals) - n], dict(zip(names, vals[len(vals) - n:]))
        self.push(self.call(f, pos, kw))

    def op_CALL_FUNCTION_EX(self, ins):
        kw = self.pop() if ins.arg & 1 else V({})
        args = self.pop()
        f = self.pop()
        if args.slot is not None or kw.slot is not None:
            self.push(self.tr.rt_call(lambda fn, a, k: fn(*a, **k), [f, args, kw], {}, "call_ex"))
            return
        self.push(self.call(f, [V(a) for a in args.v], {k: V(v) for k, v in kw.v.items()}))

    def op_CALL_METHOD(self, ins):
        args = self.popn(ins.arg)
        m = self.pop()
        self.pop()  # the NULL slot of LOAD_METHOD
        self.push(self.call(m, args, {}))

    def call(self, fv, args, kwargs):
        f = fv.v
        tr = self.tr
        if fv.slot is not None:  # calling a runtime value (e.g. a method looked up on one)
            return tr.rt_call(lambda fn, *a, **k: fn(*a, **k), [fv] + list(args), kwargs, "call")
        if f is builtins.super and not args:
            return self._zero_arg_super()
        if _is_break(f):
            tr.breaks += 1
            res = f(*[tr.real_v(a) for a in args], **{k: tr.real_v(v) for k, v in kwargs.items()})
            r = tr.record_py(f, args, kwargs, getattr(f, "__name__", "call"), res, has_result=res is not None,
                             idempotent=False)
            return r if r is not None else V(None)
        recv = fv.recv
        if recv is not None and recv.src is not None and isinstance(f, (types.BuiltinMethodType,)):
            muts = next((m for t, m in _MUTATORS.items() if isinstance(recv.v, t)), None)
            if muts is not None and f.__name__ in muts:
                # mutation of a container that outlives the call: replayed on every call
                tr.record_py(functools.partial(getattr(type(recv.v), f.__name__), recv.v), args, kwargs,
                             f"{type(recv.v).__name__}.{f.__name__}", idempotent=False)
                tr.effects += 1
                return V(f(*[tr.real_v(a) for a in args], **{k: tr.real_v(v) for k, v in kwargs.items()}))
        # reading a traced tensor's data (t.numpy(), t.item(), float(t) ...): a graph break whose Python result
        # is a runtime value, so the code after it replays on the new data instead of specialising on it
        if recv is not None and tr.is_traced(recv.v) and getattr(f, "__name__", "") in _DATA_METHODS:
            tr.breaks += 1
            name = f.__name__
            return tr.rt_call(lambda t, *a, **k: getattr(t, name)(*a, **k), [recv] + list(args), kwargs,
                              "tensor." + name)
        if f in _CONVERSIONS and len(args) == 1 and tr.is_traced(args[0].v):
            tr.breaks += 1
            return tr.rt_call(f, args, {}, f.__name__)
        if any(a.slot is not None for a in args) or any(v.slot is not None for v in kwargs.values()):
            # a library call on runtime values runs at replay (its tensor results are lifted into the program)
            target = self._inline_target(fv)
            if target is None:
                return tr.rt_call(f, args, kwargs, getattr(f, "__name__", "call"))
        target = self._inline_target(fv)
        if target is not None and self.depth < MAX_DEPTH:
            func, self_v = target
            call_args = ([self_v] if self_v is not None else []) + list(args)
            return self._inline(func, call_args, kwargs)
        return V(f(*[a.v for a in args], **{k: v.v for k, v in kwargs.items()}))

    def _inline_target(self, fv):
        f = fv.v
        from ...nn.layer.layers import Layer
        if isinstance(f, Layer):
            fwd = type(f).forward
            if "forward" in f.__dict__ or not _is_user_function(fwd) or _has_hooks(f):
                return None
            return fwd, _anchor(V(f, fv.src))
        if isinstance(f, types.MethodType) and _is_user_function(f.__func__):
            self_src = fv.recv.src if fv.recv is not None else None
            return f.__func__, V(f.__self__, self_src)
        if _is_user_function(f):
            return f, None
        return None

    def _inline(self, func, args, kwargs):
        code = func.__code__
        sig = inspect.signature(func)
        try:
            bound = sig.bind(*args, **kwargs)
        except TypeError as e:
            raise Unsupported(f"argument binding: {e}") from None
        bound.apply_defaults()
        local_vals = {}
        for name, val in bound.arguments.items():
            p = sig.parameters[name]
            if p.kind == p.VAR_POSITIONAL:
                items = [v if isinstance(v, V) else V(v) for v in val]
                local_vals[name] = self._build(items, _mk_tuple, "tuple")
            elif p.kind == p.VAR_KEYWORD:
                if any(isinstance(v, V) and v.slot is not None for v in val.values()):
                    ks = list(val)
                    local_vals[name] = self.tr.rt_call(lambda *a, _k=tuple(ks): dict(zip(_k, a)),
                                                       [val[k] for k in ks], {}, "dict")
                else:
                    local_vals[name] = V({k: (v.v if isinstance(v, V) else v) for k, v in val.items()})
            else:
                local_vals[name] = val if isinstance(val, V) else V(val)
        for name in list(local_vals):  # inspect names a comprehension's ".0" argument "implicit0"
            if name.startswith("implicit") and "." + name[8:] in code.co_varnames:
                local_vals["." + name[8:]] = local_vals.pop(name)
        self.tr.inlined += 1
        return Frame(self.tr, func, code, local_vals, self.depth + 1).run()

    def _zero_arg_super(self):
        names = self.code.co_cellvars + self.code.co_freevars
        if "__class__" not in names or not self.code.co_varnames:
            raise Unsupported("zero-argument super() outside a method")
        cls = self.cells[names.index("__class__")].cell_contents
        first = self.locals.get(self.code.co_varnames[0])
        if first is None:
            raise Unsupported("super() without self")
        return V(super(cls, first.v), None, None)


for _n in Frame._BIN:
    setattr(Frame, "op_" + _n, Frame._binary)
for _n in Frame._UN:
    setattr(Frame, "op_" + _n, Frame._unary)


def _anchor(v):
    """A Layer reached without a source path (e.g. through enumerate / zip of a sub-layer list) is anchored as a
    constant source: guards on its attributes are re-read from that very object at call time, and writes to it
    are replayed side effects, like for layers reached from the arguments."""
    if v.src is None and v.slot is None:
        from ...nn.layer.layers import Layer
        if isinstance(v.v, Layer):
            return V(v.v, Source("const", v.v), v.recv)
    return v


def _has_hooks(layer):
    for a in ("_forward_pre_hooks", "_forward_post_hooks"):
        h = getattr(layer, a, None)
        if h:
            return True
    return False


_SUPPORTED = {}


def supported(code):
    r = _SUPPORTED.get(code)
    if r is None:
        r = not (code.co_flags & _GEN_FLAGS) and all(hasattr(Frame, "op_" + i.opname)
                                                      for i in dis.get_instructions(code))
        _SUPPORTED[code] = r
    return r


def translate(fn, args, kwargs, prog, arg_values):
    """Interpret ``fn`` on ``arg_values`` (name -> (value, Source or None)) inside ``prog``'s dual trace.
    Returns (output, Translator)."""
    if not supported(fn.__code__):
        raise Unsupported(f"{fn.__qualname__}: generator / unsupported opcode")
    tr = Translator(prog, fn)
    local_vals = {}
    for name, (val, src) in arg_values.items():
        local_vals[name] = V(val, src)
        if src is not None:
            tr.guard_value(src, val)
    frame = Frame(tr, fn, fn.__code__, local_vals, 0)
    with P.trace_into(prog):
        out = frame.run()
    return out, tr
