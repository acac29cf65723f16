"""Static graph: Program IR recorded from the same ops the dynamic graph runs, and its Executor.

Reference: python/paddle/base/framework.py:5893 (Program), base/executor.py:1247 (Executor.run),
base/backward.py (append_backward, gradients), paddle/fluid/framework/new_executor/
program_interpreter.cc:142,231 (dependency analysis + garbage collection of intermediates).

Design (MI355X-first, no tracing compiler):
  * Building a Program runs the user's model code once on *meta* tensors (shape/dtype only, no data).
    A TorchFunctionMode (``_Tracer``) records every device-buffer operation that touches a traced
    value as an ``OpNode`` (callable + argument template). Hand-written HIP ops (``ops.*``) are
    recorded as ONE node each (``static_op`` hook), so replay on the GPU runs the fused CDNA4 kernels,
    not their decompositions.
  * ``Executor.run`` replays the node list on real buffers. Ordering and buffer lifetimes come from
    the native C++ scheduler (``_C_runtime.schedule``: topological order + last-use per node), so
    every intermediate is dropped right after its last consumer — the interpreter-core GC.
  * Training programs (``optimizer.minimize``) replay with autograd on, then run backward and the
    (fused HIP) optimizer step; ``gradients``/``append_backward`` are recorded as autograd nodes.
  * Programs serialize to JSON (``to_dict``/``from_dict``) naming callables from the torch / ops
    namespaces only, so loading a saved model never executes code from the file.
"""
from __future__ import annotations

import contextlib
import itertools
import threading

import numpy as np
import torch
from torch.overrides import TorchFunctionMode

from ..framework import dtype as _dt
from ..framework.tensor import Tensor, Parameter, _wrap

SENTINEL = 2  # size used for unknown (-1 / None) dims while tracing
_META = torch.device("meta")
_PURE_GETTERS = frozenset({
    "shape", "dim", "size", "dtype", "device", "is_floating_point", "numel", "stride", "requires_grad",
    "is_contiguous", "ndim", "element_size", "data_ptr", "is_cuda", "layout", "is_complex", "storage_offset",
    "get_device", "__len__", "nelement", "is_leaf", "grad_fn", "names", "is_sparse", "is_quantized",
    "is_meta", "itemsize", "nbytes", "ndimension", "__hash__", "is_nested", "_version",
})


class _Ref:
    __slots__ = ("i",)

    def __init__(self, i):
        self.i = i

    def __repr__(self):
        return f"%{self.i}"


class _Const:
    __slots__ = ("t", "idx")

    def __init__(self, t, idx):
        self.t = t
        self.idx = idx

    def __repr__(self):
        return f"$c{self.idx}"


class _DevPlaceholder:
    """A torch.device('meta') seen while tracing == "the device the program runs on"."""
    __slots__ = ()

    def __repr__(self):
        return "<run_device>"


_RUN_DEV = _DevPlaceholder()


class _Sym:
    """Affine function a*N + b of the dynamic dimension N (used by saved programs)."""
    __slots__ = ("a", "b")

    def __init__(self, a, b):
        self.a, self.b = a, b


class OpNode:
    __slots__ = ("func", "args", "kwargs", "outs", "kind", "name", "rc")

    def __init__(self, func, args, kwargs, outs, kind="torch", name=None):
        self.func, self.args, self.kwargs, self.outs, self.kind = func, args, kwargs, outs, kind
        self.name = name or _func_name(func)
        self.rc = None  # recompute segment id (ops traced inside a recompute scope), None outside

    @property
    def type(self):
        return self.name

    def __repr__(self):
        return f"{self.outs} = {self.name}{self.args}"


class GuardFailure(RuntimeError):
    """A guard of a dual-traced program saw a different Python value than at trace time."""


class GuardNode(OpNode):
    """A Python conversion of a traced value (bool(t), t.item(), t.tolist(), ...) seen while dual-tracing:
    replay recomputes it and raises GuardFailure when it differs from the traced value, because the
    Python code after it (a branch, a loop trip count, a shape) was specialised to that value."""
    __slots__ = ("expected",)

    def __init__(self, func, args, kwargs, expected, name=None):
        super().__init__(func, args, kwargs, None, "guard", name)
        self.expected = expected

    def check(self, val):
        e = self.expected
        if isinstance(e, np.ndarray) or isinstance(val, np.ndarray):
            ok = isinstance(val, np.ndarray) and isinstance(e, np.ndarray) and val.shape == e.shape and \
                val.dtype == e.dtype and bool(np.array_equal(val, e, equal_nan=val.dtype.kind in "fc"))
        else:
            ok = type(val) is type(e) and (val == e or (val != val and e != e))
        if not ok:
            raise GuardFailure(f"guard {self.name} expected {e!r}, got {val!r}")

    def __repr__(self):
        return f"guard {self.name}{self.args} == {self.expected!r}"


# Python conversions of a tensor's data (graph breaks of the reference's SOT; guards here)
_BREAK_FUNCS = frozenset({"m:__bool__", "m:item", "m:tolist", "m:__int__", "m:__float__", "m:__index__",
                          "m:__complex__", "m:numpy", "m:__array__"})


def _func_name(func):
    q = getattr(func, "__qualname__", "") or ""
    if q == "getset_descriptor.__get__" or q.endswith(".__get__"):
        return "p:" + func.__self__.__name__
    n = getattr(func, "__name__", str(func))
    if q.startswith("TensorBase.") or q.startswith("Tensor.") or q.startswith("_TensorBase."):
        return "m:" + n
    mod = getattr(func, "__module__", None) or ""
    if mod.startswith("paddlepaddle_amd.ops") or mod.startswith("paddlepaddle_amd.static"):
        return "o:" + mod + ":" + n
    return "f:" + (mod or "torch") + ":" + n


def _resolve(name):
    """Inverse of _func_name restricted to torch / our ops namespaces (no arbitrary imports)."""
    kind, _, rest = name.partition(":")
    if kind == "m":
        return getattr(torch.Tensor, rest)
    if kind == "p":
        return getattr(torch.Tensor, rest).__get__
    mod, _, attr = rest.rpartition(":")
    if kind == "o":
        if not (mod.startswith("paddlepaddle_amd.ops") or mod.startswith("paddlepaddle_amd.static")):
            raise ValueError(f"refusing to resolve {name}")
        import importlib
        m = importlib.import_module(mod)
        return getattr(m, attr)
    if kind == "f":
        if mod != "torch" and not mod.startswith("torch."):
            raise ValueError(f"refusing to resolve {name}")
        obj = torch
        for part in mod.split(".")[1:]:
            obj = getattr(obj, part)
        return getattr(obj, attr)
    raise ValueError(f"bad op name {name}")


# ---------------------------------------------------------------------------------- Program
class Program:
    _ids = itertools.count()

    def __init__(self):
        self.nodes = []
        self._slot_of = {}       # id(meta tensor) -> slot
        self._metas = []         # slot -> meta tensor (kept alive so ids stay unique)
        self._consts = []        # captured real tensors (parameters, constants)
        self._const_of = {}      # id(real tensor) -> const idx
        self._params = {}        # const idx -> Parameter
        self.feeds = {}          # name -> (slot, declared shape, paddle dtype str)
        self._names = {}         # name -> slot
        self._optimize = None    # (optimizer, loss slot)
        self._need_grad_slots = set()
        self._version = 0
        self._plans = {}
        self.random_seed = 0
        self._id = next(Program._ids)
        self._is_test = False
        self._dyn = False        # saved program with an affine dynamic dim
        self._cur = self.nodes   # node list being recorded into (a control-flow sub-block while tracing one)
        # guarded (dual) tracing: real values of the slots, computed next to the meta trace so a Python
        # conversion of a traced value (bool / item / tolist ...) yields the actual value and is recorded as
        # a GuardNode instead of ending the trace (jit.to_static's graph-break path)
        self._shadow = None
        self._shadow_dev = None
        self._rc = None          # recompute segment id stamped on the nodes being recorded
        self._rc_ids = itertools.count(1)

    # ------------------------------------------------------------ slots / values
    def _new_slot(self, meta):
        s = len(self._metas)
        self._metas.append(meta)
        self._slot_of[id(meta)] = s
        return s

    def _is_traced(self, t):
        return isinstance(t, torch.Tensor) and id(t) in self._slot_of and self._metas[self._slot_of[id(t)]] is t

    def _const(self, t):
        i = self._const_of.get(id(t))
        if i is None or self._consts[i] is not t:
            i = len(self._consts)
            self._consts.append(t)
            self._const_of[id(t)] = i
            prm = _PARAM_OF.get(id(t))
            if prm is not None:
                self._params[i] = prm  # the program owns its parameters (layers may be temporaries)
        return _Const(t, i)

    def _template(self, x):
        if isinstance(x, torch.Tensor):
            if self._is_traced(x):
                return _Ref(self._slot_of[id(x)])
            if x.device.type == "meta":
                raise RuntimeError("untraced meta tensor used in a static program")
            return self._const(x)
        if isinstance(x, Tensor):
            return self._template(x._t)
        if isinstance(x, list):
            return [self._template(v) for v in x]
        if isinstance(x, tuple):
            return tuple(self._template(v) for v in x)
        if isinstance(x, dict):
            return {k: self._template(v) for k, v in x.items()}
        if isinstance(x, torch.device) and x.type == "meta":
            return _RUN_DEV
        return x

    def _to_meta(self, x):
        if isinstance(x, torch.Tensor):
            if x.device.type == "meta":
                return x
            return x.detach().to(_META).requires_grad_(x.requires_grad) if x.is_floating_point() else x.to(_META)
        if isinstance(x, list):
            return [self._to_meta(v) for v in x]
        if isinstance(x, tuple) and not isinstance(x, torch.Size):
            return tuple(self._to_meta(v) for v in x)
        if isinstance(x, dict):
            return {k: self._to_meta(v) for k, v in x.items()}
        return x

    def _out_template(self, y):
        if isinstance(y, torch.Tensor):
            if self._is_traced(y):
                return _Ref(self._slot_of[id(y)])
            if y.device.type != "meta":
                return None  # real value produced from traced inputs (should not happen)
            return _Ref(self._new_slot(y))
        if isinstance(y, (list, tuple)) and not isinstance(y, torch.Size):
            return type(y)(self._out_template(v) for v in y) if isinstance(y, tuple) and not hasattr(y, "_fields") \
                else [self._out_template(v) for v in y]
        return None

    @staticmethod
    def _any(x, pred):
        if pred(x):
            return True
        if isinstance(x, (list, tuple)) and not isinstance(x, torch.Size):
            return any(Program._any(v, pred) for v in x)
        if isinstance(x, dict):
            return any(Program._any(v, pred) for v in x.values())
        return False

    # ------------------------------------------------------------ recording
    def _record(self, func, args, kwargs, kind="torch"):
        traced = self._any((args, kwargs), self._is_traced)
        name = _func_name(func)
        if traced and name in _BREAK_FUNCS:
            if self._shadow is None:
                raise RuntimeError(f"{name[2:]}() of a traced value: the Python result depends on tensor data")
            return self._guard(func, args, kwargs, name)
        if not traced:
            out = func(*args, **kwargs)
            # factories creating tensors on the trace device (torch.arange(..., device=x.device))
            if self._any(out, lambda t: isinstance(t, torch.Tensor) and t.device.type == "meta"
                         and not self._is_traced(t)):
                node = OpNode(func, self._template(args), self._template(kwargs), None, kind, name)
                node.outs = self._out_template(out)
                self._append(node)
            return out
        if name[2:] in _PURE_GETTERS or name.split(":")[-1] in _PURE_GETTERS:
            return func(*self._to_meta(args), **self._to_meta(kwargs))
        targs, tkw = self._template(args), self._template(kwargs)
        margs, mkw = self._to_meta(args), self._to_meta(kwargs)
        if name == "m:cpu" and self._shadow is not None:
            # a host copy of a traced value (ahead of .numpy() / .tolist()): traced as a meta value of the
            # same shape, the shadow holds the real host tensor
            with torch._C.DisableTorchFunction():
                out = torch.empty(margs[0].shape, dtype=margs[0].dtype, device=_META)
        else:
            out = func(*margs, **mkw)
        node = OpNode(func, targs, tkw, None, kind, name)
        node.outs = self._out_template(out)
        self._append(node)
        return out

    @contextlib.contextmanager
    def recompute_scope(self, enabled=True):
        """Nodes recorded inside form one recompute segment (reference: auto_parallel/interface.py:210 recompute,
        whose ops carry a recompute id the recompute pass groups by); ``enabled=False`` excludes them from any
        enclosing segment (exclude_ops_in_recompute)."""
        prev = self._rc
        self._rc = next(self._rc_ids) if enabled else None
        try:
            yield self._rc
        finally:
            self._rc = prev

    def _append(self, node):
        if self._rc is not None and hasattr(node, "rc"):
            node.rc = self._rc
        self._cur.append(node)
        self._version += 1
        self._plans.clear()
        if self._shadow is not None and self._cur is self.nodes and not isinstance(node, GuardNode):
            self._shadow_exec(node)

    def _shadow_exec(self, node):
        """Run a freshly recorded top-level node on the shadow values (no recording, no autograd)."""
        with torch._C.DisableTorchFunction(), torch.no_grad():
            _exec_node(node, self._shadow, None, self._shadow_dev, None)

    def _guard(self, func, args, kwargs, name):
        targs, tkw = self._template(args), self._template(kwargs)
        with torch._C.DisableTorchFunction(), torch.no_grad():
            val = func(*_materialize(targs, self._shadow, None, self._shadow_dev),
                       **_materialize(tkw, self._shadow, None, self._shadow_dev))
        self._append(GuardNode(func, targs, tkw, val, name))
        return val

    @contextlib.contextmanager
    def _sub_block(self):
        """Record into a fresh node list (a control-flow sub-block) sharing this program's value slots."""
        old = self._cur
        blk = []
        self._cur = blk
        try:
            yield blk
        finally:
            self._cur = old

    def _new_like(self, meta):
        """A fresh traced value with the shape / dtype of ``meta`` (control-flow outputs, loop variables)."""
        with torch._C.DisableTorchFunction():
            m = torch.empty(meta.shape, dtype=meta.dtype, device=_META)
            if meta.requires_grad and m.is_floating_point():
                m.requires_grad_(True)
        self._new_slot(m)
        return m

    # ------------------------------------------------------------ user API
    def global_block(self):
        return _Block(self)

    def block(self, i=0):
        return _Block(self)

    @property
    def num_blocks(self):
        return 1 + sum(_count_blocks(n) for n in self.nodes)

    def current_block(self):
        return _Block(self)

    def all_parameters(self):
        return [self._params[i] for i in sorted(self._params)]

    def list_vars(self):
        out = []
        for name, (slot, shape, dtype) in self.feeds.items():
            out.append(_Var(self, slot, name))
        return out + self.all_parameters()

    def clone(self, for_test=False):
        p = Program.__new__(Program)
        p.__dict__.update(self.__dict__)
        p.nodes = list(self.nodes)
        p._cur = p.nodes
        p._plans = {}
        p._id = next(Program._ids)
        if for_test:
            p._optimize = None
            p._is_test = True
        return p

    def _set_optimizer(self, opt, loss):
        slot = self._slot_of.get(id(loss._t))
        if slot is None:
            raise ValueError("loss is not a variable of this program")
        if not opt._parameter_list:
            params = [p for p in self.all_parameters() if not p.stop_gradient]
            opt._param_groups = [{"params": params}]
            opt._parameter_list = params
        self._optimize = (opt, slot)
        self._plans.clear()

    def __repr__(self):
        lines = [f"Program(id={self._id}, {len(self.nodes)} ops, feeds={list(self.feeds)})"]
        for n in self.nodes[:200]:
            lines.append("  " + repr(n))
        return "\n".join(lines)

    def to_string(self, throw_on_error=False, with_details=False):
        return repr(self)

    # ------------------------------------------------------------ (de)serialization
    def to_dict(self, fetch_slots, const_names):
        enc = _Encoder(const_names)
        nodes = [_encode_node(n, enc) for n in self.nodes]
        return {"format": "paddlepaddle_amd.program", "version": 1,
                "n_slots": len(self._metas),
                "slot_meta": [[list(m.shape), str(m.dtype).replace("torch.", "")] for m in self._metas],
                "feeds": [{"name": k, "slot": s, "shape": list(sh), "dtype": d} for k, (s, sh, d) in self.feeds.items()],
                "fetch": list(fetch_slots), "nodes": nodes, "dyn": self._dyn}

    @staticmethod
    def from_dict(d, consts_by_name):
        if d.get("format") != "paddlepaddle_amd.program":
            raise ValueError("not a paddlepaddle_amd program file")
        p = Program()
        for shape, dt in d["slot_meta"]:
            p._new_slot(torch.empty(shape, dtype=getattr(torch, dt), device=_META))
        dec = _Decoder(p, consts_by_name)
        for nd in d["nodes"]:
            p.nodes.append(_decode_node(nd, dec))
        for f in d["feeds"]:
            p.feeds[f["name"]] = (f["slot"], tuple(f["shape"]), f["dtype"])
            p._names[f["name"]] = f["slot"]
        p._dyn = d.get("dyn", False)
        return p, list(d["fetch"])


class _Block:
    def __init__(self, prog):
        self.program = prog
        self.idx = 0

    @property
    def ops(self):
        return list(self.program.nodes)

    @property
    def vars(self):
        return {v.name: v for v in self.program.list_vars()}

    def var(self, name):
        p = self.program
        if name in p._names:
            return _Var(p, p._names[name], name)
        for q in p.all_parameters():
            if q.name == name:
                return q
        raise ValueError(f"var {name} not in program")

    has_var = lambda self, name: name in self.program._names or any(  # noqa: E731
        q.name == name for q in self.program.all_parameters())

    def all_parameters(self):
        return self.program.all_parameters()


def _Var(prog, slot, name):
    t = _wrap(prog._metas[slot])
    t._name = name
    return t


from ..framework.tensor import _PARAM_OF  # noqa: E402  id(parameter buffer) -> Parameter


# ---------------------------------------------------------------------------------- tracer
class _Tracer(TorchFunctionMode):
    def __init__(self, program):
        super().__init__()
        self.program = program

    def __torch_function__(self, func, types, args=(), kwargs=None):
        return self.program._record(func, args, kwargs or {})


from ..framework.trace_hook import _state, _active_program, static_op  # noqa: E402,F401


@contextlib.contextmanager
def trace_into(program):
    """Record every op touching traced values into ``program``."""
    st = getattr(_state, "stack", None)
    if st is None:
        st = _state.stack = []
    tr = _Tracer(program)
    st.append(tr)
    tr.__enter__()
    try:
        yield program
    finally:
        tr.__exit__(None, None, None)
        st.pop()


def placeholder(program, name, shape, dtype, need_grad=False):
    """Create a traced input (feed) variable."""
    sh = [SENTINEL if (s is None or s < 0) else int(s) for s in shape]
    td = _dt.to_torch_dtype(dtype)
    with torch._C.DisableTorchFunction():
        meta = torch.empty(sh, dtype=td, device=_META)
    if need_grad and meta.is_floating_point():
        meta.requires_grad_(True)
    slot = program._new_slot(meta)
    program.feeds[name] = (slot, tuple(-1 if (s is None or s < 0) else int(s) for s in shape),
                           str(td).replace("torch.", ""))
    program._names[name] = slot
    if need_grad:
        program._need_grad_slots.add(slot)
    t = _wrap(meta)
    t._name = name
    return t


# ---------------------------------------------------------------------------------- replay
class _Plan:
    def __init__(self, order, free_after, nodes):
        self.order = order
        self.free_after = free_after  # position -> list of slots to drop
        self.nodes = nodes


def _refs(tmpl, acc):
    if isinstance(tmpl, _Ref):
        acc.append(tmpl.i)
    elif isinstance(tmpl, (list, tuple)):
        for v in tmpl:
            _refs(v, acc)
    elif isinstance(tmpl, dict):
        for v in tmpl.values():
            _refs(v, acc)
    return acc


def build_plan(program, fetch_slots, keep_slots=()):
    """Prune to what the fetches need, then let the native scheduler order nodes and compute
    last uses (reference: new_executor dependency builder + GC)."""
    from ..utils import native
    nodes = program.nodes
    reads = [_node_reads(n) for n in nodes]
    writes = [_node_writes(n) for n in nodes]
    # liveness pruning (backwards from the fetches)
    need = set(fetch_slots) | set(keep_slots)
    live = [False] * len(nodes)
    for i in range(len(nodes) - 1, -1, -1):
        if writes[i] & need or nodes[i].kind == "guard":
            live[i] = True
            need |= reads[i]
    idx = [i for i in range(len(nodes)) if live[i]]
    pos_of = {i: k for k, i in enumerate(idx)}
    creator, last_writer, readers = {}, {}, {}
    edges = set()
    for k, i in enumerate(idx):
        for s in reads[i]:
            if s in last_writer:
                edges.add((pos_of[last_writer[s]], k))
            if s in creator and creator[s] != i:
                edges.add((pos_of[creator[s]], k))
            readers.setdefault(s, []).append(k)
        for s in writes[i]:
            for r in readers.get(s, []):  # write-after-read
                if r != k:
                    edges.add((r, k))
            if s in last_writer and last_writer[s] != i:
                edges.add((pos_of[last_writer[s]], k))
            creator.setdefault(s, i)
            last_writer[s] = i
    # auto_parallel_supplement_explicit_dependencies: consecutive collectives keep their traced order
    chain = getattr(program, "_pa_comm_chain", None)
    if chain:
        at = {id(nodes[i]): k for k, i in enumerate(idx)}
        ks = [at[c] for c in chain if c in at]
        edges.update(zip(ks, ks[1:]))
    keep_nodes = {pos_of[creator[s]] for s in set(fetch_slots) | set(keep_slots) if s in creator}
    keep_nodes |= {k for k, i in enumerate(idx) if nodes[i].kind == "guard"}
    # collectives are issued as soon as their inputs exist (they run on the comm stream and overlap the
    # compute that does not depend on them)
    prio = [0 if nodes[i].kind in ("comm", "guard") else 1 for i in idx]
    order, last = native.schedule(len(idx), sorted(edges), sorted(keep_nodes), prio)
    pos = {v: p for p, v in enumerate(order)}
    free_after = {}
    feeds = {s for (s, _, _) in program.feeds.values()}
    for s, ci in creator.items():
        if s in fetch_slots or s in keep_slots or s in feeds:
            continue
        lp = last[pos_of[ci]]
        if lp >= 0:
            # a slot may be read by nodes that are not successors of its creator only through
            # in-place writers; those writers are successors, so last[] covers them
            free_after.setdefault(lp, []).append(s)
    return _Plan([idx[v] for v in order], free_after, nodes)


def _materialize(tmpl, env, consts, dev, sym_n=None):
    if isinstance(tmpl, _Ref):
        return env[tmpl.i]
    if isinstance(tmpl, _Const):
        return consts[tmpl.idx] if consts is not None else tmpl.t
    if tmpl is _RUN_DEV:
        return dev
    if isinstance(tmpl, _Sym):
        return tmpl.a * sym_n + tmpl.b
    if isinstance(tmpl, slice):
        return slice(_materialize(tmpl.start, env, consts, dev, sym_n), _materialize(tmpl.stop, env, consts, dev, sym_n),
                     _materialize(tmpl.step, env, consts, dev, sym_n))
    if isinstance(tmpl, list):
        return [_materialize(v, env, consts, dev, sym_n) for v in tmpl]
    if isinstance(tmpl, tuple):
        return tuple(_materialize(v, env, consts, dev, sym_n) for v in tmpl)
    if isinstance(tmpl, dict):
        return {k: _materialize(v, env, consts, dev, sym_n) for k, v in tmpl.items()}
    return tmpl


def _assign(tmpl, val, env):
    if isinstance(tmpl, _Ref):
        env[tmpl.i] = val
    elif isinstance(tmpl, (list, tuple)):
        for t, v in zip(tmpl, val):
            _assign(t, v, env)


def _is_inplace(n):
    return n.kind == "comm" or n.name == "m:__setitem__" or (
        n.name.startswith("m:") and n.name.endswith("_") and not n.name.endswith("__"))


def _node_reads(n):
    if isinstance(n, CFNode):
        return n.reads()
    return set(_refs((n.args, n.kwargs), []))


def _node_writes(n):
    w = set(_refs(n.outs, []))
    if n.kind == "comm":
        w |= set(_refs(n.args, []))  # a collective writes every tensor it is given (coalesced: all of them)
    elif _is_inplace(n):
        w |= set(_refs(n.args[:1], []))  # in-place: the receiver is written
    return w


def _exec_node(n, env, consts, dev, sym_n):
    if isinstance(n, CFNode):
        n.execute(env, consts, dev, sym_n)
        return
    args = _materialize(n.args, env, consts, dev, sym_n)
    kw = _materialize(n.kwargs, env, consts, dev, sym_n)
    if n.kind == "guard":
        with torch.no_grad():
            n.check(n.func(*args, **kw))
        return
    out = n.func(*args, **kw)
    if n.outs is not None:
        _assign(n.outs, out, env)


class _Streams:
    """Compute + communication HIP streams of one plan run. A collective waits for the compute issued
    before it (its input is ready), runs on the comm stream and records an event; a later node reading
    what the collective wrote waits for that event. Compute that does not depend on the collective keeps
    running on the compute stream meanwhile."""

    def __init__(self, dev):
        self.comp = torch.cuda.current_stream(dev)
        self.comm = _comm_stream(dev)
        self.pending = {}  # slot -> event recorded on the comm stream after the collective that wrote it
        self.keep = []     # tensors the comm stream touched: alive until finish() (allocators without
                           # record_stream would otherwise hand their memory to the compute stream early)

    def before(self, n, reads):
        if n.kind == "comm":
            self.comm.wait_stream(self.comp)
            return self.comm
        for s in reads:
            ev = self.pending.pop(s, None)
            if ev is not None:
                self.comp.wait_event(ev)
        return self.comp

    def after(self, n, writes, env):
        if n.kind != "comm":
            return
        ev = torch.cuda.Event()
        ev.record(self.comm)
        for s in writes:
            self.pending[s] = ev
            t = env.get(s)
            if isinstance(t, torch.Tensor) and t.is_cuda:
                t.record_stream(self.comm)
                self.keep.append(t)

    def finish(self):
        if self.pending or self.keep:
            self.comp.wait_stream(self.comm)
        self.keep = []


_COMM_STREAMS = {}


def _comm_stream(dev):
    s = _COMM_STREAMS.get(dev)
    if s is None:
        s = _COMM_STREAMS[dev] = torch.cuda.Stream(dev)
    return s


def run_plan(program, plan, env, dev, consts=None, sym_n=None):
    fa = plan.free_after
    multi = dev is not None and getattr(dev, "type", None) == "cuda" and any(
        plan.nodes[i].kind == "comm" for i in plan.order)
    st = _Streams(dev) if multi else None
    for p, ni in enumerate(plan.order):
        n = plan.nodes[ni]
        if st is None:
            _exec_node(n, env, consts, dev, sym_n)
        else:
            stream = st.before(n, _node_reads(n))
            with torch.cuda.stream(stream):
                _exec_node(n, env, consts, dev, sym_n)
            st.after(n, _node_writes(n), env)
        for s in fa.get(p, ()):
            env.pop(s, None)
    if st is not None:
        st.finish()
    return env


# ---------------------------------------------------------------------------------- control flow
class _SubBlock:
    """Ops recorded for one branch / loop body: executed in recording order on the parent's value slots;
    values created inside are dropped when the block finishes (reference: conditional_block /
    while sub-blocks run by the interpreter)."""

    def __init__(self, nodes):
        self.nodes = nodes
        self._inner = None

    def inner(self):
        """Values created in the block (not outer values it updates in place)."""
        if self._inner is None:
            w = set()
            for n in self.nodes:
                w |= set(_refs(n.outs, []))
            self._inner = w
        return self._inner

    def free_reads(self):
        r, made = set(), set()
        for n in self.nodes:
            r |= _node_reads(n) - made
            made |= set(_refs(n.outs, []))
        return r

    def run(self, env, consts, dev, sym_n):
        for n in self.nodes:
            _exec_node(n, env, consts, dev, sym_n)

    def drop(self, env, keep=()):
        for sl in self.inner():
            if sl not in keep:
                env.pop(sl, None)


class CFNode(OpNode):
    """A control-flow op owning sub-blocks (kind "cond" or "while")."""
    __slots__ = ("blocks", "res", "loop_slots")

    def __init__(self, kind, args, outs, blocks, res, loop_slots=()):
        super().__init__(None, args, {}, outs, kind=kind, name="cf:" + kind)
        self.blocks = blocks          # [_SubBlock]
        self.res = res                # per block: template of its result (cond: branch value; while: pred, body)
        self.loop_slots = tuple(loop_slots)

    def reads(self):
        r = set(_refs(self.args, []))
        for b, res in zip(self.blocks, self.res):
            r |= b.free_reads() | (set(_refs(res, [])) - b.inner())
        return r - set(self.loop_slots)

    def execute(self, env, consts, dev, sym_n):
        m = lambda t: _materialize(t, env, consts, dev, sym_n)  # noqa: E731
        if self.kind == "cond":
            pred = m(self.args[0])
            take = bool(pred.reshape(()).item()) if isinstance(pred, torch.Tensor) else bool(pred)
            i = 0 if take else 1
            blk = self.blocks[i]
            blk.run(env, consts, dev, sym_n)
            val = m(self.res[i])
            blk.drop(env)
            _assign(self.outs, val, env)
            return
        # while: loop variables live in loop_slots; blocks = (cond block, body block)
        cblk, bblk = self.blocks
        for sl, v in zip(self.loop_slots, m(self.args)):
            env[sl] = v
        while True:
            cblk.run(env, consts, dev, sym_n)
            pred = m(self.res[0])
            cblk.drop(env, keep=self.loop_slots)
            if not (bool(pred.reshape(()).item()) if isinstance(pred, torch.Tensor) else bool(pred)):
                break
            bblk.run(env, consts, dev, sym_n)
            new = m(self.res[1])
            bblk.drop(env, keep=self.loop_slots)
            for sl, v in zip(self.loop_slots, new):
                env[sl] = v
        _assign(self.outs, [env.pop(sl) for sl in self.loop_slots], env)


def _count_blocks(n):
    if not isinstance(n, CFNode):
        return 0
    return sum(1 + sum(_count_blocks(x) for x in b.nodes) for b in n.blocks)


def _encode_node(n, enc):
    if n.kind == "guard":
        raise ValueError("a program specialised by data guards (jit.to_static graph breaks) cannot be saved; "
                         "save with an input_spec instead")
    if isinstance(n, CFNode):
        return {"f": n.name, "a": enc(n.args), "o": enc(n.outs), "loop": list(n.loop_slots),
                "blocks": [[_encode_node(x, enc) for x in b.nodes] for b in n.blocks],
                "res": [enc(r) for r in n.res]}
    return {"f": n.name, "a": enc(n.args), "k": enc(n.kwargs), "o": enc(n.outs)}


def _decode_node(nd, dec):
    if nd["f"].startswith("cf:"):
        blocks = [_SubBlock([_decode_node(x, dec) for x in b]) for b in nd["blocks"]]
        return CFNode(nd["f"][3:], dec(nd["a"]), dec(nd["o"]), blocks, [dec(r) for r in nd["res"]],
                      nd.get("loop", ()))
    return OpNode(_resolve(nd["f"]), dec(nd["a"]), dec(nd["k"]), dec(nd["o"]), name=nd["f"])


def _grad_node_fn(n_targets, retain):
    def _grad(*ts):
        targets, inputs = list(ts[:n_targets]), list(ts[n_targets:])
        gs = torch.autograd.grad(targets, inputs, allow_unused=True, retain_graph=True, create_graph=False)
        return tuple(torch.zeros_like(i) if g is None else g for g, i in zip(gs, inputs))
    return _grad


# ---------------------------------------------------------------------------------- JSON codec
class _Encoder:
    def __init__(self, const_names):
        self.const_names = const_names

    def __call__(self, x):
        if isinstance(x, _Ref):
            return {"r": x.i}
        if isinstance(x, _Const):
            return {"c": self.const_names[x.idx]}
        if x is _RUN_DEV:
            return {"dev": 1}
        if isinstance(x, _Sym):
            return {"sym": [x.a, x.b]}
        if isinstance(x, torch.dtype):
            return {"dt": str(x).replace("torch.", "")}
        if isinstance(x, torch.device):
            return {"dev": 1}
        if isinstance(x, torch.memory_format):
            return {"mf": str(x).replace("torch.", "")}
        if isinstance(x, torch.layout):
            return {"ly": str(x).replace("torch.", "")}
        if isinstance(x, slice):
            return {"sl": [self(x.start), self(x.stop), self(x.step)]}
        if x is Ellipsis:
            return {"el": 1}
        if isinstance(x, float) and (x != x or x in (float("inf"), float("-inf"))):
            return {"fl": repr(x)}
        if isinstance(x, tuple):
            return {"t": [self(v) for v in x]}
        if isinstance(x, list):
            return [self(v) for v in x]
        if isinstance(x, dict):
            return {"d": {k: self(v) for k, v in x.items()}}
        if x is None or isinstance(x, (bool, int, float, str)):
            return x
        raise TypeError(f"cannot serialize program argument of type {type(x).__name__}")


class _Decoder:
    def __init__(self, prog, consts_by_name):
        self.prog = prog
        self.consts = consts_by_name

    def __call__(self, x):
        if isinstance(x, list):
            return [self(v) for v in x]
        if not isinstance(x, dict):
            return x
        if "r" in x:
            return _Ref(x["r"])
        if "c" in x:
            c = self.prog._const(self.consts[x["c"]])
            self.prog.__dict__.setdefault("_const_alias", {})[c.idx] = x["c"]  # keep the saved name
            return c
        if "dev" in x:
            return _RUN_DEV
        if "sym" in x:
            return _Sym(*x["sym"])
        if "dt" in x:
            return getattr(torch, x["dt"])
        if "mf" in x:
            return getattr(torch, x["mf"])
        if "ly" in x:
            return getattr(torch, x["ly"])
        if "sl" in x:
            return slice(*[self(v) for v in x["sl"]])
        if "el" in x:
            return Ellipsis
        if "fl" in x:
            return float(x["fl"])
        if "t" in x:
            return tuple(self(v) for v in x["t"])
        if "d" in x:
            return {k: self(v) for k, v in x["d"].items()}
        raise ValueError(f"bad program entry {x}")
