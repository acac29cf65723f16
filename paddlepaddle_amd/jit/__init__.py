"""paddle.jit: to_static / save / load / TranslatedLayer.

Reference: python/paddle/jit/api.py:197 (to_static), :880 (save), :1440 (load),
jit/dy2static/program_translator.py (StaticFunction, concrete programs), jit/translated_layer.py.

No bytecode translation and no tracing compiler: ``to_static`` records the function once per input
signature into a static ``Program`` (static/program.py: meta-tensor tracing, whole-op nodes for the
HIP kernels) and replays it; autograd flows through the replay, so training works unchanged.

Graph breaks (the reference's SOT, jit/sot/translate.py:31, splits the bytecode where Python needs a
tensor's *value*): when the meta trace hits bool(t) / t.item() / t.tolist() / ..., the function is traced
again in *guarded* mode — every op also runs on the real inputs (shadow values), each such conversion
returns the real value and is recorded as a GuardNode, so the trace follows the branch / trip count the
data selects. Replay re-evaluates the guards as early as their inputs exist; a mismatch raises
GuardFailure and the next recorded variant for that signature is tried, or a new one is traced (up to
``_MAX_VARIANTS`` per signature, then eager). So data-dependent control flow keeps running as replayed
programs (one per observed path) instead of falling back to eager. Caveat: a variant that fails a guard
after an in-place update of a parameter / buffer has applied that update once already.
Optionally the replay of an inference-only signature is captured into a hipGraph
(``to_static(..., backend="hipgraph")``; not for guarded programs — a guard reads data on the host).
``jit.save`` writes the JSON program + params; dynamic (None) dims are supported when every shape
argument in the program is an affine function of them (checked by tracing at three sizes).
"""
from __future__ import annotations

import functools
import inspect
import os
import warnings

import numpy as np
import torch

from ..framework.tensor import Tensor, Parameter, _wrap
from ..static import program as P
from ..static.executor import InputSpec
from ..static import io as _sio

_enabled = True
_ignored = set()


def enable_to_static(enable_to_static_bool=True):
    global _enabled
    _enabled = bool(enable_to_static_bool)


def ignore_module(modules):
    _ignored.update(modules if isinstance(modules, (list, tuple)) else [modules])


def not_to_static(func=None):
    if func is None:
        return not_to_static
    func._not_to_static = True
    return func


def _flatten(x, out):
    if isinstance(x, (list, tuple)):
        return type(x)(_flatten(v, out) for v in x) if not hasattr(x, "_fields") else x
    if isinstance(x, dict):
        return {k: _flatten(v, out) for k, v in x.items()}
    if isinstance(x, Tensor):
        out.append(x)
        return _Leaf(len(out) - 1)
    return x


class _Leaf:
    __slots__ = ("i",)

    def __init__(self, i):
        self.i = i

    def __eq__(self, o):
        return isinstance(o, _Leaf) and o.i == self.i

    def __hash__(self):
        return hash(("leaf", self.i))

    def __repr__(self):
        return f"<in{self.i}>"


def _key_of(struct):
    try:
        return repr(struct)
    except Exception:
        return str(id(struct))


def _rebuild(tmpl, vals):
    if isinstance(tmpl, _Leaf):
        return vals[tmpl.i]
    if isinstance(tmpl, (list, tuple)):
        return type(tmpl)(_rebuild(v, vals) for v in tmpl)
    if isinstance(tmpl, dict):
        return {k: _rebuild(v, vals) for k, v in tmpl.items()}
    return tmpl


_MAX_VARIANTS = 8


class ConcreteProgram:
    """One recorded signature (one data-dependent path when guarded): program + feed slots + output
    template."""

    def __init__(self, program, feed_slots, out_tmpl, fetch_slots):
        self.main_program = program
        self.program = program
        self.feed_slots = feed_slots
        self.out_tmpl = out_tmpl
        self.fetch_slots = fetch_slots
        self.plan = P.build_plan(program, fetch_slots)
        self.graph = None
        self.guarded = any(n.kind == "guard" for n in program.nodes)

    @property
    def guards(self):
        return [n for n in self.program.nodes if n.kind == "guard"]

    @property
    def parameters(self):
        return self.program.all_parameters()

    def run(self, tensors, dev):
        env = {s: t._t for s, t in zip(self.feed_slots, tensors)}
        P.run_plan(self.program, self.plan, env, dev)
        outs = [env[s] for s in self.fetch_slots]
        return _rebuild_out(self.out_tmpl, outs)


def _out_template(prog, out, fetch):
    if isinstance(out, Tensor):
        s = prog._slot_of.get(id(out._t))
        if s is None or prog._metas[s] is not out._t:
            return ("const", out)
        fetch.append(s)
        return ("slot", len(fetch) - 1)
    if isinstance(out, (list, tuple)):
        return (type(out).__name__, [_out_template(prog, v, fetch) for v in out])
    if isinstance(out, dict):
        return ("dict", {k: _out_template(prog, v, fetch) for k, v in out.items()})
    return ("py", out)


def _rebuild_out(t, outs):
    kind, v = t
    if kind == "slot":
        return _wrap(outs[v])
    if kind == "list":
        return [_rebuild_out(x, outs) for x in v]
    if kind == "tuple":
        return tuple(_rebuild_out(x, outs) for x in v)
    if kind == "dict":
        return {k: _rebuild_out(x, outs) for k, x in v.items()}
    return v


def trace_program(fn, args, kwargs, names=None, dyn_size=None, guarded=False):
    """Record ``fn(*args, **kwargs)`` into a fresh Program. Tensor leaves of the inputs become feeds;
    for InputSpec leaves a placeholder of that spec is created (-1 dims -> ``dyn_size``). ``guarded``:
    dual tracing on the real tensor leaves (data-dependent Python values become guards)."""
    prog = P.Program()
    leaves = []
    struct = _flatten((args, kwargs), leaves)
    spec_leaves = []

    def _spec_flat(x):
        if isinstance(x, InputSpec):
            spec_leaves.append(x)
            return _Leaf(-len(spec_leaves))
        if isinstance(x, (list, tuple)):
            return type(x)(_spec_flat(v) for v in x)
        if isinstance(x, dict):
            return {k: _spec_flat(v) for k, v in x.items()}
        return x
    struct = _spec_flat(struct)
    feeds, feed_slots, n_in = [], [], 0

    def mk(x, i):
        nonlocal n_in
        name = (names[n_in] if names and n_in < len(names) else None) or f"x{n_in}"
        n_in += 1
        if isinstance(x, InputSpec):
            shape = [dyn_size if (s is None or s < 0) and dyn_size else s for s in x.shape]
            v = P.placeholder(prog, x.name or name, shape, x.dtype)
            if dyn_size:
                slot = prog.feeds[x.name or name][0]
                prog.feeds[x.name or name] = (slot, tuple(x.shape), prog.feeds[x.name or name][2])
        else:
            v = P.placeholder(prog, name, x.shape, x.dtype, need_grad=not x.stop_gradient)
        feed_slots.append(prog.feeds[v._name][0])
        return v
    ph_tensors = [mk(x, i) for i, x in enumerate(leaves)]
    ph_specs = [mk(x, i) for i, x in enumerate(spec_leaves)]

    def fill(x):
        if isinstance(x, _Leaf):
            return ph_tensors[x.i] if x.i >= 0 else ph_specs[-x.i - 1]
        if isinstance(x, (list, tuple)):
            return type(x)(fill(v) for v in x)
        if isinstance(x, dict):
            return {k: fill(v) for k, v in x.items()}
        return x
    a, k = fill(struct)
    if guarded:
        prog._shadow = {s: x._t for s, x in zip(feed_slots, leaves)}
        prog._shadow_dev = leaves[0]._t.device if leaves else torch.device("cpu")
    try:
        with P.trace_into(prog):
            out = fn(*a, **k)
    finally:
        prog._shadow = None
    _check_defined(out)
    fetch = []
    tmpl = _out_template(prog, out, fetch)
    return prog, feed_slots, tmpl, fetch


def _check_defined(x):
    """A converted program must not return a name bound on only one path (dy2static UndefinedVar)."""
    from .dy2static.convert_operators import UndefinedVar
    if isinstance(x, UndefinedVar):
        x._fail()
    if isinstance(x, (list, tuple)):
        for v in x:
            _check_defined(v)
    elif isinstance(x, dict):
        for v in x.values():
            _check_defined(v)


class StaticFunction:
    def __init__(self, function, input_spec=None, build_strategy=None, backend=None, full_graph=True,
                 instance=None):
        self._dygraph_function = function
        self._input_spec = input_spec
        self._instance = instance
        self._cache = {}        # signature -> the most recently used program
        self._variants = {}     # signature -> guarded variants (most recently used first)
        self._backend = backend
        self._eager_keys = set()
        functools.update_wrapper(self, function)

    def __get__(self, instance, owner):
        if instance is None:
            return self
        key = "_static_fn_" + self._dygraph_function.__name__
        bound = instance.__dict__.get(key)
        if bound is None:
            bound = StaticFunction(self._dygraph_function, self._input_spec, None, self._backend, True, instance)
            instance.__dict__[key] = bound
        return bound

    def _call_eager(self, *args, **kwargs):
        if self._instance is not None:
            return self._dygraph_function(self._instance, *args, **kwargs)
        return self._dygraph_function(*args, **kwargs)

    def _signature(self, args, kwargs):
        leaves = []
        struct = _flatten((args, kwargs), leaves)
        sig = tuple((tuple(t.shape), str(t._t.dtype), t._t.device.type, t.stop_gradient) for t in leaves)
        training = getattr(self._instance, "training", None)
        return (_key_of(struct), sig, training, torch.is_grad_enabled()), leaves

    def __call__(self, *args, **kwargs):
        if not _enabled or getattr(self._dygraph_function, "_not_to_static", False) or P._active_program():
            return self._call_eager(*args, **kwargs)
        key, leaves = self._signature(args, kwargs)
        if key in self._eager_keys:
            return self._call_eager(*args, **kwargs)
        dev = leaves[0]._t.device if leaves else torch.device("cpu")
        cp = self._cache.get(key)
        if cp is None:
            try:
                cp = self._trace(args, kwargs, guarded=False)
            except Exception:  # a Python conversion of tensor data (graph break): trace with guards
                try:
                    cp = self._trace(args, kwargs, guarded=True)
                except Exception as e:
                    warnings.warn(f"to_static: falling back to eager for {self._dygraph_function.__name__}: {e}")
                    self._eager_keys.add(key)
                    return self._call_eager(*args, **kwargs)
            self._cache[key] = cp
            self._variants[key] = [cp]
        if cp.guarded:
            return self._run_guarded(key, args, kwargs, leaves, dev)
        if self._backend in ("hipgraph", "cudagraph") and dev.type == "cuda" and not torch.is_grad_enabled():
            return self._graph_call(cp, leaves, dev)
        return cp.run(leaves, dev)

    def _converted(self):
        """The dy2static (AST) conversion of the wrapped function: tensor-dependent if / while / for-range
        become control-flow nodes of the program (jit/dy2static); None when nothing was rewritten."""
        conv = self.__dict__.get("_conv")
        if conv is None:
            from .dy2static import convert_to_static
            conv = convert_to_static(self._dygraph_function)
            self._conv = conv
        return None if conv is self._dygraph_function else conv

    def _call_converted(self, *args, **kwargs):
        conv = self._converted() or self._dygraph_function
        if self._instance is not None:
            return conv(self._instance, *args, **kwargs)
        return conv(*args, **kwargs)

    def _trace(self, args, kwargs, guarded):
        from .dy2static import conversion_scope
        if not guarded:
            # converted source first: data-dependent branches / loops become one program with control-flow nodes
            try:
                with conversion_scope():
                    prog, feed_slots, tmpl, fetch = trace_program(self._call_converted, args, kwargs)
                return ConcreteProgram(prog, feed_slots, tmpl, fetch)
            except Exception:
                if self._converted() is None:
                    raise
        prog, feed_slots, tmpl, fetch = trace_program(self._call_eager, args, kwargs, guarded=guarded)
        return ConcreteProgram(prog, feed_slots, tmpl, fetch)

    def _run_guarded(self, key, args, kwargs, leaves, dev):
        vs = self._variants[key]
        for i, cp in enumerate(vs):
            try:
                out = cp.run(leaves, dev)
            except P.GuardFailure:
                continue
            if i:
                vs.insert(0, vs.pop(i))
                self._cache[key] = cp
            return out
        if len(vs) >= _MAX_VARIANTS:
            warnings.warn(f"to_static: {self._dygraph_function.__name__} took more than {_MAX_VARIANTS} "
                          "data-dependent paths for one signature; running it eagerly")
            self._eager_keys.add(key)
            return self._call_eager(*args, **kwargs)
        try:
            cp = self._trace(args, kwargs, guarded=True)
        except Exception as e:
            warnings.warn(f"to_static: falling back to eager for {self._dygraph_function.__name__}: {e}")
            self._eager_keys.add(key)
            return self._call_eager(*args, **kwargs)
        vs.insert(0, cp)
        self._cache[key] = cp
        return cp.run(leaves, dev)

    def variants(self, *args, **kwargs):
        """Programs recorded for the signature of these arguments (one per observed data-dependent path)."""
        key, _ = self._signature(args, kwargs)
        return list(self._variants.get(key, []))

    def _graph_call(self, cp, leaves, dev):
        """Capture the replay once into a hipGraph with static input/output buffers."""
        if cp.graph is None:
            static_in = [_wrap(t._t.clone()) for t in leaves]
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                cp.run(static_in, dev)  # warm-up (allocator, library handles)
            torch.cuda.current_stream().wait_stream(s)
            from ..device.cuda.graphs import CUDAGraph, capture
            g = CUDAGraph()
            with capture(g):
                out = cp.run(static_in, dev)
            cp.graph = (g, static_in, out)
        g, static_in, out = cp.graph
        for dst, src in zip(static_in, leaves):
            dst._t.copy_(src._t)
        g.replay()
        return out

    # reference API surface
    @property
    def dygraph_function(self):
        return self._dygraph_function

    def get_concrete_program(self, *args, **kwargs):
        key, leaves = self._signature(args, kwargs)
        if key not in self._cache:
            self(*args, **kwargs)
        cp = self._cache[key]
        return cp, cp.main_program

    @property
    def concrete_program(self):
        if not self._cache:
            raise RuntimeError("no concrete program yet: call the function or pass input_spec")
        return next(iter(self._cache.values()))

    @property
    def program_cache(self):
        return self._cache

    def rollback(self):
        if self._instance is not None:
            self._instance.__dict__.pop("_static_fn_" + self._dygraph_function.__name__, None)
        return self._dygraph_function

    @property
    def code(self):
        return inspect.getsource(self._dygraph_function)


def to_static(function=None, input_spec=None, build_strategy=None, backend=None, full_graph=True, **kwargs):
    """``full_graph=True`` (default here): whole-function trace into one Program (graph breaks become guarded
    variants). ``full_graph=False``: the bytecode translator (jit/sot: guards on Python-level inputs, replayed
    side effects, graph breaks at print / not_to_static calls)."""
    def deco(fn):
        from ..nn.layer.layers import Layer
        if not full_graph and input_spec is None:
            from .sot import symbolic_translate
            return symbolic_translate(fn)
        if isinstance(fn, Layer):
            sf = StaticFunction(type(fn).forward, input_spec, build_strategy, backend, full_graph, instance=fn)
            fn.__dict__["forward"] = sf
            fn._static_forward = sf
            return fn
        return StaticFunction(fn, input_spec, build_strategy, backend, full_graph)
    if function is None:
        return deco
    return deco(function)


declarative = to_static


# ------------------------------------------------------------------------------ save / load
def _specs_for(layer, input_spec):
    if input_spec is None:
        fwd = layer.__dict__.get("forward")
        if isinstance(fwd, StaticFunction) and fwd._input_spec is not None:
            input_spec = fwd._input_spec
        elif isinstance(fwd, StaticFunction) and fwd._cache:
            cp = next(iter(fwd._cache.values()))
            return [InputSpec(cp.program._metas[s].shape, str(cp.program._metas[s].dtype).replace("torch.", ""))
                    for s in cp.feed_slots]
        else:
            raise ValueError("jit.save needs input_spec (or a to_static layer that has been called)")
    out = []
    for s in input_spec:
        if isinstance(s, InputSpec):
            out.append(s)
        elif isinstance(s, Tensor):
            out.append(InputSpec(s.shape, str(s._t.dtype).replace("torch.", ""), s._name))
        else:
            raise TypeError(f"unsupported input_spec entry {s!r}")
    return out


def _fit_affine(t2, t3, t5, n=(2, 3, 5)):
    """Merge three traces of the same template into one with _Sym entries for dims that change."""
    if isinstance(t2, bool) or t2 is None:
        if t2 != t3 or t2 != t5:
            raise ValueError("dynamic dim changes a non-integer argument")
        return t2
    if isinstance(t2, int) and isinstance(t3, int) and isinstance(t5, int):
        if t2 == t3 == t5:
            return t2
        a = (t3 - t2) // (n[1] - n[0])
        b = t2 - a * n[0]
        if a * (n[1] - n[0]) != t3 - t2 or a * n[2] + b != t5:
            raise ValueError("shape argument is not affine in the dynamic dim")
        return P._Sym(a, b)
    if isinstance(t2, (list, tuple)):
        if not isinstance(t3, type(t2)) or len(t2) != len(t3) or len(t2) != len(t5):
            raise ValueError("program structure depends on the dynamic dim")
        return type(t2)(_fit_affine(a, b, c, n) for a, b, c in zip(t2, t3, t5))
    if isinstance(t2, dict):
        return {k: _fit_affine(t2[k], t3[k], t5[k], n) for k in t2}
    if isinstance(t2, slice):
        return slice(_fit_affine(t2.start, t3.start, t5.start, n), _fit_affine(t2.stop, t3.stop, t5.stop, n),
                     _fit_affine(t2.step, t3.step, t5.step, n))
    if isinstance(t2, P._Ref):
        if t2.i != t3.i or t2.i != t5.i:
            raise ValueError("program structure depends on the dynamic dim")
        return t2
    if isinstance(t2, P._Const):
        a, b, c = t2.t, t3.t, t5.t
        if a is not b and (a.shape != b.shape or a.shape != c.shape or not torch.equal(a, b)):
            raise ValueError("a captured constant depends on the dynamic dim")
        return t2
    if isinstance(t2, float):
        if t2 != t3 or t2 != t5:
            raise ValueError("dynamic dim changes a float argument")
        return t2
    return t2


def _trace_layer(layer, specs, dyn):
    from .dy2static import conversion_scope, convert_to_static
    names = [s.name for s in specs]
    fwd = layer.__dict__.get("forward")
    if isinstance(fwd, StaticFunction):
        fn = fwd._call_converted
    elif isinstance(layer, StaticFunction):
        fn = layer._call_converted
    else:
        fn = convert_to_static(layer.forward)
    with conversion_scope():
        return trace_program(fn, tuple(specs), {}, names=names, dyn_size=dyn)


class _FunctionHolder:
    """jit.save of a to_static function (reference: jit/api.py:1110-1115 saves a StaticFunction's concrete
    program): the Layer-shaped view save() works on."""
    training = False

    def __init__(self, sf):
        self._sf = sf
        self.__dict__["forward"] = sf

    def eval(self):
        pass

    def train(self):
        pass


def save(layer, path, input_spec=None, **configs):
    from ..nn.layer.layers import Layer
    if isinstance(layer, StaticFunction) and layer._instance is None:
        layer = _FunctionHolder(layer)
    elif isinstance(layer, StaticFunction):
        layer = layer._instance
    elif not isinstance(layer, Layer):
        if callable(layer):
            layer = _FunctionHolder(StaticFunction(layer))
        else:
            raise TypeError("jit.save expects a Layer or a (to_static) function")
    specs = _specs_for(layer, input_spec)
    was_training = layer.training
    layer.eval()
    try:
        dynamic = any(any(s is None or s < 0 for s in sp.shape) for sp in specs)
        if not dynamic:
            prog, feed_slots, tmpl, fetch = _trace_layer(layer, specs, None)
        else:
            traces = [_trace_layer(layer, specs, n) for n in (2, 3, 5)]
            prog, feed_slots, tmpl, fetch = traces[0]
            (p2, _, _, f2), (p3, _, _, f3), (p5, _, _, f5) = traces
            if len(p2.nodes) != len(p3.nodes) or len(p2.nodes) != len(p5.nodes) or f2 != f3 or f2 != f5:
                raise ValueError("jit.save: the program structure depends on the dynamic dim; use fixed shapes")
            for n2, n3, n5 in zip(p2.nodes, p3.nodes, p5.nodes):
                if n2.name != n3.name or n2.name != n5.name:
                    raise ValueError("jit.save: op sequence depends on the dynamic dim; use fixed shapes")
                n2.args = _fit_affine(n2.args, n3.args, n5.args)
                n2.kwargs = _fit_affine(n2.kwargs, n3.kwargs, n5.kwargs)
            prog._dyn = True
        q = _sio._prune(prog, fetch)
        _sio.write_program(path, q, fetch)
        import json
        with open(path + ".pdmodel.info", "w") as f:
            json.dump({"out": _jsonable_tmpl(tmpl)}, f)
    finally:
        if was_training:
            layer.train()


def _jsonable_tmpl(t):
    kind, v = t
    if kind == "slot":
        return ["slot", v]
    if kind in ("list", "tuple"):
        return [kind, [_jsonable_tmpl(x) for x in v]]
    if kind == "dict":
        return ["dict", {k: _jsonable_tmpl(x) for k, x in v.items()}]
    if kind == "py" and (v is None or isinstance(v, (int, float, str, bool))):
        return ["py", v]
    return ["py", None]


def _from_json_tmpl(t):
    kind, v = t
    if kind in ("list", "tuple"):
        return (kind, [_from_json_tmpl(x) for x in v])
    if kind == "dict":
        return ("dict", {k: _from_json_tmpl(x) for k, x in v.items()})
    return (kind, v)


from ..nn.layer.layers import Layer as _Layer  # noqa: E402


class TranslatedLayer(_Layer):
    """A loaded jit program as a Layer: parameters are real (fine-tunable) Parameters."""

    def __init__(self, program, fetch, out_tmpl, consts):
        super().__init__()
        self._program = program
        self._fetch = fetch
        self._out_tmpl = out_tmpl
        idx = 0
        for i, t in enumerate(program._consts):
            name = next((k for k, v in consts.items() if v is t), None)
            if name is not None and not name.startswith("__const_") and t.is_floating_point():
                p = Parameter(t, trainable=True, name=name)
                setattr(self, f"param_{idx}", p)
                program._consts[i] = p._t
                program._params[i] = p
                idx += 1
        self._plan = P.build_plan(program, fetch)
        self._feed_slots = [s for (s, _, _) in program.feeds.values()]

    def forward(self, *inputs):
        dev = inputs[0]._t.device if inputs and isinstance(inputs[0], Tensor) else torch.device("cpu")
        env = {}
        sym_n = None
        for (name, (slot, shape, dtype)), x in zip(self._program.feeds.items(), inputs):
            t = x._t if isinstance(x, Tensor) else torch.as_tensor(np.asarray(x))
            env[slot] = t
            if self._program._dyn and sym_n is None and -1 in shape:
                sym_n = int(t.shape[list(shape).index(-1)])
        consts = None
        P.run_plan(self._program, self._plan, env, dev, consts, sym_n)
        return _rebuild_out(self._out_tmpl, [env[s] for s in self._fetch])

    def program(self, method_name="forward"):
        return self._program


def load(path, **configs):
    import json
    from ..framework.place import _get_torch_device
    prog, fetch, consts = _sio.read_program(path, _get_torch_device())
    info = path + ".pdmodel.info"
    if os.path.exists(info):
        with open(info) as f:
            tmpl = _from_json_tmpl(json.load(f)["out"])
    else:
        tmpl = ("list", [("slot", i) for i in range(len(fetch))]) if len(fetch) != 1 else ("slot", 0)
    return TranslatedLayer(prog, fetch, tmpl, consts)


class TracedLayer:
    """Reference: jit TracedLayer.trace(layer, inputs) -> (outputs, traced)."""

    def __init__(self, layer, sf):
        self._layer = layer
        self._sf = sf

    @staticmethod
    def trace(layer, inputs):
        sf = StaticFunction(type(layer).forward, instance=layer)
        out = sf(*inputs)
        return out, TracedLayer(layer, sf)

    def __call__(self, *inputs):
        return self._sf(*inputs)

    def save_inference_model(self, path, feed=None, fetch=None, **kw):
        save(self._layer, path, input_spec=[InputSpec(s.shape, str(s.dtype).replace("torch.", ""))
                                            for s in [self._sf.concrete_program.program._metas[x]
                                                      for x in self._sf.concrete_program.feed_slots]])


def set_code_level(level=100, also_to_stdout=False):
    pass


def set_verbosity(level=0, also_to_stdout=False):
    pass

from . import sot  # noqa: E402,F401  (bytecode translator: paddle.jit.sot.symbolic_translate)
