"""Static-graph user API: default programs, program_guard, data, Executor, gradients, scope.

Reference: python/paddle/base/framework.py (program_guard, default_main_program), static/input.py
(data, InputSpec), base/executor.py:1247 (Executor.run), base/backward.py:1912 (append_backward),
:2404 (gradients), base/executor.py global_scope.
"""
from __future__ import annotations

import contextlib

import numpy as np
import torch

from ..framework import dtype as _dt
from ..framework.tensor import Tensor, Parameter, _wrap
from . import program as P
from ..framework.trace_hook import static_op


class _StaticMode:
    enabled = False


_static_mode = _StaticMode()
_main = P.Program()
_startup = P.Program()
_global_tracer = None


def default_main_program():
    return _main


def default_startup_program():
    return _startup


def _reset_default_programs():
    """Fresh default main / startup programs (what a new process starts with)."""
    global _main, _startup
    _main, _startup = P.Program(), P.Program()
    _retarget_tracer()


def _retarget_tracer():
    global _global_tracer
    if _global_tracer is not None:
        _global_tracer.__exit__(None, None, None)
        P._state.stack.remove(_global_tracer)
        _global_tracer = None
    if _static_mode.enabled:
        tr = P._Tracer(_main)
        st = getattr(P._state, "stack", None)
        if st is None:
            st = P._state.stack = []
        st.append(tr)
        tr.__enter__()
        _global_tracer = tr


def enable_static():
    _static_mode.enabled = True
    _retarget_tracer()


def disable_static(place=None):
    _static_mode.enabled = False
    _retarget_tracer()


@contextlib.contextmanager
def program_guard(main_program, startup_program=None):
    global _main, _startup
    old = (_main, _startup)
    _main = main_program
    if startup_program is not None:
        _startup = startup_program
    _retarget_tracer()
    try:
        yield
    finally:
        _main, _startup = old
        _retarget_tracer()


def data(name, shape, dtype=None, lod_level=0, append_batch_size=False):
    """Feed variable. Unknown dims (None / -1) are traced with a placeholder size; shape-generic code
    (reshape(-1, ...)) runs at any size, code that reads the traced size keeps it fixed.
    ``append_batch_size`` (legacy fluid.layers.data): prepend a -1 batch dimension."""
    dtype = dtype or _dt.get_default_dtype()
    if append_batch_size:
        shape = [-1] + list(shape)
    return P.placeholder(_main, name, shape, dtype)


class InputSpec:
    """Reference: python/paddle/static/input.py InputSpec."""

    def __init__(self, shape, dtype="float32", name=None, stop_gradient=False):
        self.shape = tuple(-1 if s is None else int(s) for s in shape)
        self.dtype = _dt.convert_dtype(dtype)
        self.name = name
        self.stop_gradient = stop_gradient

    @classmethod
    def from_tensor(cls, tensor, name=None):
        return cls(tensor.shape, tensor.dtype, name or getattr(tensor, "_name", None))

    @classmethod
    def from_numpy(cls, ndarray, name=None):
        return cls(ndarray.shape, str(ndarray.dtype), name)

    def batch(self, batch_size):
        """Insert ``batch_size`` in front of the shape, in place (reference input.py: returns self)."""
        if isinstance(batch_size, (list, tuple)):
            if len(batch_size) != 1:
                raise ValueError(f"Length of batch_size: {batch_size} shall be 1, but received {len(batch_size)}.")
            batch_size = batch_size[0]
        elif not isinstance(batch_size, int):
            raise TypeError(f"type(batch_size) shall be `int`, but received {type(batch_size).__name__}.")
        self.shape = (int(batch_size),) + tuple(self.shape)
        return self

    def unbatch(self):
        """Remove the first dim of the shape, in place."""
        if len(self.shape) == 0:
            raise ValueError("Not support to unbatch a InputSpec when len(shape) == 0.")
        self.shape = tuple(self.shape[1:])
        return self

    def __repr__(self):
        return (f"{type(self).__name__}(shape={self.shape}, dtype={self.dtype}, name={self.name}, "
                f"stop_gradient={self.stop_gradient})")

    def __eq__(self, o):
        return isinstance(o, InputSpec) and (self.shape, self.dtype, self.name) == (o.shape, o.dtype, o.name)

    def __hash__(self):
        return hash((self.shape, self.dtype, self.name))


def _slot_of(prog, v):
    if isinstance(v, str):
        if v in prog._names:
            return prog._names[v]
        raise KeyError(f"no variable named {v} in program")
    t = v._t if isinstance(v, Tensor) else v
    s = prog._slot_of.get(id(t))
    if s is None or prog._metas[s] is not t:
        raise KeyError("fetch target is not a variable of this program")
    return s


def append_backward(loss, parameter_list=None, no_grad_set=None, callbacks=None, checkpoints=None):
    """Returns [(param, grad_var)]; grads are computed by an autograd node at replay."""
    prog = _main
    params = parameter_list or [p for p in prog.all_parameters() if not p.stop_gradient]
    params = [p if isinstance(p, Tensor) else next(q for q in prog.all_parameters() if q.name == p) for p in params]
    grads = gradients([loss], params)
    return list(zip(params, grads))


def gradients(targets, inputs, target_gradients=None, no_grad_set=None):
    prog = P._active_program() or _main
    targets = targets if isinstance(targets, (list, tuple)) else [targets]
    inputs_l = inputs if isinstance(inputs, (list, tuple)) else [inputs]
    for x in inputs_l:
        s = prog._slot_of.get(id(x._t))
        if s is not None and s in {v[0] for v in prog.feeds.values()}:
            prog._need_grad_slots.add(s)
            prog._metas[s].requires_grad_(True)
    fn = P._grad_node_fn(len(targets), True)
    targs = tuple(prog._template(t._t) for t in targets) + tuple(prog._template(x._t) for x in inputs_l)
    with torch._C.DisableTorchFunction():
        metas = tuple(torch.empty_like(x._t, device="meta") for x in inputs_l)
    node = P.OpNode(fn, targs, {}, None, kind="grad", name="g:grad")
    node.outs = prog._out_template(metas)
    prog._append(node)
    out = [_wrap(m) for m in metas]
    return out if isinstance(inputs, (list, tuple)) else out


class Scope:
    def find_var(self, name):
        for p in list(P._PARAM_OF.values()):
            if p.name == name:
                return _ScopeVar(p)
        return None

    def var(self, name):
        return self.find_var(name)


class _ScopeVar:
    def __init__(self, p):
        self._p = p

    def get_tensor(self):
        return _LoDTensorView(self._p)


class _LoDTensorView:
    def __init__(self, p):
        self._p = p

    def __array__(self, dtype=None):
        a = self._p.numpy()
        return a if dtype is None else a.astype(dtype)

    def set(self, value, place=None):
        with torch.no_grad():
            self._p._t.copy_(torch.as_tensor(np.asarray(value)).to(self._p._t.dtype))

    def shape(self):
        return list(self._p.shape)


_scope = Scope()


def global_scope():
    return _scope


@contextlib.contextmanager
def scope_guard(scope):
    yield


class BuildStrategy:
    """Graph-build options; the fusion switches select registered program passes (distributed/passes), applied
    once to a CompiledProgram's program on its first run (reference framework/ir.py:56 apply_build_strategy)."""

    def __init__(self):
        self.fuse_elewise_add_act_ops = False
        self.fuse_bn_act_ops = False
        self.fuse_bn_add_act_ops = False
        self.fuse_gemm_epilogue = False
        self.fused_attention = False
        self.fused_feedforward = False
        self.fuse_dot_product_attention = False
        self.fuse_adamw = False
        self.fuse_all_optimizer_ops = False
        self.fuse_relu_depthwise_conv = False
        self.fuse_resunit = False
        self.enable_inplace = True
        self.memory_optimize = True
        self.fuse_all_reduce_ops = True
        self.enable_addto = False
        # reference base/executor.py:993: the new executor captures the program into a CUDA graph; here the
        # whole run (forward, backward, optimizer update) is captured into a hipGraph and replayed (_GraphRun)
        self.allow_cuda_graph_capture = False
        self.build_cuda_graph = False


class ExecutionStrategy:
    def __init__(self):
        self.num_threads = 1
        self.num_iteration_per_drop_scope = 100


# BuildStrategy switch -> pass, in application order (AMP-independent fusions first, GEMM epilogue before the
# passes that consume fused_linear nodes)
_BUILD_PASSES = (("fuse_relu_depthwise_conv", "fuse_relu_depthwise_conv"),
                 ("fuse_bn_act_ops", "fuse_bn_act"), ("fuse_bn_add_act_ops", "fuse_bn_add_act"),
                 ("fuse_resunit", "fuse_resunit"),
                 ("fuse_dot_product_attention", "fuse_dot_product_attention"),
                 ("fuse_gemm_epilogue", "fuse_gemm_epilogue"), ("fused_feedforward", "fused_feedforward"),
                 ("fused_attention", "fused_attention"), ("fuse_elewise_add_act_ops", "fuse_elewise_add_act"),
                 ("fuse_adamw", "fuse_adamw"), ("fuse_all_optimizer_ops", "fuse_optimizer"))


def apply_build_strategy(program, build_strategy):
    """Apply the passes ``build_strategy`` enables to ``program`` (in place); returns {pass: context}."""
    from ..distributed.passes import new_pass
    done = {}
    for attr, name in _BUILD_PASSES:
        if getattr(build_strategy, attr, False):
            done[name] = new_pass(name).apply(program, None)
    return done


class CompiledProgram:
    def __init__(self, program_or_graph, build_strategy=None):
        self._program = program_or_graph
        self._build_strategy = build_strategy or BuildStrategy()
        self._applied = None  # {pass name: context} once the build strategy's passes ran

    def with_data_parallel(self, loss_name=None, build_strategy=None, exec_strategy=None, places=None):
        return self


class _GraphRun:
    """One captured Executor.run of a fixed-shape program: static feed buffers, the hipGraph of plan replay +
    backward + optimizer step, and the fetch tensors it writes. Captured on the third run with these shapes
    (the first runs pick kernels, grow the allocator and create optimizer state eagerly); a run is
    replayed after copying the new feed values into the static buffers."""

    WARMUP = 2

    def __init__(self):
        self.runs = 0
        self.graph = None
        self.feeds = None
        self.fetch = None
        self.failed = None
        self.host_before = self.host_after = None  # optimizer host state around the captured step
        self.lr = None


_GRAPH_STATS = {"captured": 0, "replayed": 0}


class Executor:
    """Replays a Program: feeds -> native-scheduled op list -> fetches (+ backward/optimizer)."""

    def __init__(self, place=None):
        self.place = place
        self._graphs = {}

    def _device(self, prog):
        for p in prog.all_parameters():
            return p._t.device
        if self.place is not None:
            from ..framework.place import to_torch_device
            return to_torch_device(self.place)
        from ..framework.place import _get_torch_device
        return _get_torch_device()

    def close(self):
        pass

    def run(self, program=None, feed=None, fetch_list=None, feed_var_name="feed", fetch_var_name="fetch",
            scope=None, return_numpy=True, use_program_cache=False, use_prune=False):
        prog = program if program is not None else _main
        use_graph = False
        if isinstance(prog, CompiledProgram):
            bs = prog._build_strategy
            use_graph = bool(getattr(bs, "allow_cuda_graph_capture", False) or getattr(bs, "build_cuda_graph", False))
            if prog._applied is None and isinstance(prog._program, P.Program):
                prog._applied = apply_build_strategy(prog._program, bs)
            prog = prog._program
        from ..framework.program_desc import ProgramDescRunner
        from ..framework.pir_json import PirRunner
        from ..framework.native_interp import NativeRunner
        if isinstance(prog, (ProgramDescRunner, PirRunner, NativeRunner)):  # a reference-format model from load_inference_model
            outs = prog.run(feed or {})
            return [o.numpy() for o in outs] if return_numpy else outs
        if not prog.nodes and not prog.feeds:
            return []  # startup program: parameters are initialised eagerly at creation
        fetch_list = [] if fetch_list is None else (fetch_list if isinstance(fetch_list, (list, tuple))
                                                    else [fetch_list])
        fetch = [_slot_of(prog, v) for v in fetch_list]
        opt = prog._optimize
        keep = (opt[1],) if opt is not None else ()
        key = (tuple(fetch), keep, prog._version)
        plan = prog._plans.get(key)
        if plan is None:
            plan = P.build_plan(prog, fetch, keep)
            prog._plans[key] = plan
        dev = self._device(prog)
        nat = self._native_runner(prog, plan, fetch, dev, key) if not use_graph else None
        if nat is not None:
            try:
                outs = nat.run(self._feed(prog, feed or {}, dev))
            except RuntimeError as e:
                # it ran before (a real failure of this step), or it got far enough to change device state (BN
                # statistics, gradients, the dp all-reduce, the update): replaying it would apply that twice
                if nat.runs or not nat.replayable():
                    raise
                # an operand the native kernels reject at run time: this program keeps the Python replay
                prog._native_runners[(key, str(dev))] = None
                prog._native_reason = f"first native run failed: {e}"
            else:
                nat.runs += 1
                return [(_wrap(t).numpy() if return_numpy else _wrap(t)) for t in outs]
        if use_graph and dev.type == "cuda" and self._graph_ok(prog):
            outs = self._run_graph(prog, plan, fetch, feed or {}, dev, key)
            if outs is not None:
                return [(_wrap(t).numpy() if return_numpy else _wrap(t.clone())) for t in outs]
        env = self._feed(prog, feed or {}, dev)
        grad_on = opt is not None or any(prog.nodes[i].kind == "grad" for i in plan.order)
        from .. import amp as _amp
        with torch.set_grad_enabled(grad_on):
            sym_n = self._sym_n(prog, feed or {})
            P.run_plan(prog, plan, env, dev, sym_n=sym_n)
        if opt is not None:
            optimizer, ls = opt
            gm = getattr(prog, "_grad_merge", None)  # (k_steps, avg) from auto_parallel_gradient_merge
            k, avg = gm if gm is not None else (1, False)
            count = getattr(prog, "_gm_count", 0)
            if count % k == 0:
                optimizer.clear_grad(set_to_zero=False)
                _master_grads_clear(prog, optimizer)
            last = (count + 1) % k == 0
            # auto_parallel_data_parallel_optimization: bucket all-reduces launched from backward hooks
            red = _OverlapReducer(prog, optimizer) if last and _dp_overlap(prog) else None
            (env[ls] / k if avg else env[ls]).backward()
            _master_grads_accumulate(prog, optimizer)
            if gm is not None:
                prog._gm_count = count + 1
            if last:
                if red is not None:
                    red.finish()
                elif _master_on(prog):
                    pg = getattr(prog, "_dp_sync", None)
                    if pg is not None:  # the fp32 sums are what data parallelism averages
                        _allreduce_mean(list(getattr(prog, "_pa_main_grads", {}).values()), pg)
                else:
                    _dp_sync(prog, optimizer)
                with _master_grads_as_grads(prog, optimizer):
                    optimizer.step()
        outs = []
        for s in fetch:
            t = env[s]
            t = t.detach() if isinstance(t, torch.Tensor) else t
            outs.append(_wrap(t).numpy() if return_numpy else _wrap(t))
        return outs

    # ------------------------------------------------------------------ native training executor
    def _native_runner(self, prog, plan, fetch, dev, key):
        """The lowered program on the native executor (static/native_train.py) when FLAGS_static_native_executor
        allows it and the program lowers; the reason it did not is kept on the program (``_native_reason``)."""
        from ..framework.flags import flag
        mode = str(flag("FLAGS_static_native_executor", "auto")).lower()
        if mode in ("0", "off", "false") or (mode == "auto" and dev.type != "cuda"):
            return None
        cache = prog.__dict__.setdefault("_native_runners", {})
        k = (key, str(dev))
        if k not in cache:
            from . import native_train
            runner, reason = native_train.compile_training(prog, plan, fetch, dev, native_kernels=dev.type == "cuda")
            cache[k] = runner
            prog._native_reason = reason
        return cache[k]

    # ------------------------------------------------------------------ hipGraph execution
    @staticmethod
    def _graph_ok(prog):
        """Programs whose run is one fixed launch sequence: no guard nodes (data-dependent Python decisions),
        no dynamic dims, no gradient merge (host-side step counting)."""
        if prog._dyn or getattr(prog, "_grad_merge", None) is not None or getattr(prog, "_dp_sync", None) is not None:
            return False
        return not any(isinstance(n, P.GuardNode) for n in prog.nodes)

    def _step(self, prog, plan, env, dev):
        opt = prog._optimize
        grad_on = opt is not None or any(prog.nodes[i].kind == "grad" for i in plan.order)
        with torch.set_grad_enabled(grad_on):
            P.run_plan(prog, plan, env, dev)
        if opt is not None:
            optimizer, ls = opt
            optimizer.clear_grad(set_to_zero=False)
            env[ls].backward()
            optimizer.step()

    def _run_graph(self, prog, plan, fetch, feed, dev, key):
        sig = tuple(sorted((k, tuple(v.shape) if isinstance(v, (Tensor, torch.Tensor)) else np.shape(v))
                           for k, v in feed.items()))
        gkey = (id(prog), key, sig)
        st = self._graphs.get(gkey)
        if st is None:
            st = self._graphs[gkey] = _GraphRun()
        if st.failed:
            return None
        optimizer = prog._optimize[0] if prog._optimize is not None else None
        if optimizer is not None and not optimizer._graph_capturable():
            # the update reads host-side hyper-parameters / step counters a replay would freeze
            st.failed = f"{type(optimizer).__name__} step is not replayable from a hipGraph"
            return None
        if st.graph is not None and optimizer is not None and not optimizer._graph_replay_valid(st.lr):
            st.graph.reset()  # the learning rate baked into the captured launch changed: capture again
            st = self._graphs[gkey] = _GraphRun()
            st.runs = _GraphRun.WARMUP
        env = self._feed(prog, feed, dev)
        if st.graph is None:
            st.runs += 1
            if st.runs <= _GraphRun.WARMUP:
                return None  # eager warm-up runs (the caller continues with this env's feeds)
            from ..device.cuda.graphs import CUDAGraph
            st.feeds = {s: (t.detach().clone().requires_grad_(t.requires_grad) if t.is_floating_point() else
                            t.clone()) for s, t in env.items()}
            cap_env = dict(st.feeds)
            torch.cuda.synchronize(dev)
            g = CUDAGraph()
            before = optimizer._graph_host_state() if optimizer is not None else None
            try:
                g.capture_begin()
                try:
                    self._step(prog, plan, cap_env, dev)
                finally:
                    g.capture_end()
            except Exception as e:  # noqa: BLE001 - a host sync / allocation inside the program: run eagerly
                st.failed = repr(e)
                g.reset()
                if optimizer is not None:  # the partial capture advanced host counters no device work matched
                    optimizer._graph_restore_host_state(before)
                return None
            if optimizer is not None:
                st.host_before, st.host_after = before, optimizer._graph_host_state()
                st.lr = optimizer.get_lr()
            st.graph = g
            st.fetch = [cap_env[s] for s in fetch]
            _GRAPH_STATS["captured"] += 1
        else:
            for s, t in env.items():
                st.feeds[s].data.copy_(t, non_blocking=True) if st.feeds[s].requires_grad else \
                    st.feeds[s].copy_(t, non_blocking=True)
            if optimizer is not None:  # the capture run's host update stands for its own (first) replay
                optimizer._graph_replayed(st.host_before, st.host_after)
        st.graph.replay()
        _GRAPH_STATS["replayed"] += 1
        return [t.detach() if isinstance(t, torch.Tensor) else t for t in st.fetch]

    @staticmethod
    def _sym_n(prog, feed):
        if not prog._dyn:
            return None
        for name, (slot, shape, _) in prog.feeds.items():
            if name in feed and -1 in shape:
                v = feed[name]
                sh = v.shape if hasattr(v, "shape") else np.asarray(v).shape
                return int(sh[list(shape).index(-1)])
        return None

    @staticmethod
    def _feed(prog, feed, dev):
        env = {}
        for name, val in feed.items():
            if name not in prog.feeds:
                raise KeyError(f"feed '{name}' is not a data variable of the program")
            slot, shape, dtype = prog.feeds[name]
            if isinstance(val, Tensor):
                t = val._t
            elif isinstance(val, torch.Tensor):
                t = val
            else:
                t = torch.from_numpy(np.ascontiguousarray(np.asarray(val)))
            t = t.to(device=dev, dtype=_dt.to_torch_dtype(dtype), non_blocking=True)
            if len(shape) == t.dim():
                for a, b in zip(shape, t.shape):
                    if a >= 0 and a != b:
                        raise ValueError(f"feed '{name}' has shape {list(t.shape)}, declared {list(shape)}")
            if slot in prog._need_grad_slots and t.is_floating_point():
                t = t.detach().requires_grad_(True)
            env[slot] = t
        return env


def cpu_places(device_count=None):
    from ..framework.place import CPUPlace
    return [CPUPlace()] * (device_count or 1)


def cuda_places(device_ids=None):
    from ..framework.place import CUDAPlace
    ids = device_ids if device_ids is not None else range(max(torch.cuda.device_count(), 1))
    return [CUDAPlace(i) for i in ids]


@contextlib.contextmanager
def device_guard(device=None):
    yield


@contextlib.contextmanager
def name_scope(prefix=None):
    yield


_PRINT_COUNTS: dict = {}


@static_op
def print_tensor(x, key, first_n, message, summarize, name, show_type, show_shape, show_layout):
    """The Print op (reference: operators/print_op.cc): prints ``x`` when executed (at most first_n times per
    op) and returns it (a view). Recorded as one node of a static program, so it prints on every run."""
    if x.device.type == "meta":  # being traced
        return x.view_as(x)
    n = _PRINT_COUNTS.get(key, 0)
    if first_n < 0 or n < first_n:
        _PRINT_COUNTS[key] = n + 1
        parts = [message] if message else []
        if name:
            parts.append(f"Variable: {name}")
        if show_type:
            parts.append(f"  - dtype: {str(x.dtype).replace('torch.', '')}")
        if show_shape:
            parts.append(f"  - shape: {list(x.shape)}")
        if show_layout:
            parts.append("  - layout: NCHW")
        flat = x.detach().reshape(-1)
        vals = flat[:summarize] if summarize >= 0 else flat
        parts.append(f"  - data: {vals.float().cpu().tolist()}")
        print("\n".join(parts), flush=True)
    return x.view_as(x)


def Print(input, first_n=-1, message=None, summarize=20, print_tensor_name=True, print_tensor_type=True,
          print_tensor_shape=True, print_tensor_layout=True, print_tensor_lod=True, print_phase="both"):
    """Prints the tensor when the program runs (static: recorded as an op of the program; dygraph: now).
    Reference: python/paddle/static/nn/control_flow.py Print."""
    t = input._t if isinstance(input, Tensor) else input
    name = getattr(input, "name", None) if print_tensor_name else None
    key = f"print:{id(input)}:{message}"
    out = print_tensor(t, key, int(first_n), message, int(summarize), name, bool(print_tensor_type),
                       bool(print_tensor_shape), bool(print_tensor_layout))
    return _wrap(out) if isinstance(input, Tensor) else out


def create_global_var(shape, value, dtype, persistable=False, force_cpu=False, name=None):
    from ..tensor.creation import full
    t = full(shape, value, dtype)
    p = Parameter(t._t, trainable=False, name=name)
    return p


def create_parameter(shape, dtype, name=None, attr=None, is_bias=False, default_initializer=None):
    from .. import create_parameter as _cp
    return _cp(shape, dtype, name, attr, is_bias, default_initializer)


# ---------------------------------------------------------------------------------------------------------------
# auto_parallel_master_grad_pass: fp32 gradient accumulation for 16-bit parameters
def _master_on(prog):
    return bool(getattr(prog, "_pa_master_grad", False))


def _master_grads_clear(prog, optimizer):
    if _master_on(prog):
        prog._pa_main_grads = {}


@torch.no_grad()
def _master_grads_accumulate(prog, optimizer):
    """Each backward's 16-bit gradient is added into the parameter's fp32 main gradient and released."""
    if not _master_on(prog):
        return
    mg = prog.__dict__.setdefault("_pa_main_grads", {})
    for p in optimizer._parameter_list:
        g = p._t.grad
        if g is None or g.dtype not in (torch.bfloat16, torch.float16):
            continue
        acc = mg.get(id(p))
        if acc is None:
            mg[id(p)] = g.float()
        else:
            acc.add_(g.float())
        p._t.grad = None


@contextlib.contextmanager
def _master_grads_as_grads(prog, optimizer):
    """The optimizer step (and the data-parallel reduction before it) reads the fp32 sums, rounded once."""
    if not _master_on(prog):
        yield
        return
    mg = getattr(prog, "_pa_main_grads", {})
    with torch.no_grad():
        for p in optimizer._parameter_list:
            acc = mg.get(id(p))
            if acc is not None:
                p._t.grad = acc.to(p._t.dtype)
    try:
        yield
    finally:
        prog._pa_main_grads = {}


# ---------------------------------------------------------------------------------------------------------------
# auto_parallel_data_parallel_optimization: gradient buckets all-reduced from backward hooks
def _dp_overlap(prog):
    cfg = getattr(prog, "_pa_dp_opt", None)
    return (cfg is not None and cfg.get("overlap", True) and getattr(prog, "_dp_sync", None) is not None
            and not _master_on(prog))


DP_OVERLAP_STATS = {"launched_in_backward": 0}


class _OverlapReducer:
    """Buckets (one dtype each, ``bucket_mb``) over the parameters in reverse registration order — the order
    backward produces their gradients; a bucket's flat all-reduce starts (async, on the communicator's stream)
    from the post-accumulate hook of its last parameter, overlapping the rest of backward. finish() waits,
    averages and scatters back; buckets whose hooks never fired (unused parameters) reduce there."""

    def __init__(self, prog, optimizer):
        import torch.distributed as tdist
        self.pg = prog._dp_sync
        self.n = tdist.get_world_size(self.pg)
        cap = int(prog._pa_dp_opt["bucket_bytes"])
        params = [p for p in optimizer._parameter_list if p._t.requires_grad]
        self.buckets, self.of = [], {}
        cur, size, dt = [], 0, None
        for p in reversed(params):
            nb = p._t.numel() * p._t.element_size()
            if cur and (p._t.dtype != dt or size + nb > cap):
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nb
            dt = p._t.dtype
        if cur:
            self.buckets.append(cur)
        self.pending = [len(b) for b in self.buckets]
        self.work = [None] * len(self.buckets)
        self.flat = [None] * len(self.buckets)
        self.handles = []
        for bi, b in enumerate(self.buckets):
            for p in b:
                self.handles.append(p._t.register_post_accumulate_grad_hook(self._hook(bi)))

    def _hook(self, bi):
        def h(_t):
            self.pending[bi] -= 1
            if self.pending[bi] == 0:
                self._launch(bi)
        return h

    @torch.no_grad()
    def _launch(self, bi):
        import torch.distributed as tdist
        b = self.buckets[bi]
        if any(p._t.grad is None for p in b):
            return
        flat = torch.cat([p._t.grad.reshape(-1) for p in b])
        self.flat[bi] = flat
        self.work[bi] = tdist.all_reduce(flat, group=self.pg, async_op=True)
        DP_OVERLAP_STATS["launched_in_backward"] += 1

    @torch.no_grad()
    def finish(self):
        for h in self.handles:
            h.remove()
        rest = []
        for bi, b in enumerate(self.buckets):
            if self.work[bi] is None:
                rest.extend(p._t.grad for p in b if p._t.grad is not None)
                continue
            self.work[bi].wait()
            flat = self.flat[bi].mul_(1.0 / self.n)
            off = 0
            for p in b:
                k = p._t.numel()
                p._t.grad.copy_(flat[off:off + k].view_as(p._t.grad))
                off += k
        if rest:
            _allreduce_mean(rest, self.pg)


def _dp_sync(prog, optimizer):
    """Static collective data parallelism (fleet.distributed_optimizer(...).minimize in static mode): average the
    gradients over the program's data-parallel group — one coalesced all-reduce per dtype (reference
    raw_program_optimizer: c_allreduce_sum + scale 1 / nranks, fused by fuse_all_reduce)."""
    pg = getattr(prog, "_dp_sync", None)
    if pg is None:
        return
    _allreduce_mean([p._t.grad for p in optimizer._parameter_list if p._t.grad is not None], pg)


def _allreduce_mean(grads, pg):
    """grads <- mean over ``pg``: flat all-reduces per dtype in buckets of FLAGS_dp_bucket_mb (few, large messages
    for the xGMI rings without a second copy of every gradient); also the native executor's gradient hook."""
    import torch.distributed as tdist
    from ..framework.flags import flag
    n = tdist.get_world_size(pg)
    cap = max(1, int(flag("FLAGS_dp_bucket_mb", 128))) << 20
    by_dtype = {}
    for g in grads:
        by_dtype.setdefault(g.dtype, []).append(g)
    with torch.no_grad():
        for gs in by_dtype.values():
            bucket, size = [], 0
            for i, g in enumerate(gs):
                bucket.append(g)
                size += g.numel() * g.element_size()
                if size >= cap or i == len(gs) - 1:
                    flat = torch.cat([x.reshape(-1) for x in bucket])
                    tdist.all_reduce(flat, group=pg)
                    flat.mul_(1.0 / n)
                    off = 0
                    for x in bucket:
                        k = x.numel()
                        x.copy_(flat[off:off + k].view_as(x))
                        off += k
                    bucket, size = [], 0
