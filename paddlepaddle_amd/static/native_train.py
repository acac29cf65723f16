"""Lower a traced static training Program onto the native training executor (csrc/interpreter/train_interp.cpp,
module ``_C_train``): forward, backward and optimizer update of one Executor.run in a single C++ call.

Reference: paddle/fluid/framework/new_executor/pir_interpreter.cc (BuildInstruction :805, dependency build
:1078) and program_interpreter.cc:142,231 (instruction list + last-use GC). The reference's program carries
explicit backward and optimizer ops; here the traced forward program is lowered instruction by instruction and the
backward is the C++ autograd engine over what the instructions recorded:

  * the hot static ops (fused_linear, linear_nt, layer_norm, rms_norm, flash_attention[_qkvpacked],
    softmax_cross_entropy, conv2d on channels-last activations, batch_norm_act_nhwc) become native instructions:
    C++ autograd nodes on the hand-written MFMA / norm / attention / CE / implicit-GEMM conv / BN kernels;
  * every other op is replayed once on meta tensors under a dispatch mode that records the ATen operators it
    reached (below autograd, so CompositeImplicit ops are already decomposed): each becomes one boxed dispatcher
    call, its non-tensor arguments converted to IValues against the operator schema at lowering time;
  * the optimizer (Adam / AdamW / Momentum, one parameter group, optional global-norm clip) becomes one
    multi-tensor kernel launch over a pointer table built in C++; its state tensors are the Python optimizer's own
    accumulators, so state_dict / checkpoints see every native step.

  * collectives of the program (``c:`` comm nodes: all_reduce / broadcast / the fuse_all_reduce coalesced
    buckets) become communication instructions: issued on the executor's own HIP stream after the compute issued
    before them, with an event that the first later instruction reading what they wrote waits on, so compute that
    does not depend on a collective overlaps it (reference new_executor/interpreter/stream_analyzer.cc:44,
    dependency_builder.cc:87).

``compile_training`` returns None (with ``reason``) for programs it cannot lower — control flow, guards, gradient
merge, optimizers or clips outside the list above — and the Executor keeps the Python replay.
"""
from __future__ import annotations

import math

import torch
from torch.utils._python_dispatch import TorchDispatchMode

from . import program as P

_META = torch.device("meta")


def _module():
    try:
        from .. import _C_train
        return _C_train
    except ImportError:
        return None


def available():
    return _module() is not None


def kernel_calls():
    m = _module()
    return dict(m.kernel_calls()) if m is not None else {}


def reset_kernel_calls():
    m = _module()
    if m is not None:
        m.reset_kernel_calls()


class Unsupported(Exception):
    pass


class _Capture(TorchDispatchMode):
    """Records the ATen operators (OpOverloads) a call reaches on meta tensors."""

    def __init__(self):
        super().__init__()
        self.ops = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        out = func(*args, **kwargs)
        self.ops.append((func, args, kwargs, out))
        return out


class _NoTrace:
    """Suspend static-mode tracing (the global tracer of paddle.enable_static and any active program) while the
    lowering replays nodes on meta tensors."""

    def __enter__(self):
        from ..framework.trace_hook import _state
        self._st = getattr(_state, "stack", None)
        _state.stack = []
        self._dis = torch._C.DisableTorchFunction()
        self._dis.__enter__()
        return self

    def __exit__(self, *exc):
        from ..framework.trace_hook import _state
        self._dis.__exit__(*exc)
        _state.stack = self._st
        return False


def _arg(n, i, name, default=None):
    if i < len(n.args):
        return n.args[i]
    return n.kwargs.get(name, default)


def _const_value(t):
    """A template argument that must be a plain Python value (not a traced / captured tensor)."""
    if isinstance(t, (P._Ref, P._Const)):
        raise Unsupported("tensor where a constant attribute was expected")
    return t


class _Lowering:
    def __init__(self, prog, dev, native_kernels):
        self.prog = prog
        self.dev = dev
        self.native = native_kernels
        self.n = len(prog._metas)
        self.slot_of_id = {}     # id(meta tensor) -> slot
        self.keep = []           # every meta referenced by id (ids stay unique)
        self.instrs = []
        self.binds = {}          # slot -> real tensor (parameters, constants)
        self.const_meta = {}     # const idx -> meta stand-in
        for s, m in enumerate(prog._metas):
            if isinstance(m, torch.Tensor):
                self._register(m, s)

    def _register(self, t, s):
        self.slot_of_id[id(t)] = s
        self.keep.append(t)

    def new_slot(self):
        s = self.n
        self.n += 1
        return s

    # -------------------------------------------------------------- templates -> slots / meta values
    def _const_slot(self, c):
        t = c.t
        if c.idx in self.const_meta:
            return self.slot_of_id[id(self.const_meta[c.idx])]
        s = self.new_slot()
        self.binds[s] = t
        with torch._C.DisableTorchFunction():
            m = torch.empty(t.shape, dtype=t.dtype, device=_META).requires_grad_(t.requires_grad)
        self.const_meta[c.idx] = m
        self._register(m, s)
        return s

    def slot(self, tmpl):
        if tmpl is None:
            return -1
        if isinstance(tmpl, P._Ref):
            return tmpl.i
        if isinstance(tmpl, P._Const) and isinstance(tmpl.t, torch.Tensor):
            return self._const_slot(tmpl)
        raise Unsupported(f"operand {tmpl!r} is not a tensor")

    def meta_of(self, tmpl):
        if isinstance(tmpl, P._Ref):
            return self.prog._metas[tmpl.i]
        if isinstance(tmpl, P._Const):
            if isinstance(tmpl.t, torch.Tensor):
                self._const_slot(tmpl)
                return self.const_meta[tmpl.idx]
            return tmpl.t
        if tmpl is P._RUN_DEV:
            return _META
        if isinstance(tmpl, P._Sym):
            raise Unsupported("dynamic dims")
        if isinstance(tmpl, slice):
            return slice(self.meta_of(tmpl.start), self.meta_of(tmpl.stop), self.meta_of(tmpl.step))
        if isinstance(tmpl, list):
            return [self.meta_of(v) for v in tmpl]
        if isinstance(tmpl, tuple):
            return tuple(self.meta_of(v) for v in tmpl)
        if isinstance(tmpl, dict):
            return {k: self.meta_of(v) for k, v in tmpl.items()}
        return tmpl

    # -------------------------------------------------------------- generic ops: captured ATen operators
    def _encode(self, v, ty=None):
        if isinstance(v, torch.Tensor):
            s = self.slot_of_id.get(id(v))
            if s is None:
                if v.dim() == 0 and v.device.type == "cpu":  # a wrapped Python number: a constant operand
                    return (2, v.detach().clone())
                raise Unsupported("a tensor not produced by the program reached an ATen operator")
            return (0, s)
        if ty is not None and isinstance(v, (bool, int, float)) and isinstance(ty, torch.TensorType):
            return (2, torch.tensor(v))
        if isinstance(v, (list, tuple)) and v and all(isinstance(x, torch.Tensor) for x in v):
            return (1, [self._encode(x)[1] for x in v])
        if isinstance(v, (list, tuple)) and v and any(isinstance(x, torch.Tensor) for x in v):
            return (4, [-1 if x is None else self._encode(x)[1] for x in v])
        if isinstance(v, torch.device):
            return (3, None) if v.type == "meta" else (2, v)
        return (2, v)

    def _out_slots(self, out):
        if isinstance(out, torch.Tensor):
            s = self.new_slot()
            self._register(out, s)
            return s
        if isinstance(out, (list, tuple)):
            return [self._out_slots(o) for o in out]
        return -1

    def lower_generic(self, n):
        args = self.meta_of(n.args)
        kwargs = self.meta_of(n.kwargs)
        cap = _Capture()
        with cap:
            out = n.func(*args, **kwargs)
        for func, a, kw, o in cap.ops:
            schema = func._schema
            full = []
            for i, arg in enumerate(schema.arguments):
                if not arg.kwarg_only and i < len(a):
                    v = a[i]
                elif arg.name in kw:
                    v = kw[arg.name]
                elif arg.has_default_value():
                    v = arg.default_value
                else:
                    raise Unsupported(f"{func}: missing argument {arg.name}")
                full.append(self._encode(v, arg.type))
            if any(isinstance(r.type, torch.ListType) for r in schema.returns) and not isinstance(o, (list, tuple)):
                raise Unsupported(f"{func}: unexpected return structure")
            outs = self._out_slots(o)
            outs = outs if isinstance(outs, list) and len(schema.returns) > 1 else [outs]
            name = schema.name
            self.instrs.append(("aten", name, schema.overload_name, full, outs))
            self.keep.append(o)
        self._bind_outputs(n, out)

    def _bind_outputs(self, n, out):
        """The node's program output slots take the captured results (an alias instruction each)."""
        if n.outs is None:
            return

        def walk(tmpl, val):
            if isinstance(tmpl, P._Ref):
                if not isinstance(val, torch.Tensor):
                    raise Unsupported(f"{n.name}: non-tensor output")
                src = self.slot_of_id.get(id(val))
                if src is None:
                    raise Unsupported(f"{n.name}: output not produced by a captured operator")
                if src != tmpl.i:
                    self.instrs.append(("native", "alias", [src], [tmpl.i], [], []))
            elif isinstance(tmpl, (list, tuple)):
                if not isinstance(val, (list, tuple)) or len(val) != len(tmpl):
                    raise Unsupported(f"{n.name}: output structure")
                for t, v in zip(tmpl, val):
                    walk(t, v)
        walk(n.outs, out)

    # -------------------------------------------------------------- native hot ops
    def _native(self, kind, ins, n, ia=(), fa=()):
        if not isinstance(n.outs, P._Ref):
            raise Unsupported(f"{n.name}: expected one output")
        self.instrs.append(("native", kind, [self.slot(t) for t in ins], [n.outs.i], list(ia), list(fa)))

    def lower_native(self, n):
        """True when ``n`` became a native instruction."""
        short = n.name.rsplit(":", 1)[-1]
        m = lambda t: self.meta_of(t)  # noqa: E731
        if short == "fused_linear" and n.name.startswith("o:"):
            x, w, b = _arg(n, 0, "x"), _arg(n, 1, "w"), _arg(n, 2, "b")
            act, hook = _arg(n, 3, "act"), _arg(n, 4, "dx_hook")
            acts = {None: 0, "gelu": 1, "gelu_tanh": 1, "gelu_approximate": 1, "relu": 2}
            if hook is not None or act not in acts or m(w).dim() != 2 or (acts[act] == 1 and b is None):
                return False
            self._native("linear", [x, w, b], n, [acts[act]])
            return True
        if short == "linear_nt" and n.name.startswith("o:"):
            x, w = _arg(n, 0, "x"), _arg(n, 1, "w")
            if m(w).dim() != 2:
                return False
            self._native("linear_nt", [x, w], n)
            return True
        if short in ("layer_norm", "rms_norm") and n.name.startswith("o:paddlepaddle_amd.ops.norm"):
            rms = short == "rms_norm"
            x, w = _arg(n, 0, "x"), _arg(n, 1, "w")
            b = None if rms else _arg(n, 2, "b")
            eps = _const_value(_arg(n, 2 if rms else 3, "eps", 1e-6 if rms else 1e-5))
            for t in (w, b):
                if t is not None and m(t).numel() != m(x).shape[-1]:
                    return False
            self._native("norm", [x, w, b], n, [int(rms)], [float(eps)])
            return True
        if short == "flash_attention" and n.name.startswith("o:paddlepaddle_amd.ops.attention"):
            q, k, v = _arg(n, 0, "q"), _arg(n, 1, "k"), _arg(n, 2, "v")
            causal, scale = _const_value(_arg(n, 3, "causal", False)), _const_value(_arg(n, 4, "scale"))
            mask, p = _arg(n, 5, "mask"), _const_value(_arg(n, 6, "dropout", 0.0))
            qm = m(q)
            if mask is not None or (p and _const_value(_arg(n, 7, "training", True))) or not _attn_dims(qm, m(k), m(v)):
                return False
            D = qm.shape[-1]
            self._native("flash_attention", [q, k, v], n, [int(bool(causal))],
                         [1.0 / math.sqrt(D) if scale is None else float(scale)])
            return True
        if short == "flash_attention_qkvpacked" and n.name.startswith("o:paddlepaddle_amd.ops.attention"):
            qkv = _arg(n, 0, "qkv")
            causal, scale = _const_value(_arg(n, 1, "causal", True)), _const_value(_arg(n, 2, "scale"))
            p = _const_value(_arg(n, 3, "dropout", 0.0))
            qm = m(qkv)
            if qm.dim() != 5 or qm.shape[3] != 3 or (p and _const_value(_arg(n, 4, "training", True))):
                return False
            if qm.dtype not in (torch.bfloat16, torch.float16) or qm.shape[-1] not in (64, 128, 256):
                return False
            D = qm.shape[-1]
            self._native("flash_attention_qkvpacked", [qkv], n, [int(bool(causal))],
                         [1.0 / math.sqrt(D) if scale is None else float(scale)])
            return True
        if short == "softmax_cross_entropy" and n.name.startswith("o:"):
            lg, lb = _arg(n, 0, "logits"), _arg(n, 1, "labels")
            ig = _const_value(_arg(n, 2, "ignore_index", -100))
            lm = m(lg)
            if lm.dtype not in (torch.float32, torch.bfloat16, torch.float16) or lm.shape[-1] % 8:
                return False
            self._native("softmax_ce", [lg, lb], n, [int(ig)])
            return True
        if n.name in ("f:torch:conv2d", "f:torch.nn.functional:conv2d"):
            x, w, b = _arg(n, 0, "input"), _arg(n, 1, "weight"), _arg(n, 2, "bias")
            st, pd = _const_value(_arg(n, 3, "stride", 1)), _const_value(_arg(n, 4, "padding", 0))
            dl, gr = _const_value(_arg(n, 5, "dilation", 1)), _const_value(_arg(n, 6, "groups", 1))
            two = lambda v: (int(v), int(v)) if isinstance(v, int) else tuple(int(u) for u in v)  # noqa: E731
            if isinstance(pd, str) or m(x).dim() != 4:
                return False
            st, pd, dl = two(st), two(pd), two(dl)
            if st[0] != st[1] or dl[0] != dl[1]:
                return False
            self._native("conv2d", [x, w, b], n, [st[0], pd[0], pd[1], dl[0], int(gr)])
            return True
        if short == "batch_norm_act_nhwc" and n.name.startswith("o:paddlepaddle_amd.ops.bn"):
            x, w, b = _arg(n, 0, "x"), _arg(n, 1, "weight"), _arg(n, 2, "bias")
            rm, rv = _arg(n, 3, "running_mean"), _arg(n, 4, "running_var")
            training = _const_value(_arg(n, 5, "training", True))
            mom, eps = _const_value(_arg(n, 6, "momentum", 0.9)), _const_value(_arg(n, 7, "eps", 1e-5))
            act, res, sink = _const_value(_arg(n, 8, "act")), _arg(n, 9, "residual"), _arg(n, 10, "grad_sink")
            xm = m(x)
            if act not in (None, "relu") or sink is not None or xm.dtype != torch.bfloat16 or xm.shape[-1] % 8:
                return False
            for t in (w, b, rm, rv):
                if t is not None and m(t).dtype != torch.float32:
                    return False
            self._native("batch_norm_act", [x, w, b, rm, rv, res], n, [int(bool(training)), int(act == "relu")],
                         [float(mom), float(eps)])
            return True
        return False


def _attn_dims(q, k, v):
    if q.dim() != 4 or k.dim() != 4 or v.dim() != 4 or q.dtype not in (torch.bfloat16, torch.float16):
        return False
    D = q.shape[-1]
    return D in (64, 128, 256) and k.shape[-1] == D and v.shape[-1] == D and q.shape[2] % k.shape[2] == 0 and \
        k.dtype == q.dtype and v.dtype == q.dtype


# ------------------------------------------------------------------------------------------------ optimizer
def _optimizer_spec(opt):
    """(kind, params, per-param tensors, clip_norm, scalars_fn) for the native update, or a reason string."""
    from ..optimizer.adam import Adam
    from ..optimizer.others import Momentum
    from ..nn.clip import ClipGradByGlobalNorm
    groups = opt._param_groups
    if len(groups) != 1:
        return "more than one parameter group"
    group = groups[0]
    params = [p for p in group["params"] if getattr(p, "trainable", True) and not p.stop_gradient]
    if not params:
        return "no trainable parameters"
    clip = opt._grad_clip
    if clip is not None and not (isinstance(clip, ClipGradByGlobalNorm) and all(getattr(p, "need_clip", True)
                                                                                 for p in params)):
        return f"gradient clip {type(clip).__name__}"
    clip_norm = float(clip.clip_norm) if clip is not None else 0.0
    masters = [opt._master(p) for p in params]
    lr_mult = [float(p.optimize_attr.get("learning_rate", 1.0)) if hasattr(p, "optimize_attr") else 1.0
               for p in params]
    for p in params:
        if p._t.dtype != torch.float32 and opt._master(p) is None:
            return "low-precision parameters without master weights"
    if isinstance(opt, Adam):
        if opt._amsgrad:
            return "amsgrad"
        if not opt._decoupled and opt._has_l2(group, params):
            return "Adam with L2 regularization"
        m1 = [opt._acc("moment1", p) for p in params]
        m2 = [opt._acc("moment2", p) for p in params]
        coeff = [float(opt._coeff_for(group, p)) for p in params]

        def scalars():
            b1, b2, eps = opt._hyper(group)
            steps = []
            for p in params:
                s = opt._param_step.get(id(p), 0) + 1
                opt._param_step[id(p)] = s
                steps.append(s)
            if any(s != steps[0] for s in steps):
                raise RuntimeError("native train executor: parameters at different Adam steps")
            st = steps[0]
            opt._last_step = st
            return [opt._group_lr(group), b1, b2, eps, 1 - b1 ** st, 1 - b2 ** st]
        return "adam", params, masters, m1, m2, coeff, lr_mult, clip_norm, scalars
    if isinstance(opt, Momentum):
        coeff = []
        for p in params:
            reg = opt._regularizer_for(p, group)
            if reg is not None and type(reg).__name__ != "L2Decay":
                return f"momentum with {type(reg).__name__}"
            coeff.append(float(reg._coeff) if reg is not None else 0.0)
        vel = [opt._acc("velocity", p) for p in params]

        def scalars():
            return [opt._group_lr(group, None), float(group.get("momentum", opt._momentum)), float(opt._rescale),
                    float(bool(opt._nesterov))]
        return "momentum", params, masters, vel, vel, coeff, lr_mult, clip_norm, scalars
    return f"optimizer {type(opt).__name__}"


class NativeTrainRunner:
    """One lowered program: ``run(env_feeds)`` -> fetched tensors (the optimizer updated in place)."""

    def __init__(self, tp, feed_slots, fetch, opt, scalars_fn, clip_norm, need_grad_slots, lowering):
        self.tp = tp
        self.feed_slots = feed_slots
        self.fetch = fetch
        self.opt = opt
        self.scalars_fn = scalars_fn
        self.clip_norm = clip_norm
        self.need_grad = need_grad_slots
        self.num_instructions = tp.num_instructions
        self.num_native = tp.num_native
        self.num_comm = tp.num_comm
        self._lowering = lowering  # keeps bound tensors alive
        self.runs = 0

    def replayable(self):
        """After run() raised: True when the step may be replayed by another executor without applying device
        state twice — it stopped in the forward (no backward, gradient all-reduce or update ran) and neither a
        completed instruction nor the failing one writes an input in place (BN running statistics, in-place ATen
        ops)."""
        if self.tp.phase != 0:
            return False
        upto = min(self.tp.done + 1, len(self._lowering.instrs))
        return not any(_mutates(ins) for ins in self._lowering.instrs[:upto])

    def run(self, env):
        feeds = []
        for s, t in env.items():
            if s in self.need_grad and t.is_floating_point() and not t.requires_grad:
                t = t.detach().requires_grad_(True)
            feeds.append((s, t))
        train = self.opt is not None
        snap = (self.opt._step_count, dict(getattr(self.opt, "_param_step", {}))) if train else None
        try:
            return self._run(feeds, train)
        except Exception:
            if snap is not None:  # host bookkeeping back to before this step (the Executor may replay it in Python)
                self.opt._step_count = snap[0]
                if hasattr(self.opt, "_param_step"):
                    self.opt._param_step.clear()
                    self.opt._param_step.update(snap[1])
            raise

    def _run(self, feeds, train):
        scalars = []
        if train and self.scalars_fn is not None:
            from ..ops.linear import bump_weight_epoch
            bump_weight_epoch()
            self.opt._step_count += 1
            scalars = [self.scalars_fn()]
        elif train:
            self.opt.clear_grad(set_to_zero=False)
        outs = self.tp.run(feeds, train, scalars, self.clip_norm)
        if train and self.scalars_fn is None:  # forward + backward native, update by the Python optimizer
            pg = getattr(self, "dp_pg", None)
            if pg is not None:  # static collective DP (the native update runs it as the executor's gradient hook)
                from .executor import _allreduce_mean
                _allreduce_mean([p._t.grad for p in self.opt._parameter_list if p._t.grad is not None], pg)
            self.opt.step()
        return outs


def _mutates(ins):
    """Whether a lowered instruction writes device state that outlives the step."""
    if ins[0] == "comm":
        return True  # a collective: other ranks took part, it cannot be issued again alone
    if ins[0] == "native":
        return ins[1] == "batch_norm_act"
    name, overload = ins[1], ins[2]
    try:
        op = getattr(getattr(torch.ops.aten, name.split("::")[-1]), overload or "default")
    except AttributeError:
        return True  # unknown: assume it does
    return any(a.alias_info is not None and a.alias_info.is_write for a in op._schema.arguments)


def compile_training(prog, plan, fetch, dev, native_kernels=True):
    """-> (NativeTrainRunner, None) or (None, reason)."""
    m = _module()
    if m is None:
        return None, "_C_train not built"
    if prog._dyn or getattr(prog, "_grad_merge", None) is not None:
        return None, "dynamic dims / gradient merge"
    opt_entry = prog._optimize
    low = _Lowering(prog, dev, native_kernels)
    try:
        with _NoTrace():
            _lower_all(low, plan, native_kernels)
    except Unsupported as e:
        return None, str(e)
    except Exception as e:  # noqa: BLE001 - anything the capture cannot replay on meta tensors
        return None, f"lowering failed: {type(e).__name__}: {e}"
    return _build(m, low, prog, fetch, dev, native_kernels, opt_entry)


def _lower_all(low, plan, native_kernels):
    if True:
        for i in plan.order:
            n = plan.nodes[i]
            if isinstance(n, (P.CFNode, P.GuardNode)) or n.kind in ("grad", "guard"):
                raise Unsupported(f"{type(n).__name__} {n.name}")
            if n.kind == "comm":  # a collective: an instruction on the executor's communication stream
                if not n.args or not all(isinstance(a, P._Ref) for a in n.args) or n.kwargs:
                    raise Unsupported(f"collective {n.name} with non-tensor operands")
                low.instrs.append(("comm", n.func, [a.i for a in n.args], n.name))
                continue
            if native_kernels and low.lower_native(n):
                continue
            low.lower_generic(n)


def _build(m, low, prog, fetch, dev, native_kernels, opt_entry):
    tp = m.TrainProgram(low.n, str(dev))
    try:
        for ins in low.instrs:
            if ins[0] == "aten":
                tp.add_aten(f"{ins[1]}", ins[2], [tuple(a) for a in ins[3]], ins[4])
            elif ins[0] == "comm":
                tp.add_comm(ins[1], ins[2], ins[3])
            else:
                tp.add_native(ins[1], ins[2], ins[3], ins[4], ins[5])
    except Exception as e:  # noqa: BLE001 - an operator argument the schema conversion rejects
        return None, f"instruction build failed: {type(e).__name__}: {e}"
    for s, t in low.binds.items():
        tp.bind(s, t)
    scalars_fn, clip_norm, opt = None, 0.0, None
    if opt_entry is not None:
        opt, loss_slot = opt_entry
        tp.set_loss(loss_slot)
        spec = _optimizer_spec(opt) if native_kernels and dev.type == "cuda" else "optimizer runs in Python"
        if not isinstance(spec, str):
            kind, params, masters, m1, m2, coeff, lr_mult, clip_norm, scalars_fn = spec
            bound = {id(t) for t in low.binds.values()}
            if any(id(p._t) not in bound for p in params):
                # a parameter the program never reads would get no gradient: keep the Python update
                scalars_fn, clip_norm = None, 0.0
            else:
                tp.add_optimizer(kind, [p._t for p in params], [mm if mm is not None else p._t
                                                                 for p, mm in zip(params, masters)],
                                 [int(mm is not None) for mm in masters], m1, m2, coeff, lr_mult)
    pg = getattr(prog, "_dp_sync", None)
    if pg is not None:  # static collective DP: average the gradients before the update
        from . import executor as _ex
        tp.set_grad_hook(lambda grads: _ex._allreduce_mean(grads, pg))
    tp.finalize(list(fetch))
    feed_slots = {name: v[0] for name, v in prog.feeds.items()}
    runner = NativeTrainRunner(tp, feed_slots, fetch, opt, scalars_fn, clip_norm, set(prog._need_grad_slots), low)
    runner.dp_pg = pg
    return runner, None
