"""Registered program passes over the traced static Program (static/program.py).

* ``fuse_gemm_epilogue`` (reference passes/cpp_pass.py FuseGemmEpiloguePass, a C++ IR fusion there):
  ``matmul(x, W) + b`` and ``fused_linear(x, W, b)`` followed by relu / gelu become ONE
  ``ops.linear.fused_linear(x, W, b, act)`` node, so replay runs the hand-written MFMA GEMM with the bias +
  GELU epilogue (ops/linear.py _LinearBiasGeluFn) instead of three kernels and two [M, N] round trips.
* ``dead_code_elimination``: drops nodes that no fetch, the optimizer loss, a guard, a collective or an
  in-place write to a parameter depends on (the Executor already prunes per fetch list; this shrinks the
  program itself, e.g. before save_inference_model).
* ``auto_parallel_amp`` / ``auto_parallel_fp16`` (reference auto_parallel_amp.py / auto_parallel_fp16.py):
  insert casts so white-list ops (GEMMs, convolutions, attention) run in bf16/fp16 and black-list ops
  (softmax, norms, losses, reductions) in fp32; parameters stay fp32 masters. Output dtypes are propagated
  by re-running each op on meta tensors, the same way the program was traced.
* ``auto_parallel_gradient_merge`` (reference auto_parallel_gradient_merge.py): the Executor accumulates
  gradients over ``k_steps`` runs and applies the optimizer on the last one (``avg`` scales by 1/k).
* ``auto_parallel_recompute``: ops between consecutive checkpoints become recompute segments (node.rc), run
  checkpointed by the static auto-parallel engine; ``allreduce_matmul_grad_overlapping`` /
  ``auto_parallel_sharding`` mark the program for the engine's partition-time TP dX overlap and ZeRO-1/2.
* ``fuse_bn_act`` / ``fuse_bn_add_act`` / ``fuse_elewise_add_act``: batch_norm (+ residual) + relu -> one
  batch_norm_act_nhwc node; bias add + tanh GELU -> one bias_gelu node.
"""
from __future__ import annotations

import torch

from .pass_base import PassBase, PassType, register_pass
from ...static import program as P

__all__ = ["FuseGemmEpiloguePass", "DeadCodeEliminationPass", "AMPPass", "FP16Pass", "GradientMergePass",
           "FuseSiblingLinearsPass", "FuseRMSNormResidualPass",
           "RecomputePass", "AllreduceMatmulGradOverlappingPass", "ShardingPass", "FuseBNActPass",
           "FuseBNAddActPass", "FuseElewiseAddActPass", "FuseAllReducePass", "ReplaceWithParallelCrossEntropyPass",
           "CEmbeddingPass"]

_RELU = {"f:torch.nn.functional:relu", "f:torch:relu", "m:relu"}
_GELU = {"o:paddlepaddle_amd.ops.activation:gelu", "f:torch.nn.functional:gelu"}
_ADD = {"m:add", "f:torch:add", "m:__add__", "m:__radd__"}
_MATMUL = {"f:torch:matmul", "m:matmul", "f:torch:mm", "m:mm", "m:__matmul__"}
_LINEAR = "o:paddlepaddle_amd.ops.linear:fused_linear"



def _keep_rc(node, src):
    """A rewritten node stays in the recompute segment of the node it replaces."""
    node.rc = getattr(src, "rc", None)
    return node

def _slot(t):
    return t.i if isinstance(t, P._Ref) else None


def _vars_to_slots(prog, vs):
    out = set()
    for v in vs or ():
        if isinstance(v, str):
            if v in prog._names:
                out.add(prog._names[v])
            continue
        t = getattr(v, "_t", v)
        s = prog._slot_of.get(id(t))
        if s is not None:
            out.add(s)
    return out


def _protected(prog, attrs_fetch):
    keep = _vars_to_slots(prog, attrs_fetch)
    keep |= set(prog._names.values())
    if prog._optimize is not None:
        keep.add(prog._optimize[1])
    return keep


def _use_counts(nodes):
    cnt = {}
    for n in nodes:
        for s in P._node_reads(n):
            cnt[s] = cnt.get(s, 0) + 1
    return cnt


def _shape_of(prog, t):
    if isinstance(t, P._Ref):
        return tuple(prog._metas[t.i].shape)
    if isinstance(t, P._Const):
        return tuple(t.t.shape)
    return None


def _act_of(n):
    """fused_linear activation name for an activation node, or None."""
    if n.name in _RELU and len(n.args) == 1 and not n.kwargs.get("inplace", False):
        return "relu"
    if n.name in _GELU:
        approx = n.args[1] if len(n.args) > 1 else n.kwargs.get("approximate", False)
        if isinstance(approx, str):
            approx = approx == "tanh"
        return "gelu" if approx else "gelu_erf"
    return None


@register_pass("fuse_gemm_epilogue")
class FuseGemmEpiloguePass(PassBase):
    _after = ("auto_parallel_amp", "auto_parallel_fp16")

    def _type(self):
        return PassType.FUSION_OPT

    def _apply_single_impl(self, prog, startup, context):
        lin = P._resolve(_LINEAR)
        keep = _protected(prog, self.get_attr("fetch_vars"))
        nodes = prog.nodes
        fused = 0
        changed = True
        while changed:
            changed = False
            uses = _use_counts(nodes)
            producer = {}
            for i, n in enumerate(nodes):
                if not isinstance(n, P.CFNode):
                    for s in P._node_writes(n):
                        producer.setdefault(s, i)

            def single(s):
                return s is not None and uses.get(s, 0) == 1 and s not in keep

            for j, n in enumerate(nodes):
                if isinstance(n, P.CFNode) or n.kind == "guard":
                    continue
                # matmul(x, W) + b  ->  fused_linear(x, W, b)
                if n.name in _ADD and len(n.args) == 2 and not n.kwargs:
                    a, b = n.args
                    if _slot(a) is None or not isinstance(n.outs, P._Ref):
                        a, b = b, a
                    i = producer.get(_slot(a))
                    if i is None or not single(_slot(a)):
                        continue
                    m = nodes[i]
                    if m.name not in _MATMUL or len(m.args) != 2 or m.kwargs:
                        continue
                    ws, bs = _shape_of(prog, m.args[1]), _shape_of(prog, b)
                    if ws is None or bs is None or len(ws) != 2 or bs != (ws[1],):
                        continue
                    nodes[j] = _keep_rc(P.OpNode(lin, (m.args[0], m.args[1], b), {}, n.outs, "op", _LINEAR), m)
                    del nodes[i]
                    fused += 1
                    changed = True
                    break
                # fused_linear(x, W, b) -> act  ->  fused_linear(x, W, b, act)
                act = _act_of(n)
                if act is not None:
                    s = _slot(n.args[0])
                    i = producer.get(s)
                    if i is None or not single(s):
                        continue
                    m = nodes[i]
                    if m.name != _LINEAR or m.kwargs or len(m.args) != 3 or not isinstance(m.outs, P._Ref):
                        continue
                    nodes[j] = _keep_rc(P.OpNode(lin, tuple(m.args) + (act,), {}, n.outs, "op", _LINEAR), m)
                    del nodes[i]
                    fused += 1
                    changed = True
                    break
        context.set_attr("fuse_gemm_epilogue.fused", context.get_attr("fuse_gemm_epilogue.fused", 0) + fused)


@register_pass("dead_code_elimination")
class DeadCodeEliminationPass(PassBase):
    def _apply_single_impl(self, prog, startup, context):
        need = _vars_to_slots(prog, self.get_attr("fetch_vars"))
        if not need:
            need = set(prog._names.values())
        if prog._optimize is not None:
            need.add(prog._optimize[1])
        consts_written = lambda n: P._is_inplace(n) and n.args and isinstance(n.args[0], P._Const)  # noqa: E731
        live = []
        for n in reversed(prog.nodes):
            w = P._node_writes(n)
            if (w & need or isinstance(n, P.CFNode) or n.kind in ("guard", "comm", "grad")
                    or consts_written(n)):
                live.append(n)
                need |= P._node_reads(n)
        removed = len(prog.nodes) - len(live)
        prog.nodes[:] = live[::-1]
        context.set_attr("dead_code_elimination.removed", removed)


_WHITE = {"f:torch:matmul", "m:matmul", "f:torch:mm", "m:mm", "f:torch:bmm", "f:torch:addmm", "m:__matmul__",
          "f:torch.nn.functional:linear", "f:torch.nn.functional:conv1d", "f:torch.nn.functional:conv2d",
          "f:torch.nn.functional:conv3d", "f:torch.nn.functional:scaled_dot_product_attention", _LINEAR,
          "f:torch:einsum"}
_BLACK = {"f:torch:softmax", "m:softmax", "f:torch.nn.functional:softmax", "f:torch.nn.functional:log_softmax",
          "f:torch.nn.functional:layer_norm", "f:torch.nn.functional:batch_norm", "f:torch.nn.functional:group_norm",
          "f:torch.nn.functional:cross_entropy", "f:torch.nn.functional:nll_loss", "f:torch:exp", "m:exp",
          "f:torch:log", "m:log", "m:mean", "f:torch:mean", "m:sum", "f:torch:sum", "f:torch:logsumexp",
          "f:torch.nn.functional:mse_loss", "f:torch:pow", "m:pow", "f:torch:sqrt", "f:torch:rsqrt"}


def _is_float(t):
    return isinstance(t, torch.Tensor) and t.is_floating_point()


@register_pass("auto_parallel_amp")
class AMPPass(PassBase):
    """attrs: dtype ('bfloat16' | 'float16'), level ('o1' | 'o2'), custom_white_list, custom_black_list
    (op names as in the program listing, e.g. 'f:torch:matmul', or bare 'matmul')."""

    def _type(self):
        return PassType.CALC_OPT

    def _check_self(self):
        return str(self.get_attr("level", "o1")).lower() in ("o1", "o2")

    def _lists(self):
        def norm(xs):
            return {x for x in xs or ()}
        white = set(_WHITE) | norm(self.get_attr("custom_white_list"))
        black = (set(_BLACK) | norm(self.get_attr("custom_black_list"))) - norm(self.get_attr("custom_white_list"))
        white -= norm(self.get_attr("custom_black_list"))
        return white, black

    @staticmethod
    def _listed(name, lst):
        return name in lst or name.rsplit(":", 1)[-1] in lst

    def _apply_single_impl(self, prog, startup, context):
        if any(isinstance(n, P.CFNode) for n in prog.nodes) or prog._dyn:
            raise NotImplementedError("auto_parallel_amp: programs with control-flow blocks or dynamic dims "
                                      "are not rewritten; use paddle.amp.auto_cast while building them")
        from ...framework import dtype as _dt
        low = _dt.to_torch_dtype(self.get_attr("dtype", "bfloat16"))
        o2 = str(self.get_attr("level", "o1")).lower() == "o2"
        white, black = self._lists()
        meta_dev = torch.device("meta")
        env = dict(enumerate(prog._metas))  # slot -> meta with the dtype it has after the rewrite
        consts = [c.detach().to(meta_dev) if isinstance(c, torch.Tensor) else c for c in prog._consts]
        new_nodes, casts = [], 0
        to = torch.Tensor.to

        def cast_arg(a, dt):
            nonlocal casts
            if isinstance(a, (list, tuple)):
                return type(a)(cast_arg(v, dt) for v in a)
            if not isinstance(a, (P._Ref, P._Const)):
                return a
            m = env[a.i] if isinstance(a, P._Ref) else consts[a.idx]
            if not _is_float(m) or m.dtype == dt or m.dtype == torch.float64:
                return a
            with torch._C.DisableTorchFunction():
                cm = torch.empty(m.shape, dtype=dt, device=meta_dev)
            s = prog._new_slot(cm)
            env[s] = cm
            new_nodes.append(_keep_rc(P.OpNode(to, (a, dt), {}, P._Ref(s), "torch", "m:to"), cur[0]))
            casts += 1
            return P._Ref(s)

        cur = [None]
        for n in prog.nodes:
            cur[0] = n
            if n.kind in ("op", "torch") and n.outs is not None:
                if self._listed(n.name, black):
                    n.args = cast_arg(n.args, torch.float32)
                elif self._listed(n.name, white) or o2:
                    n.args = cast_arg(n.args, low)
            new_nodes.append(n)
            if n.outs is not None and n.kind in ("op", "torch"):
                with torch._C.DisableTorchFunction(), torch.no_grad():
                    out = n.func(*P._materialize(n.args, env, consts, meta_dev),
                                 **P._materialize(n.kwargs, env, consts, meta_dev))
                P._assign(n.outs, out, env)
        prog.nodes[:] = new_nodes
        context.set_attr("auto_parallel_amp.casts", casts)


@register_pass("auto_parallel_fp16")
class FP16Pass(AMPPass):
    """The reference's pure-fp16 (O2) pass: every op that is not black-listed runs in the low dtype."""

    def _apply_single_impl(self, prog, startup, context):
        self._attrs.setdefault("level", "o2")
        self._attrs.setdefault("dtype", "float16")
        super()._apply_single_impl(prog, startup, context)


@register_pass("auto_parallel_gradient_merge")
class GradientMergePass(PassBase):
    def _type(self):
        return PassType.CALC_OPT

    def _check_self(self):
        return int(self.get_attr("k_steps", 1)) >= 1

    def _apply_single_impl(self, prog, startup, context):
        if prog._optimize is None:
            raise ValueError("auto_parallel_gradient_merge needs a program with optimizer.minimize(loss)")
        prog._grad_merge = (int(self.get_attr("k_steps", 1)), bool(self.get_attr("avg", True)))
        prog._gm_count = 0


# ------------------------------------------------------------------------------------------------------------------
_MULTI = "o:paddlepaddle_amd.ops.linear:multi_linear"


@register_pass("fuse_sibling_linears")
class FuseSiblingLinearsPass(PassBase):
    """Sibling linears -> one ``ops.linear.multi_linear`` node (reference: fuse_attention_ffn_qkv_pass,
    auto_parallel/static/engine.py:675, which concatenates the q / k / v and gate / up weights into new fused
    parameters). Here every ``fused_linear(x, W_i)`` (no bias, no activation) that reads the same input x becomes
    ONE node computing all outputs with an N-segmented GEMM and, in backward, the input gradient with one
    K-segmented GEMM — the parameters stay separate, so sharding, checkpoints and optimizer state are untouched.

    Attributes: ``weights`` (optional set of slots the W_i must belong to: the parameters), ``group_key`` (optional
    callable slot -> key; only weights with equal keys fuse, e.g. their distributed placements), ``max_group``
    (default 4: the segment limit of the GEMM)."""

    def _type(self):
        return PassType.FUSION_OPT

    def _apply_single_impl(self, prog, startup, context):
        ml = P._resolve(_MULTI)
        weights = self.get_attr("weights")
        key_of = self.get_attr("group_key") or (lambda s: None)
        max_group = int(self.get_attr("max_group", 4))
        nodes = prog.nodes
        producer = {}
        for i, n in enumerate(nodes):
            if not isinstance(n, P.CFNode):
                for s in P._node_writes(n):
                    producer.setdefault(s, i)
        groups = {}
        for i, n in enumerate(nodes):
            if isinstance(n, P.CFNode) or n.kind == "guard" or n.name != _LINEAR or n.kwargs:
                continue
            args = tuple(n.args)
            if len(args) > 2 and any(a is not None for a in args[2:]):
                continue  # bias / activation / hooks: keep the plain fused_linear
            x = _slot(args[0]) if args else None
            warg = args[1] if len(args) > 1 else None
            if x is None or not isinstance(n.outs, P._Ref):
                continue
            if isinstance(warg, P._Ref):  # a traced weight (the auto-parallel engine's parameter slots)
                w, wm = warg.i, prog._metas[warg.i]
                if weights is not None and w not in weights:
                    continue
                key = key_of(w)
            elif isinstance(warg, P._Const):  # a static-graph parameter captured as a program constant
                w, wm, key = None, warg.t, None
            else:
                continue
            if wm.dim() != 2:
                continue
            groups.setdefault((x, wm.shape[0], wm.dtype, key), []).append(i)
        fused = 0
        dead = set()
        for (x, _, _, _), idxs in groups.items():
            for c in range(0, len(idxs), max_group):
                chunk = idxs[c:c + max_group]
                if len(chunk) < 2:
                    continue
                first = chunk[0]
                ws = [nodes[i].args[1] for i in chunk]
                # every weight must exist where the first linear runs (parameters do; a derived weight must be
                # produced before it)
                if any(_slot(w) is not None and producer.get(_slot(w), -1) > first for w in ws):
                    continue
                outs = [nodes[i].outs for i in chunk]
                nodes[first] = _keep_rc(P.OpNode(ml, (nodes[first].args[0], list(ws)), {}, outs, "op", _MULTI), nodes[first])
                dead.update(chunk[1:])
                fused += len(chunk)
        if dead:
            prog.nodes[:] = [n for k, n in enumerate(nodes) if k not in dead]
        context.set_attr("fuse_sibling_linears.fused", context.get_attr("fuse_sibling_linears.fused", 0) + fused)


# the reference's name for the same rewrite
PassBase._REGISTERED_PASSES["fuse_attention_ffn_qkv"] = FuseSiblingLinearsPass

_RMS = "o:paddlepaddle_amd.ops.norm:rms_norm"
_RMS_RES = "o:paddlepaddle_amd.ops.norm:rms_norm_residual"


@register_pass("fuse_rms_norm_residual")
class FuseRMSNormResidualPass(PassBase):
    """Pre-norm residual blocks: ``h = rms_norm(x, w)`` where x also feeds a residual ``add`` becomes
    ``(r, h) = rms_norm_residual(x, w)`` with the add reading r: on the HIP path the residual branch's gradient
    is summed into dx inside the RMSNorm backward kernel (pa_rms_norm_bwd_res) instead of autograd's separate
    bf16 accumulation add — the op-level form of the fusion models/llama.py applies in its norm layers."""

    def _type(self):
        return PassType.FUSION_OPT

    def _apply_single_impl(self, prog, startup, context):
        rr = P._resolve(_RMS_RES)
        nodes = prog.nodes
        readers = {}
        for i, n in enumerate(nodes):
            if isinstance(n, P.CFNode):
                continue
            for s in P._node_reads(n):
                readers.setdefault(s, []).append(i)
        fused = 0
        for i, n in enumerate(list(nodes)):
            if isinstance(n, P.CFNode) or n.name != _RMS or n.kwargs or not isinstance(n.outs, P._Ref):
                continue
            x = _slot(n.args[0]) if n.args else None
            if x is None:
                continue
            others = [j for j in readers.get(x, []) if j != i]
            adds = [j for j in others if nodes[j].name in _ADD and not nodes[j].kwargs and j > i
                    and any(_slot(a) == x for a in nodes[j].args)]
            if len(others) != 1 or len(adds) != 1:
                continue  # x must feed exactly this norm and one residual add
            j = adds[0]
            m = prog._metas[x]
            with torch._C.DisableTorchFunction():
                r = prog._new_slot(torch.empty(tuple(m.shape), dtype=m.dtype, device="meta")
                                   .requires_grad_(m.requires_grad))
            nodes[i] = _keep_rc(P.OpNode(rr, tuple(n.args), {}, (P._Ref(r), n.outs), "op", _RMS_RES), n)
            a = nodes[j]
            nodes[j] = _keep_rc(P.OpNode(a.func, tuple(P._Ref(r) if _slot(v) == x else v for v in a.args), {},
                                         a.outs, a.kind, a.name), a)
            fused += 1
        context.set_attr("fuse_rms_norm_residual.fused", context.get_attr("fuse_rms_norm_residual.fused", 0) + fused)


# ------------------------------------------------------------------------------------------------------------------
@register_pass("auto_parallel_recompute")
class RecomputePass(PassBase):
    """Activation recompute by checkpoints (reference: distributed/passes/auto_parallel_recompute.py): the ops
    between consecutive ``checkpoints`` (value slots, or names the program knows) become recompute segments — the
    static auto-parallel engine runs each as a checkpointed region whose activations are rebuilt in backward
    (``strategy.recompute``). Without checkpoints the segments traced from ``recompute`` scopes are kept.
    ``no_recompute_segments``: segment indices to leave alone. Ops that already carry a segment keep it."""

    def _type(self):
        return PassType.CALC_OPT

    def _apply_single_impl(self, prog, startup, context):
        cps = self.get_attr("checkpoints") or []
        skip = set(int(i) for i in (self.get_attr("no_recompute_segments") or []))
        marks = set(c for c in cps if isinstance(c, int)) | _vars_to_slots(
            prog, [c for c in cps if not isinstance(c, int)])
        segs = 0
        if marks:
            base = next(prog._rc_ids) * 100000
            seg, cur = 0, []
            for n in prog.nodes:
                if isinstance(n, (P.CFNode, P.GuardNode)):
                    continue
                if n.rc is None and seg not in skip:
                    n.rc = base + seg
                    cur.append(n)
                if P._node_writes(n) & marks:
                    segs += bool(cur)
                    seg, cur = seg + 1, []
            for n in cur:  # the ops after the last checkpoint (the loss) are not recomputed
                n.rc = None
        else:
            segs = len(set(n.rc for n in prog.nodes if getattr(n, "rc", None) is not None))
        prog._pa_recompute = True
        context.set_attr("auto_parallel_recompute.segments", segs)


@register_pass("allreduce_matmul_grad_overlapping")
class AllreduceMatmulGradOverlappingPass(PassBase):
    """Reference: distributed/passes/allreduce_matmul_grad_overlapping.py — the tensor-parallel all-reduce of a
    column-parallel linear's input gradient overlaps its weight-gradient GEMM. The partitioned per-rank program
    only exists inside the static engine, so the pass marks the program and the engine folds each
    ``copy_to_parallel -> fused_linear`` pair into the linear's asynchronous dX hook at partition time
    (static_engine._overlap_tp_dx_allreduce; also selected by strategy.mp_optimization)."""

    def _type(self):
        return PassType.COMM_OPT

    def _apply_single_impl(self, prog, startup, context):
        prog._pa_tp_overlap = True


@register_pass("auto_parallel_sharding")
class ShardingPass(PassBase):
    """Reference: distributed/passes/auto_parallel_sharding.py — optimizer-state sharding over a data-parallel
    mesh dim. ``stage`` 1 / 2 / 3 and ``sharding_mesh_dim`` (default "dp") are recorded on the program; the engine
    flattens the parameters per placement group, reduce-scatters the accumulated gradients once per step, updates
    this rank's shards and all-gathers them (static_engine._zero_*); at stage 3 only the shards stay resident
    between steps (gathered when a step starts, released after its update)."""

    def _type(self):
        return PassType.PARALLEL_OPT

    def _check_self(self):
        return int(self.get_attr("stage", 1)) in (1, 2, 3)

    def _apply_single_impl(self, prog, startup, context):
        prog._pa_sharding = {"stage": int(self.get_attr("stage", 1)),
                             "dim": self.get_attr("sharding_mesh_dim", "dp")}


# ------------------------------------------------------------------------------------------------------------------
_BN = "o:paddlepaddle_amd.ops.bn:batch_norm_act_nhwc"
_BIAS_GELU = "o:paddlepaddle_amd.ops.activation:bias_gelu"


def _bn_args(n):
    """Positional (x, w, b, rm, rv, training, momentum, eps, act, residual, grad_sink) of a BN node, or None."""
    if n.name != _BN or n.kwargs or len(n.args) != 11 or not isinstance(n.outs, P._Ref):
        return None
    return list(n.args)


class _Producers:
    def __init__(self, prog, keep):
        self.nodes = prog.nodes
        self.uses = _use_counts(self.nodes)
        self.producer = {}
        for i, n in enumerate(self.nodes):
            if not isinstance(n, P.CFNode):
                for s in P._node_writes(n):
                    self.producer.setdefault(s, i)
        self.keep = keep

    def single(self, ref):
        s = _slot(ref)
        return s is not None and self.uses.get(s, 0) == 1 and s not in self.keep

    def of(self, ref):
        i = self.producer.get(_slot(ref))
        return (i, self.nodes[i]) if i is not None else (None, None)


def _rewrite_until_fixed(prog, keep, step):
    fused = 0
    while True:
        pr = _Producers(prog, keep)
        done = False
        for j, n in enumerate(pr.nodes):
            if isinstance(n, P.CFNode) or n.kind == "guard":
                continue
            if step(pr, j, n):
                fused += 1
                done = True
                break
        if not done:
            return fused


@register_pass("fuse_bn_act")
class FuseBNActPass(PassBase):
    """Reference passes/cpp_pass.py FuseBatchNormActPass (fuse_bn_act_pass.cc): batch_norm followed by relu
    becomes ONE batch_norm_act_nhwc node with the ReLU in the kernel's epilogue (ops/bn.py, csrc/kernels/bn.hip),
    so the normalised activation is not written and re-read by a separate ReLU."""
    _after = ("auto_parallel_amp", "auto_parallel_fp16")

    def _type(self):
        return PassType.FUSION_OPT

    def _apply_single_impl(self, prog, startup, context):
        bn = P._resolve(_BN)

        def step(pr, j, n):
            if _act_of(n) != "relu":
                return False
            i, m = pr.of(n.args[0])
            a = _bn_args(m) if m is not None else None
            if a is None or a[8] is not None or not pr.single(n.args[0]):
                return False
            a[8] = "relu"
            pr.nodes[j] = _keep_rc(P.OpNode(bn, tuple(a), {}, n.outs, m.kind, _BN), m)
            del pr.nodes[i]
            return True

        n = _rewrite_until_fixed(prog, _protected(prog, self.get_attr("fetch_vars")), step)
        context.set_attr("fuse_bn_act.fused", context.get_attr("fuse_bn_act.fused", 0) + n)


@register_pass("fuse_bn_add_act")
class FuseBNAddActPass(PassBase):
    """Reference cpp_pass.py FuseBatchNormAddActPass: batch_norm -> + residual -> relu becomes ONE
    batch_norm_act_nhwc(residual=..., act="relu") node (the residual add and ReLU in the BN apply kernel; the
    backward emits the residual's gradient from the same kernel)."""
    _after = ("auto_parallel_amp", "auto_parallel_fp16")

    def _type(self):
        return PassType.FUSION_OPT

    def _apply_single_impl(self, prog, startup, context):
        bn = P._resolve(_BN)

        def step(pr, k, n):
            if _act_of(n) != "relu" or not pr.single(n.args[0]):
                return False
            j, add = pr.of(n.args[0])
            if add is None or add.name not in _ADD or len(add.args) != 2 or add.kwargs:
                return False
            for x, r in (add.args, add.args[::-1]):
                i, m = pr.of(x)
                a = _bn_args(m) if m is not None else None
                if a is None or a[8] is not None or a[9] is not None or not pr.single(x) or _slot(r) is None:
                    continue
                if _shape_of(prog, r) != _shape_of(prog, x) or prog._metas[_slot(r)].dtype != \
                        prog._metas[_slot(x)].dtype:
                    continue
                a[8], a[9] = "relu", r
                pr.nodes[k] = _keep_rc(P.OpNode(bn, tuple(a), {}, n.outs, m.kind, _BN), m)
                for d in sorted((i, j), reverse=True):
                    del pr.nodes[d]
                return True
            return False

        n = _rewrite_until_fixed(prog, _protected(prog, self.get_attr("fetch_vars")), step)
        context.set_attr("fuse_bn_add_act.fused", context.get_attr("fuse_bn_add_act.fused", 0) + n)


@register_pass("fuse_elewise_add_act")
class FuseElewiseAddActPass(PassBase):
    """Reference cpp_pass.py FuseElementwiseAddActPass: ``x + b`` (b a vector over the last dim) followed by the
    tanh GELU becomes ONE bias_gelu node (ops/activation.py, one HIP kernel forward and backward). A matmul
    producer is left to fuse_gemm_epilogue, which folds bias and GELU into the GEMM itself."""
    _after = ("auto_parallel_amp", "auto_parallel_fp16", "fuse_gemm_epilogue")

    def _type(self):
        return PassType.FUSION_OPT

    def _apply_single_impl(self, prog, startup, context):
        bg = P._resolve(_BIAS_GELU)

        def step(pr, k, n):
            if _act_of(n) != "gelu" or not pr.single(n.args[0]):
                return False
            j, add = pr.of(n.args[0])
            if add is None or add.name not in _ADD or len(add.args) != 2 or add.kwargs:
                return False
            for x, b in (add.args, add.args[::-1]):
                xs, bs = _shape_of(prog, x), _shape_of(prog, b)
                if _slot(x) is None or xs is None or bs is None or len(xs) < 1 or bs != (xs[-1],):
                    continue
                pi, pm = pr.of(x)
                if pm is not None and pm.name in _MATMUL:
                    continue  # the GEMM epilogue pass owns this pattern
                pr.nodes[k] = _keep_rc(P.OpNode(bg, (x, b), {}, n.outs, "op", _BIAS_GELU), add)
                del pr.nodes[j]
                return True
            return False

        n = _rewrite_until_fixed(prog, _protected(prog, self.get_attr("fetch_vars")), step)
        context.set_attr("fuse_elewise_add_act.fused", context.get_attr("fuse_elewise_add_act.fused", 0) + n)


@register_pass("fuse_all_reduce")
class FuseAllReducePass(PassBase):
    """Reference passes/fuse_all_reduce.py: consecutive all-reduces of one group / reduce op / dtype become ONE
    coalesced all-reduce over a flat buffer (the tensors are packed, reduced once and unpacked), up to
    ``max_memory_size`` bytes per bucket (default 256 MiB: few, large messages suit the per-link xGMI rings)."""

    def _type(self):
        return PassType.COMM_OPT

    def _apply_single_impl(self, prog, startup, context):
        cap = int(self.get_attr("max_memory_size", 256 << 20))
        nodes, out, fused, run = prog.nodes, [], 0, []

        def meta(n):
            m = getattr(n.func, "_pa_comm", None) if n.kind == "comm" else None
            if m is None or m[0] != "all_reduce" or len(n.args) != 1 or _slot(n.args[0]) is None:
                return None
            t = prog._metas[_slot(n.args[0])]
            return (m[1], id(m[2]) if m[2] is not None else None, t.dtype), m, t.numel() * t.element_size()

        def flush():
            nonlocal fused
            if len(run) > 1:
                out.append(_keep_rc(_coalesced([n for n, _ in run]), run[0][0]))
                fused += len(run) - 1
            else:
                out.extend(n for n, _ in run)
            run.clear()

        size = 0
        for n in nodes:
            mk = meta(n) if not isinstance(n, P.CFNode) else None
            if mk is None:
                flush()
                size = 0
                out.append(n)
                continue
            key, m, nbytes = mk
            if run and (run[0][1][0] != key or size + nbytes > cap or
                        any(_slot(r.args[0]) == _slot(n.args[0]) for r, _ in run)):
                flush()
                size = 0
            run.append((n, (key, m)))
            size += nbytes
        flush()
        prog.nodes[:] = out
        context.set_attr("fuse_all_reduce.fused", context.get_attr("fuse_all_reduce.fused", 0) + fused)


def _coalesced(nodes):
    import torch.distributed as tdist
    from ..collective import _TORCH_OP, _pg
    _, op, group = nodes[0].func._pa_comm
    refs = tuple(n.args[0] for n in nodes)

    def run(*xs):
        flat = torch.cat([x.reshape(-1) for x in xs])
        tdist.all_reduce(flat, op=_TORCH_OP[op], group=_pg(group))
        off = 0
        for x in xs:
            k = x.numel()
            x.copy_(flat[off:off + k].view_as(x))
            off += k
        return None
    run._pa_comm = ("all_reduce_coalesced", op, group)
    return P.OpNode(run, refs, {}, None, kind="comm", name="c:all_reduce_coalesced")


@register_pass("replace_with_parallel_cross_entropy")
class ReplaceWithParallelCrossEntropyPass(PassBase):
    """Reference passes/auto_parallel_replace_with_parallel_cross_entropy.py: a softmax cross entropy whose logits
    are sharded on the vocabulary runs on the local slice (c_softmax_with_cross_entropy) instead of gathering the
    logits. The per-rank program exists only inside the static engine, so the pass marks the program and the
    engine rewrites the op at partition time (static_engine._vocab_parallel: one all-gather of per-token
    (logsumexp, label logit) pairs)."""

    def _type(self):
        return PassType.PARALLEL_OPT

    def _apply_single_impl(self, prog, startup, context):
        prog._pa_vocab_ce = True


@register_pass("auto_parallel_c_embedding_pass")
class CEmbeddingPass(PassBase):
    """Reference passes/auto_parallel_c_embedding.py: an embedding lookup into a vocabulary-sharded table becomes
    c_embedding (masked local lookup, Partial(sum) output) instead of gathering the table; marks the program for
    the static engine's partition-time rewrite (static_engine._vocab_parallel)."""

    def _type(self):
        return PassType.PARALLEL_OPT

    def _apply_single_impl(self, prog, startup, context):
        prog._pa_vocab_emb = True
