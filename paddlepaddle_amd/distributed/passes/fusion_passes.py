"""More registered program passes over traced static Programs (static/program.py): the fusion passes of the
reference's build strategy / cpp_pass.py and the auto-parallel passes the engines apply.

* ``fused_feedforward`` (reference cpp_pass.py:89 fused_feedforward_pass): ``fused_linear(x, W1, b1, gelu)`` whose
  only consumer is ``fused_linear(h, W2, b2)`` becomes ONE ``ops.linear.ffn_gelu`` node: one autograd node whose
  backward can run the GELU backward and fc1's bias-gradient column sums in fc2's data-gradient GEMM epilogue.
* ``fused_attention`` (cpp_pass.py:76 fused_attention_pass): the attention core of a traced block is already one
  flash-attention op; what this pass fuses is the block's output side — the out-projection ``fused_linear`` whose
  only consumer is a residual ``add`` becomes ``fused_linear(..., residual=r)`` (the add read by the GEMM epilogue,
  no [M, N] elementwise pass). Applies to any linear + residual add.
* ``fuse_dot_product_attention`` (cpp_pass.py:128): ``matmul(q, k^T) [* scale] [+ mask] -> softmax(-1) ->
  matmul(p, v)`` over [B, H, S, D] becomes ONE ``ops.attention.attention_bhsd`` node (the flash-attention kernel:
  no [B, H, S, S] score / probability tensors).
* ``fuse_adamw`` / ``fuse_optimizer`` (cpp_pass.py:115 / :141): the program's optimizer updates run as multi-tensor
  launches; parameter groups with identical hyper-parameters are merged so each dtype's update is one launch
  (the HIP update kernels take every parameter of a group in one table).
* ``auto_parallel_master_grad_pass`` (auto_parallel_master_grad.py:84): 16-bit parameters' gradients accumulate in
  fp32 ``main_grad`` buffers across backward passes (gradient merge) and the optimizer reads their sum, rounded
  once (static/executor.py).
* ``auto_parallel_grad_clip`` (auto_parallel_grad_clip.py:294): the global-norm clip of a partitioned program
  counts every parameter's squared norm once over the whole mesh (tensor-parallel shards summed, replicas
  counted once, pipeline stages summed) — installed on the optimizer's clip by the static engine through this pass.
* ``auto_parallel_data_parallel_optimization`` (auto_parallel_data_parallel_optimization.py:55): static collective
  data parallelism launches each gradient bucket's all-reduce from backward hooks as soon as the bucket is
  complete (overlap with the rest of backward), buckets of ``bucket_size_mb``.
* ``auto_parallel_quantization`` (auto_parallel_quantization.py:48): quantization-aware training on the program —
  fake quant-dequant of activations (moving-average abs-max) and weights (abs-max / channel-wise) with
  straight-through gradients in front of every linear / matmul / conv (static/quantization quant_aware).
"""
from __future__ import annotations

import torch

from .pass_base import PassBase, PassType, register_pass
from ...static import program as P
from .program_passes import _ADD, _LINEAR, _MATMUL, _keep_rc, _protected, _rewrite_until_fixed, _shape_of, _slot

__all__ = ["FusedFeedforwardPass", "FusedAttentionPass", "FuseDotProductAttentionPass", "FuseAdamWPass",
           "FuseOptimizerPass", "MasterGradPass", "GradClipPass", "DataParallelOptimizationPass", "QuantizationPass"]

_FFN = "o:paddlepaddle_amd.ops.linear:ffn_gelu"
_ATTN_BHSD = "o:paddlepaddle_amd.ops.attention:attention_bhsd"
_SOFTMAX = {"o:paddlepaddle_amd.ops.activation:softmax", "f:torch:softmax", "m:softmax",
            "f:torch.nn.functional:softmax"}
_GELU_TANH = {"o:paddlepaddle_amd.ops.activation:gelu"}
_MUL = {"m:mul", "m:__mul__", "f:torch:mul", "m:__rmul__"}
_DIV = {"m:div", "m:__truediv__", "f:torch:div"}
_TRANSPOSE = {"m:transpose", "f:torch:transpose"}


def _linear_parts(n):
    """(x, w, b, act) of a plain fused_linear node (positional form, no hooks / residual), else None."""
    if n is None or n.name != _LINEAR or n.kwargs or not isinstance(n.outs, P._Ref):
        return None
    a = list(n.args) + [None] * (4 - len(n.args))
    if len(n.args) > 4 and any(v is not None for v in n.args[4:]):
        return None
    return a[0], a[1], a[2], a[3]


def _meta(prog, ref):
    if isinstance(ref, P._Ref):
        return prog._metas[ref.i]
    if isinstance(ref, P._Const):
        return ref.t
    return None


@register_pass("fused_feedforward")
class FusedFeedforwardPass(PassBase):
    _after = ("auto_parallel_amp", "auto_parallel_fp16", "fuse_gemm_epilogue")

    def _type(self):
        return PassType.FUSION_OPT

    def _apply_single_impl(self, prog, startup, context):
        ffn = P._resolve(_FFN)

        def step(pr, k, n):
            second = _linear_parts(n)
            if second is None or second[3] is not None or not pr.single(second[0]):
                return False
            j, m = pr.of(second[0])
            act_i = None
            first = _linear_parts(m)
            if first is None and m is not None and m.name in _GELU_TANH:  # fused_linear -> gelu(tanh) -> linear
                approx = m.args[1] if len(m.args) > 1 else m.kwargs.get("approximate", False)
                if approx is not True or not pr.single(m.args[0]):
                    return False
                act_i = j
                j, m = pr.of(m.args[0])
                first = _linear_parts(m)
                if first is None or first[3] is not None:
                    return False
            elif first is None or first[3] not in ("gelu", "gelu_tanh", "gelu_approximate"):
                return False
            x, w1, b1, _ = first
            if b1 is None:
                return False
            w2, b2 = second[1], second[2]
            m1, m2 = _meta(prog, w1), _meta(prog, w2)
            if m1 is None or m2 is None or m1.dim() != 2 or m2.dim() != 2 or m1.shape[1] != m2.shape[0]:
                return False
            pr.nodes[k] = _keep_rc(P.OpNode(ffn, (x, w1, b1, w2, b2), {}, n.outs, "op", _FFN), m)
            for d in sorted([i for i in (j, act_i) if i is not None], reverse=True):
                del pr.nodes[d]
            return True

        n = _rewrite_until_fixed(prog, _protected(prog, self.get_attr("fetch_vars")), step)
        context.set_attr("fused_feedforward.fused", context.get_attr("fused_feedforward.fused", 0) + n)


@register_pass("fused_attention")
class FusedAttentionPass(PassBase):
    _after = ("auto_parallel_amp", "auto_parallel_fp16", "fuse_gemm_epilogue")

    def _type(self):
        return PassType.FUSION_OPT

    def _apply_single_impl(self, prog, startup, context):
        lin = P._resolve(_LINEAR)

        def step(pr, k, n):
            if n.name not in _ADD or len(n.args) != 2 or n.kwargs or not isinstance(n.outs, P._Ref):
                return False
            for y, r in (n.args, n.args[::-1]):
                if _slot(y) is None or _slot(r) is None or not pr.single(y):
                    continue
                j, m = pr.of(y)
                parts = _linear_parts(m)
                if parts is None or parts[3] is not None:
                    continue
                my, mr = prog._metas[_slot(y)], prog._metas[_slot(r)]
                if tuple(my.shape) != tuple(mr.shape) or my.dtype != mr.dtype:
                    continue
                x, w, b, _ = parts
                pr.nodes[k] = _keep_rc(P.OpNode(lin, (x, w, b, None, None, r), {}, n.outs, "op", _LINEAR), m)
                del pr.nodes[j]
                return True
            return False

        n = _rewrite_until_fixed(prog, _protected(prog, self.get_attr("fetch_vars")), step)
        context.set_attr("fused_attention.fused", context.get_attr("fused_attention.fused", 0) + n)


@register_pass("fuse_dot_product_attention")
class FuseDotProductAttentionPass(PassBase):
    _after = ("auto_parallel_amp", "auto_parallel_fp16")

    def _type(self):
        return PassType.FUSION_OPT

    def _apply_single_impl(self, prog, startup, context):
        op = P._resolve(_ATTN_BHSD)

        def scalar(v):
            return isinstance(v, (int, float)) and not isinstance(v, bool)

        def step(pr, k, n):
            # matmul(p, v) with p = softmax(s, -1)
            if n.name not in _MATMUL or len(n.args) != 2 or n.kwargs or not isinstance(n.outs, P._Ref):
                return False
            pv, v = n.args
            if not pr.single(pv) or _slot(v) is None:
                return False
            i_sm, sm = pr.of(pv)
            if sm is None or sm.name not in _SOFTMAX or sm.kwargs.get("dtype") is not None:
                return False
            axis = sm.args[1] if len(sm.args) > 1 else sm.kwargs.get("axis", sm.kwargs.get("dim", -1))
            mv = prog._metas[_slot(v)]
            if mv.dim() != 4 or axis not in (-1, 3) or not pr.single(sm.args[0]):
                return False
            dead = [i_sm]
            cur = sm.args[0]
            mask, scale = None, 1.0
            i_c, c = pr.of(cur)
            if c is not None and c.name in _ADD and len(c.args) == 2 and not c.kwargs:  # + additive mask
                a0, a1 = c.args
                if _slot(a1) is not None and pr.single(cur):
                    dead.append(i_c)
                    cur, mask = a0, a1
                    i_c, c = pr.of(cur)
            if c is not None and (c.name in _MUL or c.name in _DIV) and len(c.args) == 2 and not c.kwargs \
                    and scalar(c.args[1]) and pr.single(cur):
                scale = float(c.args[1]) if c.name in _MUL else 1.0 / float(c.args[1])
                dead.append(i_c)
                cur = c.args[0]
                i_c, c = pr.of(cur)
            if c is None or c.name not in _MATMUL or len(c.args) != 2 or c.kwargs or not pr.single(cur):
                return False
            q, kt = c.args
            dead.append(i_c)
            i_t, t = pr.of(kt)
            if t is None or t.name not in _TRANSPOSE or not pr.single(kt) or len(t.args) != 3:
                return False
            dims = {int(d) % 4 for d in t.args[1:]}
            if dims != {2, 3}:
                return False
            kk = t.args[0]
            dead.append(i_t)
            mq, mk = _meta(prog, q), _meta(prog, kk)
            if mq is None or mk is None or mq.dim() != 4 or mk.dim() != 4 or mq.shape[-1] != mk.shape[-1] or \
                    mk.shape[-2] != mv.shape[-2]:
                return False
            pr.nodes[k] = _keep_rc(P.OpNode(op, (q, kk, v, scale, mask), {}, n.outs, "op", _ATTN_BHSD), c)
            for d in sorted(dead, reverse=True):
                del pr.nodes[d]
            return True

        n = _rewrite_until_fixed(prog, _protected(prog, self.get_attr("fetch_vars")), step)
        context.set_attr("fuse_dot_product_attention.fused",
                         context.get_attr("fuse_dot_product_attention.fused", 0) + n)


def _merge_groups(opt):
    """Merge parameter groups whose hyper-parameters are equal (one multi-tensor launch per dtype per group)."""
    groups = getattr(opt, "_param_groups", None)
    if not groups or len(groups) < 2 or not isinstance(groups[0], dict):
        return 0
    merged, keys = [], []
    for g in groups:
        key = {k: v for k, v in g.items() if k != "params"}
        for mk, mg in zip(keys, merged):
            if mk == key:
                mg["params"] = list(mg["params"]) + list(g["params"])
                break
        else:
            keys.append(key)
            merged.append(dict(g, params=list(g["params"])))
    n = len(groups) - len(merged)
    opt._param_groups = merged
    return n


class _FuseOptBase(PassBase):
    _kinds = ()

    def _type(self):
        return PassType.FUSION_OPT

    def _apply_single_impl(self, prog, startup, context):
        if prog._optimize is None:
            return
        opt = prog._optimize[0]
        inner = getattr(opt, "_inner_opt", opt)
        if type(inner).__name__ not in self._kinds:
            return
        inner._use_multi_tensor = True
        n = _merge_groups(inner)
        context.set_attr(f"{self.name}.merged_groups", n)
        context.set_attr(f"{self.name}.optimizer", type(inner).__name__)


@register_pass("fuse_adamw")
class FuseAdamWPass(_FuseOptBase):
    name = "fuse_adamw"
    _kinds = ("AdamW", "Adam")


@register_pass("fuse_optimizer")
class FuseOptimizerPass(_FuseOptBase):
    name = "fuse_optimizer"
    _kinds = ("AdamW", "Adam", "SGD", "Momentum", "Lamb")


@register_pass("auto_parallel_master_grad_pass")
class MasterGradPass(PassBase):
    def _type(self):
        return PassType.CALC_OPT

    def _apply_single_impl(self, prog, startup, context):
        if prog._optimize is None:
            raise ValueError("auto_parallel_master_grad_pass needs a program with optimizer.minimize(loss)")
        prog._pa_master_grad = True
        context.set_attr("auto_parallel_master_grad_pass.applied", True)


@register_pass("auto_parallel_grad_clip")
class GradClipPass(PassBase):
    """attrs: ``optimizer`` (whose ``_grad_clip`` is a global-norm clip) and ``sq_norm_fn`` (params -> global
    squared norm of this rank's gradients reduced over the mesh, from the partitioning engine)."""

    def _type(self):
        return PassType.PARALLEL_OPT

    def _check_self(self):
        return self.get_attr("optimizer") is not None and callable(self.get_attr("sq_norm_fn"))

    def _apply_single_impl(self, prog, startup, context):
        clip = getattr(self.get_attr("optimizer"), "_grad_clip", None)
        ok = clip is not None and hasattr(clip, "_extra_sq_norm_fn")
        if ok:
            clip._param_sq_fn = self.get_attr("sq_norm_fn")
        context.set_attr("auto_parallel_grad_clip.applied", ok)


@register_pass("auto_parallel_data_parallel_optimization")
class DataParallelOptimizationPass(PassBase):
    """attrs: ``bucket_size_mb`` (default FLAGS_dp_bucket_mb or 128), ``overlap`` (default True)."""

    def _type(self):
        return PassType.COMM_OPT

    def _apply_single_impl(self, prog, startup, context):
        from ...framework.flags import flag
        mb = float(self.get_attr("bucket_size_mb", flag("FLAGS_dp_bucket_mb", 128)))
        prog._pa_dp_opt = {"bucket_bytes": max(1, int(mb * (1 << 20))), "overlap": bool(self.get_attr("overlap", True))}
        context.set_attr("auto_parallel_data_parallel_optimization.config", dict(prog._pa_dp_opt))


@register_pass("auto_parallel_quantization")
class QuantizationPass(PassBase):
    """attrs: the quant_aware config keys (weight_bits, activation_bits, weight_quantize_type,
    activation_quantize_type, quantize_op_types, moving_rate)."""

    def _type(self):
        return PassType.CALC_OPT

    def _apply_single_impl(self, prog, startup, context):
        from ...static.quantization.quanter import quant_aware
        keys = ("weight_bits", "activation_bits", "weight_quantize_type", "activation_quantize_type",
                "quantize_op_types", "moving_rate", "is_full_quantize")
        cfg = {k: self.get_attr(k) for k in keys if self.get_attr(k) is not None}
        quant_aware(prog, config=cfg)
        context.set_attr("auto_parallel_quantization.quantized", len(getattr(prog, "_quant_nodes", [])))


# ------------------------------------------------------------------------------------------------------------------
from .program_passes import GradientMergePass  # noqa: E402


@register_pass("auto_parallel_gradient_merge_pass")
class GradientMergeAliasPass(GradientMergePass):
    """The reference's registered name for gradient merge (auto_parallel_gradient_merge.py:808); the same pass as
    ``auto_parallel_gradient_merge``: the Executor / engine accumulate ``k_steps`` runs and update on the last."""


@register_pass("auto_parallel_sequence_parallel_optimization")
class SequenceParallelOptimizationPass(PassBase):
    """Reference auto_parallel_sequence_parallel_optimization.py:32 (strategy.sp_optimization): a row-parallel
    output that enters a sequence-parallel region is reduced with ONE reduce-scatter instead of an all-reduce
    followed by a slice (``_fuse_allreduce_split`` there). The pass marks the program; the static engine's
    partitioner emits the reduce-scatter for every Partial -> Shard conversion of a marked program
    (static_engine._convert)."""

    def _type(self):
        return PassType.COMM_OPT

    def _apply_single_impl(self, prog, startup, context):
        prog._pa_sp_opt = True
        context.set_attr("auto_parallel_sequence_parallel_optimization.enabled", True)


@register_pass("auto_parallel_pipeline")
class AutoParallelPipelinePass(PassBase):
    """Reference auto_parallel_pipeline.py:48 (the static pipeline pass of the auto-parallel engine): builds the
    stage's job list for ``schedule_mode`` (FThenB / 1F1B / Eager1F1B / ZBH1 / VPP / ZBVPP) through the registered
    ``pipeline_scheduler_<mode>`` pass and returns it as ``auto_parallel_pipeline.job_list``."""

    _MODES = {"FTHENB": "FThenB", "1F1B": "1F1B", "EAGER1F1B": "Eager1F1B", "ZBH1": "ZBH1", "VPP": "VPP",
              "ZBVPP": "ZBVPP"}

    def _type(self):
        return PassType.PARALLEL_OPT

    def _check_self(self):
        return str(self.get_attr("schedule_mode", "1F1B")).upper() in self._MODES

    def _apply_single_impl(self, prog, startup, context):
        from .pass_base import new_pass
        mode = self._MODES[str(self.get_attr("schedule_mode", "1F1B")).upper()]
        attrs = {k: self.get_attr(k) for k in ("num_micro_batches", "pp_stage", "pp_degree", "vpp_degree")
                 if self.get_attr(k) is not None}
        ctx = new_pass(f"pipeline_scheduler_{mode}", attrs).apply(prog, startup)
        context.set_attr("auto_parallel_pipeline.job_list", ctx.get_attr("pipeline_scheduler.job_list"))
        context.set_attr("auto_parallel_pipeline.mode", mode)


_SUM = 0  # distributed.collective.ReduceOp.SUM


def _first_rank_of(comm_node):
    """Whether this process is rank 0 of the group of a recorded collective (meta = (kind, op, group))."""
    meta = getattr(comm_node.func, "_pa_comm", None)
    group = meta[2] if isinstance(meta, tuple) and len(meta) > 2 else None
    from .. import collective as C
    return C.get_rank(group) == 0 if group is not None else C.get_rank() == 0


@register_pass("auto_parallel_fused_linear_promotion")
class FusedLinearPromotionPass(PassBase):
    """Reference auto_parallel_fused_linear_promotion.py:130: in tensor parallelism a row-parallel linear is
    ``matmul -> all_reduce(sum) -> + bias``, which keeps the bias add out of the GEMM. The bias is promoted in front
    of the reduction on the group's first rank only — ``fused_linear(x, W, b)`` there (the bias in the hand-written
    GEMM's epilogue), the plain matmul on the other ranks — and the add disappears (its output aliases the reduced
    tensor). The reduction then sums exactly one copy of the bias. Only the first rank's bias gets a gradient (and
    an update), as in the reference."""
    _after = ("auto_parallel_amp", "auto_parallel_fp16")

    def _type(self):
        return PassType.FUSION_OPT

    def _apply_single_impl(self, prog, startup, context):
        lin = P._resolve(_LINEAR)
        keep = _protected(prog, self.get_attr("fetch_vars"))

        def step(pr, k, n):
            if n.name not in _ADD or len(n.args) != 2 or n.kwargs or not isinstance(n.outs, P._Ref):
                return False
            for h, b in (n.args, n.args[::-1]):
                s = _slot(h)
                hs, bs = _shape_of(prog, h), _shape_of(prog, b)
                if s is None or hs is None or bs is None or bs != (hs[-1],) or s in keep:
                    continue
                writers = [i for i in range(k) if s in P._node_writes(pr.nodes[i])]
                if len(writers) != 2 or pr.uses.get(s, 0) != 2:  # created by the matmul, reduced in place, read here
                    continue
                i_m, i_c = writers
                m, c = pr.nodes[i_m], pr.nodes[i_c]
                meta = getattr(c.func, "_pa_comm", None)
                if c.kind != "comm" or not isinstance(meta, tuple) or meta[0] != "all_reduce" or \
                        meta[1] != _SUM or len(c.args) != 1:
                    continue
                if m.name not in _MATMUL or len(m.args) != 2 or m.kwargs:
                    continue
                ws = _shape_of(prog, m.args[1])
                if ws is None or len(ws) != 2 or ws[1] != bs[0]:
                    continue
                if _first_rank_of(c):
                    pr.nodes[i_m] = _keep_rc(P.OpNode(lin, (m.args[0], m.args[1], b), {}, m.outs, "op", _LINEAR), m)
                pr.nodes[k] = _keep_rc(P.OpNode(torch.Tensor.view_as, (h, h), {}, n.outs, "op", "m:view_as"), n)
                return True
            return False

        n = _rewrite_until_fixed(prog, keep, step)
        context.set_attr("auto_parallel_fused_linear_promotion.promoted",
                         context.get_attr("auto_parallel_fused_linear_promotion.promoted", 0) + n)


@register_pass("auto_parallel_supplement_explicit_dependencies")
class SupplementExplicitDependenciesPass(PassBase):
    """Reference auto_parallel_supplement_explicit_dependencies.py:41: a graph executor that may reorder ops must
    not let the ranks issue their collectives in different orders (a hang). The executors here replay an ordered
    instruction list, and the native scheduler (static/program.py build_plan) issues collectives as early as their
    inputs allow — the pass pins program order instead: it adds an explicit ordering edge from every collective to
    the next one (``prog._pa_comm_chain``, honoured by build_plan), so the scheduled order of the collectives is
    the traced order on every rank whatever the priorities of the ops between them. Returns the chain length as
    ``auto_parallel_supplement_explicit_dependencies.chained``."""

    def _type(self):
        return PassType.COMM_OPT

    def _apply_single_impl(self, prog, startup, context):
        comm = [i for i, n in enumerate(prog.nodes) if not isinstance(n, P.CFNode) and n.kind == "comm"]
        prog._pa_comm_chain = [id(prog.nodes[i]) for i in comm]
        context.set_attr("auto_parallel_supplement_explicit_dependencies.chained", max(0, len(comm) - 1))
