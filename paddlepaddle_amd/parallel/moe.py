"""Mixture of Experts with expert parallelism over RCCL all-to-all.

Reference: python/paddle/incubate/distributed/models/moe/moe_layer.py:263 (MoELayer, MoEScatter /
MoEGather PyLayers, prepare_forward), gate/{naive_gate,gshard_gate,switch_gate}.py, grad_clip.py
(ClipGradForMOEByGlobalNorm), incubate/nn/functional/fused_moe.py.

Dispatch on MI355X: tokens are sorted by destination expert once (stable argsort on the device),
per-rank counts are exchanged with a tiny all-to-all, then ONE variable-split all-to-all moves the
tokens (each rank pair has its own xGMI link on an 8-GPU node, so an 8-way EP all-to-all is a single
hop per pair). Local experts run on contiguous slices, the reverse all-to-all brings
results home, and the weighted combine is one index_add. Backward is the mirror image (the
all-to-all autograd node swaps the split vectors).

Experts given as ``GroupedExperts`` (E same-shape FFNs with stacked weights) run as ONE grouped GEMM per
projection over all experts (csrc/kernels/grouped_gemm.hip via ops.moe), with routing offsets computed on the
device: without expert parallelism that layer never synchronises with the host and can be captured in a
hipGraph. ``fused_moe`` takes the same path.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist
import torch.nn.functional as TF

from .. import nn
from ..framework.tensor import Tensor, _wrap
from ..nn import initializer as I


def _ws(g):
    return 1 if g is None else g.nranks


class _AllToAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, in_splits, out_splits, group):
        ctx.in_splits, ctx.out_splits, ctx.group = in_splits, out_splits, group
        out = x.new_empty((sum(out_splits),) + tuple(x.shape[1:]))
        dist.all_to_all_single(out, x.contiguous(), out_splits, in_splits, group=group.process_group)
        return out

    @staticmethod
    def backward(ctx, g):
        out = g.new_empty((sum(ctx.in_splits),) + tuple(g.shape[1:]))
        dist.all_to_all_single(out, g.contiguous(), ctx.in_splits, ctx.out_splits, group=ctx.group.process_group)
        return out, None, None, None


# ------------------------------------------------------------------------------------- gates
class BaseGate(nn.Layer):
    def __init__(self, num_expert, world_size):
        super().__init__()
        self.world_size = world_size
        self.num_expert = num_expert
        self.tot_expert = world_size * num_expert
        self.loss = None

    def set_loss(self, loss):
        self.loss = loss

    def get_loss(self, clear=True):
        loss = self.loss
        if clear:
            self.loss = None
        return loss


class NaiveGate(BaseGate):
    """Linear router + top-k, no capacity limit."""

    def __init__(self, d_model, num_expert, world_size, topk=2):
        super().__init__(num_expert, world_size)
        self.gate = nn.Linear(d_model, self.tot_expert)
        self.top_k = topk

    def _logits(self, x):
        return self.gate(x)._t.float()

    def forward(self, inp, return_all_scores=False):
        logits = self._logits(inp)
        val, idx = logits.topk(self.top_k, -1)
        val = torch.softmax(val, -1)
        if return_all_scores:
            return _wrap(val), _wrap(idx), _wrap(logits)
        return _wrap(val), _wrap(idx)


def _limit_by_capacity(idx, capacity, n_exp):
    """Drop (set to -1) the assignments beyond each expert's capacity, in token order, slot-major."""
    flat = idx.t().reshape(-1)  # slot-major: all first choices before second choices
    valid = flat >= 0
    onehot = TF.one_hot(flat.clamp(min=0), n_exp) * valid[:, None]
    pos = onehot.cumsum(0) * onehot
    keep = (pos.sum(-1) <= capacity) & valid
    flat = torch.where(keep, flat, torch.full_like(flat, -1))
    return flat.view(idx.shape[1], idx.shape[0]).t()


class GShardGate(NaiveGate):
    """Top-2 with capacity factor and the GShard load-balancing auxiliary loss."""

    def __init__(self, d_model, num_expert, world_size, topk=2, capacity=(1.2, 2.4), random_routing=True,
                 group=None):
        assert topk == 2, "GShardGate is top-2"
        super().__init__(d_model, num_expert, world_size, topk)
        self.capacity = capacity
        self.random_routing = random_routing
        self.group = group

    def forward(self, x):
        logits = self._logits(x)
        probs = torch.softmax(logits, -1)
        val, idx = probs.topk(2, -1)
        n = logits.shape[0]
        # aux loss: mean prob per expert x fraction of tokens whose top-1 is the expert
        me = probs.mean(0)
        ce = TF.one_hot(idx[:, 0], self.tot_expert).float().mean(0)
        self.set_loss(_wrap((me * ce).sum() * self.tot_expert))
        cap_f = self.capacity[0] if self.training else self.capacity[1]
        cap = int(math.ceil(cap_f * n / self.tot_expert)) * 1
        if self.random_routing:
            rnd = torch.rand(n, device=x._t.device)
            drop2 = 2 * val[:, 1] < rnd
            idx = torch.stack([idx[:, 0], torch.where(drop2, torch.full_like(idx[:, 1], -1), idx[:, 1])], 1)
        idx = _limit_by_capacity(idx, cap, self.tot_expert)
        val = val / val.sum(-1, keepdim=True).clamp_min(1e-9)
        return _wrap(val), _wrap(idx)


class SwitchGate(NaiveGate):
    """Top-1 with capacity and the Switch-Transformer balance loss."""

    def __init__(self, d_model, num_expert, world_size, topk=1, switch_eps=0.1, capacity=(1.2, 2.4), group=None):
        assert topk == 1, "SwitchGate is top-1"
        super().__init__(d_model, num_expert, world_size, topk)
        self.switch_eps = switch_eps
        self.capacity = capacity
        self.group = group

    def forward(self, inp):
        logits = self._logits(inp)
        if self.training and self.switch_eps > 0:
            logits = logits + torch.empty_like(logits).uniform_(1 - self.switch_eps, 1 + self.switch_eps).log()
        probs = torch.softmax(logits, -1)
        val, idx = probs.topk(1, -1)
        n = logits.shape[0]
        frac = TF.one_hot(idx[:, 0], self.tot_expert).float().mean(0)
        self.set_loss(_wrap((frac * probs.mean(0)).sum() * self.tot_expert))
        cap = int(math.ceil((self.capacity[0] if self.training else self.capacity[1]) * n / self.tot_expert))
        idx = _limit_by_capacity(idx, cap, self.tot_expert)
        return _wrap(val), _wrap(idx)


# ------------------------------------------------------------------------------------- experts
class GroupedExperts(nn.Layer):
    """``num_experts`` FFN experts (fc1 [d, h] -> activation -> fc2 [h, d]) with stacked weights
    ``w1`` [E, d, h], ``w2`` [E, h, d] (+ biases [E, h], [E, d]). ``activation``: "gelu", "relu", "silu" or
    "swiglu" (then w1 is [E, d, 2h] and the two halves are the value / gate inputs)."""

    def __init__(self, num_experts, d_model, d_hidden, activation="gelu", bias=True, weight_attr=None):
        super().__init__()
        self.num_experts, self.d_model, self.d_hidden = num_experts, d_model, d_hidden
        self.activation = activation
        h1 = 2 * d_hidden if activation == "swiglu" else d_hidden
        init = I.XavierUniform() if weight_attr is None else None
        self.w1 = self.create_parameter([num_experts, d_model, h1], attr=weight_attr, default_initializer=init)
        self.w2 = self.create_parameter([num_experts, d_hidden, d_model], attr=weight_attr,
                                        default_initializer=init)
        self.b1 = self.create_parameter([num_experts, h1], is_bias=True) if bias else None
        self.b2 = self.create_parameter([num_experts, d_model], is_bias=True) if bias else None

    def __len__(self):
        return self.num_experts

    def forward_sorted(self, xs, offs):
        """xs [n, d] rows sorted by expert (offs [E + 1]) -> [n, d]; rows past offs[E] come out 0."""
        from ..ops import moe as M
        t = lambda p: None if p is None else p._t
        h = M.grouped_linear(xs, self.w1._t, offs, t(self.b1))
        if self.activation == "swiglu":
            from .. import ops as _ops
            h = _ops.swiglu(h)
        elif self.activation == "gelu":
            h = TF.gelu(h)
        elif self.activation == "relu":
            h = TF.relu(h)
        elif self.activation == "silu":
            h = TF.silu(h)
        return M.grouped_linear(h, self.w2._t, offs, t(self.b2))

    def forward(self, x, expert_index):
        """Dense helper: run every row of ``x`` through expert ``expert_index[row]``."""
        from ..ops import moe as M
        xt = x._t if isinstance(x, Tensor) else x
        ei = expert_index._t if isinstance(expert_index, Tensor) else expert_index
        offs, perm = M.route(ei, self.num_experts)
        y = self.forward_sorted(xt[perm], offs)
        out = torch.zeros_like(y).index_copy(0, perm, y)
        return _wrap(out)


# ------------------------------------------------------------------------------------- layer
class MoELayer(nn.Layer):
    """Experts ``experts`` are this rank's local experts; global expert e lives on rank
    e // num_local at local index e % num_local."""

    def __init__(self, d_model, experts, gate=None, moe_group=None, mp_group=None, recompute_interval=0,
                 recompute_ctx=None):
        super().__init__()
        self.d_model = d_model
        self.experts = experts
        self.num_expert = len(experts)
        self.group = moe_group
        self.world_size = _ws(moe_group)
        self.mp_group = mp_group
        self.recompute_interval = recompute_interval
        if gate is None or isinstance(gate, dict):
            cfg = gate or {}
            typ = cfg.get("type", "gshard")
            k = cfg.get("top_k", 2)
            if typ == "naive" or typ is None:
                gate = NaiveGate(d_model, self.num_expert, self.world_size, topk=k)
            elif typ == "gshard":
                gate = GShardGate(d_model, self.num_expert, self.world_size, topk=k, group=moe_group)
            elif typ == "switch":
                gate = SwitchGate(d_model, self.num_expert, self.world_size, topk=k, group=moe_group)
            else:
                raise ValueError(f"unknown gate type {typ}")
        self.gate = gate
        for p in self.experts.parameters():
            p.is_distributed = self.world_size > 1  # expert params differ per rank (not DP-replicated)

    def _grouped_local(self, x, val, idx):
        """Experts on this rank only, as grouped GEMMs with device-side routing (no host sync)."""
        from ..ops import moe as M
        N, K = idx.shape
        E = self.num_expert
        offs, perm = M.route(idx.reshape(-1), E)
        tok = perm // K
        n = perm.numel()
        valid = torch.arange(n, device=x.device, dtype=torch.int32) < offs[E]
        wts = torch.where(valid, val.reshape(-1)[perm], torch.zeros((), dtype=val.dtype, device=val.device))
        y = self.experts.forward_sorted(x[tok], offs)
        out = torch.zeros_like(x, dtype=y.dtype)
        return out.index_add(0, tok, y * wts[:, None].to(y.dtype))

    def _run_experts(self, x, counts):
        if isinstance(self.experts, GroupedExperts):
            offs = torch.zeros(len(counts) + 1, dtype=torch.int32)
            offs[1:] = torch.cumsum(torch.tensor(counts, dtype=torch.int64), 0).to(torch.int32)
            return self.experts.forward_sorted(x, offs.to(x.device))
        outs, off = [], 0
        for i, c in enumerate(counts):
            if c:
                seg = _wrap(x[off:off + c])
                if self.recompute_interval and self.training:
                    from ..distributed.fleet.recompute import recompute
                    outs.append(recompute(self.experts[i], seg)._t)
                else:
                    outs.append(self.experts[i](seg)._t)
            off += c
        return torch.cat(outs, 0) if outs else x[:0]

    def forward(self, inp):
        shape = inp.shape
        x = inp._t.reshape(-1, self.d_model)
        val, idx = self.gate(_wrap(x))
        val, idx = val._t, idx._t
        if self.world_size == 1 and isinstance(self.experts, GroupedExperts):
            return _wrap(self._grouped_local(x, val, idx).reshape(shape))
        N, K = idx.shape
        E = self.num_expert * self.world_size
        flat_e = idx.reshape(-1)
        keep = flat_e >= 0
        tok = torch.arange(N, device=x.device).repeat_interleave(K)[keep]
        wts = val.reshape(-1)[keep]
        fe = flat_e[keep]
        order = torch.argsort(fe, stable=True)
        tok, wts, fe = tok[order], wts[order], fe[order]
        counts_e = torch.bincount(fe, minlength=E)  # per global expert
        xs = x[tok]
        if self.world_size > 1:
            g = self.group
            send = counts_e.view(self.world_size, self.num_expert)
            recv = torch.empty_like(send)
            dist.all_to_all_single(recv, send.contiguous(), group=g.process_group)
            in_splits = send.sum(1).tolist()
            out_splits = recv.sum(1).tolist()
            xr = _AllToAll.apply(xs, in_splits, out_splits, g)
            # received blocks are [src rank][local expert]; regroup by local expert
            rc = recv.tolist()
            pieces, off = [], 0
            for r in range(self.world_size):
                for e in range(self.num_expert):
                    pieces.append((e, r, off, rc[r][e]))
                    off += rc[r][e]
            perm = [torch.arange(o, o + c, device=x.device) for e, r, o, c in sorted(pieces)]
            perm = torch.cat(perm) if perm else torch.zeros(0, dtype=torch.long, device=x.device)
            local_counts = recv.sum(0).tolist()
            y = self._run_experts(xr[perm], local_counts)
            inv = torch.empty_like(perm)
            inv[perm] = torch.arange(perm.numel(), device=x.device)
            y = _AllToAll.apply(y[inv], out_splits, in_splits, g)
        else:
            y = self._run_experts(xs, counts_e.tolist())
        out = torch.zeros_like(x, dtype=y.dtype)
        out = out.index_add(0, tok, y * wts[:, None].to(y.dtype))
        return _wrap(out.reshape(shape))


class ClipGradForMOEByGlobalNorm(nn.ClipGradByGlobalNorm):
    """Global-norm clip where expert parameters' squared norms are summed over the MoE group."""

    def __init__(self, clip_norm, is_expert_param_func=None, moe_group=None, group_name="default_moe_group"):
        super().__init__(clip_norm, group_name)
        self.is_expert = is_expert_param_func or (lambda p: getattr(p, "is_distributed", False))
        self.moe_group = moe_group

        def _param_sq(params, _self=self):
            from ..ops.optim import global_sq_norm
            ex = [p._t.grad for p in params if _self.is_expert(p)]
            nx = [p._t.grad for p in params if not _self.is_expert(p)]
            dev = params[0]._t.device
            sq_e = (global_sq_norm(ex) if ex else torch.zeros((), device=dev)).reshape(1).clone()
            if _self.moe_group is not None and _self.moe_group.nranks > 1:
                dist.all_reduce(sq_e, group=_self.moe_group.process_group)
            sq_n = global_sq_norm(nx) if nx else torch.zeros((), device=dev)
            return (sq_e + sq_n).reshape(())
        self._param_sq_fn = _param_sq


# ------------------------------------------------------------------------------------- fused
def fused_moe(x, gate_weight, ffn1_weight, ffn2_weight, ffn1_bias=None, ffn1_scale=None, ffn2_bias=None,
              ffn2_scale=None, quant_method="None", moe_topk=2, norm_topk_prob=True):
    """All experts local: route with the gate *logits* ``gate_weight`` [.., E], SwiGLU FFN per expert
    (ffn1 [E, d, 2f] -> swiglu -> ffn2 [E, f, d]); routing and both projections run on the device as grouped
    GEMMs over the expert-sorted tokens (no host sync)."""
    from .. import ops as _ops
    xt = x._t
    d = xt.shape[-1]
    xf = xt.reshape(-1, d)
    g = gate_weight._t.reshape(xf.shape[0], -1).float()
    probs = torch.softmax(g, -1)
    val, idx = probs.topk(moe_topk, -1)
    if norm_topk_prob:
        val = val / val.sum(-1, keepdim=True)
    from ..ops import moe as M
    N, K = idx.shape
    E = ffn1_weight.shape[0]
    offs, perm = M.route(idx.reshape(-1), E)
    tok = perm // K
    wts = val.reshape(-1)[perm]
    b1 = ffn1_bias._t.reshape(E, -1) if ffn1_bias is not None else None
    b2 = ffn2_bias._t.reshape(E, -1) if ffn2_bias is not None else None
    h = M.grouped_linear(xf[tok], ffn1_weight._t, offs, b1)
    h = _ops.swiglu(h)
    y = M.grouped_linear(h, ffn2_weight._t, offs, b2)
    out = torch.zeros_like(xf).index_add(0, tok, (y * wts[:, None].to(y.dtype)).to(xf.dtype))
    return _wrap(out.reshape(xt.shape))
