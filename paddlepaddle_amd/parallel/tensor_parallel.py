"""Tensor (model) parallel layers and collective autograd ops.

Reference: python/paddle/distributed/fleet/layers/mpu/mp_layers.py:49 VocabParallelEmbedding, :336
ColumnParallelLinear, :543 RowParallelLinear, :744 ParallelCrossEntropy; mpu/mp_ops.py (_c_identity,
_c_concat, _c_split, _mp_allreduce); parallel_layers/random.py (RNG state tracker).

MI355X notes: one RCCL all-reduce per row-parallel GEMM (bf16, in place on the GEMM output); with
TP=2 on an 8xMI355X node the two ranks talk over one direct xGMI link. The GEMMs themselves use
the same fused linear path as the single-GPU model (hipBLASLt + HIP epilogues).
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist

from .. import nn
from ..distributed import collective as C
from ..framework.tensor import Tensor, _wrap
from ..nn import initializer as I
from .. import ops as _ops


def _mp_group():
    from ..distributed.fleet.topology import _get_hcg
    h = _get_hcg()
    return None if h is None else h.get_model_parallel_group()


def _ws(g):
    return 1 if g is None else g.nranks


def _mp_init_ctx(world):
    """Distributed (per-mp-rank) weights draw from the tracker's model_parallel_rng stream so the shards
    of one logical weight differ across the mp group (reference mp_layers.py creates them under
    get_rng_state_tracker().rng_state())."""
    if world > 1 and "model_parallel_rng" in _TRACKER.states_:
        return _TRACKER.rng_state()
    return contextlib.nullcontext()


def _rank(g):
    return 0 if g is None else g.rank


class _Identity(torch.autograd.Function):
    """forward: identity; backward: all-reduce over the mp group (c_identity)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        if _ws(ctx.group) > 1:
            g = g.contiguous()
            dist.all_reduce(g, group=ctx.group.process_group)
        return g, None


class _AllReduce(torch.autograd.Function):
    """forward: all-reduce; backward: identity (mp_allreduce)."""

    @staticmethod
    def forward(ctx, x, group):
        if _ws(group) > 1:
            x = x.contiguous().clone()
            dist.all_reduce(x, group=group.process_group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class _Split(torch.autograd.Function):
    """forward: keep my slice of the last dim; backward: all-gather (c_split)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        n = _ws(group)
        if n == 1:
            return x
        return x.chunk(n, -1)[_rank(group)].contiguous()

    @staticmethod
    def backward(ctx, g):
        return _gather_last(g, ctx.group), None


def _gather_last(x, group):
    n = _ws(group)
    if n == 1:
        return x
    x = x.contiguous()
    out = torch.empty((n,) + tuple(x.shape), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out.view(-1), x.view(-1), group=group.process_group)
    return torch.cat(list(out.unbind(0)), -1)


class _Concat(torch.autograd.Function):
    """forward: all-gather along last dim; backward: split (c_concat)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _gather_last(x, group)

    @staticmethod
    def backward(ctx, g):
        n = _ws(ctx.group)
        if n == 1:
            return g, None
        return g.chunk(n, -1)[_rank(ctx.group)].contiguous(), None


def _async_allreduce_hook(group):
    """dX hook of a column-parallel linear: all-reduce over the mp group on the collective stream, waited
    for (a stream dependency, no host block) after the dW GEMM has been issued."""
    def hook(dx):
        work = dist.all_reduce(dx, group=group.process_group, async_op=True)
        return work.wait
    return hook


def c_identity(t, group=None):
    g = group or _mp_group()
    return _Identity.apply(t, g) if _ws(g) > 1 else t


def mp_allreduce(t, group=None):
    g = group or _mp_group()
    return _AllReduce.apply(t, g) if _ws(g) > 1 else t


def c_split(t, group=None):
    g = group or _mp_group()
    return _Split.apply(t, g)


def c_concat(t, group=None):
    g = group or _mp_group()
    return _Concat.apply(t, g)


# paddle-style names operating on paddle Tensors
def _c_identity(tensor, group=None, skip_c_identity_dynamic=False):
    return _wrap(c_identity(tensor._t, group))


def _mp_allreduce(tensor, op=None, group=None, use_calc_stream=True, use_model_parallel=True,
                  skip_c_identity_dynamic=False):
    return _wrap(mp_allreduce(tensor._t, group))


def _c_split(tensor, group=None):
    return _wrap(c_split(tensor._t, group))


def _c_concat(tensor, group=None):
    return _wrap(c_concat(tensor._t, group))


class ColumnParallelLinear(nn.Layer):
    def __init__(self, in_features, out_features, weight_attr=None, has_bias=None, gather_output=True,
                 fuse_matmul_bias=False, mp_group=None, name=None, fuse_bias_act=None):
        super().__init__()
        self.group = mp_group or _mp_group()
        self.world = _ws(self.group)
        assert out_features % self.world == 0, "out_features must be divisible by the mp degree"
        self.out_per = out_features // self.world
        self.gather_output = gather_output
        self.act = fuse_bias_act
        with _mp_init_ctx(self.world):
            self.weight = self.create_parameter([in_features, self.out_per], attr=weight_attr)
        self.weight.is_distributed = self.world > 1
        self.bias = self.create_parameter([self.out_per], is_bias=True) if has_bias in (None, True) else None
        if self.bias is not None:
            self.bias.is_distributed = self.world > 1

    def forward(self, x):
        t = x._t
        w = self.weight._t
        if t.dtype != w.dtype:
            t = t.to(w.dtype)
        # c_identity's backward all-reduce, issued asynchronously right after the dX GEMM so it overlaps the
        # weight-gradient GEMM (reference: mp_layers.py ColumnParallelLinear + mp_async_allreduce)
        hook = _async_allreduce_hook(self.group) if self.world > 1 else None
        y = _ops.fused_linear(t, w, None if self.bias is None else self.bias._t, act=self.act, dx_hook=hook)
        if self.gather_output:
            y = c_concat(y, self.group)
        return _wrap(y)


class RowParallelLinear(nn.Layer):
    def __init__(self, in_features, out_features, weight_attr=None, has_bias=True, input_is_parallel=False,
                 fuse_matmul_bias=False, mp_group=None, name=None):
        super().__init__()
        self.group = mp_group or _mp_group()
        self.world = _ws(self.group)
        assert in_features % self.world == 0
        self.in_per = in_features // self.world
        self.input_is_parallel = input_is_parallel
        with _mp_init_ctx(self.world):
            self.weight = self.create_parameter([self.in_per, out_features], attr=weight_attr)
        self.weight.is_distributed = self.world > 1
        self.bias = self.create_parameter([out_features], is_bias=True) if has_bias else None

    def forward(self, x):
        t = x._t
        if not self.input_is_parallel:
            t = c_split(t, self.group)
        w = self.weight._t
        if t.dtype != w.dtype:
            t = t.to(w.dtype)
        y = _ops.fused_linear(t, w, None)
        y = mp_allreduce(y, self.group)
        if self.bias is not None:
            y = y + self.bias._t
        return _wrap(y)


class _VocabEmbed(torch.autograd.Function):
    pass


class VocabParallelEmbedding(nn.Layer):
    def __init__(self, num_embeddings, embedding_dim, weight_attr=None, mp_group=None, name=None):
        super().__init__()
        self.group = mp_group or _mp_group()
        self.world = _ws(self.group)
        self.per = (num_embeddings + self.world - 1) // self.world
        self.start = _rank(self.group) * self.per
        with _mp_init_ctx(self.world):
            self.weight = self.create_parameter([self.per, embedding_dim], attr=weight_attr,
                                                default_initializer=I.XavierNormal())
        self.weight.is_distributed = self.world > 1

    def local_lookup(self, ids):
        """This rank's partial embedding (rows of other ranks' vocab slices are 0), before the mp sum."""
        local = ids - self.start
        mask = (local < 0) | (local >= self.per)
        local = local.masked_fill(mask, 0)
        emb = torch.nn.functional.embedding(local, self.weight._t)
        return emb.masked_fill(mask.unsqueeze(-1), 0.0)

    def forward(self, x):
        ids = x._t
        if self.world == 1:
            return _wrap(torch.nn.functional.embedding(ids, self.weight._t))
        local = ids - self.start
        mask = (local < 0) | (local >= self.per)
        local = local.masked_fill(mask, 0)
        emb = torch.nn.functional.embedding(local, self.weight._t)
        emb = emb.masked_fill(mask.unsqueeze(-1), 0.0)
        return _wrap(mp_allreduce(emb, self.group))


class _ParallelCE(torch.autograd.Function):
    """Vocab-parallel softmax cross entropy with ONE collective. Each rank reduces its vocabulary slice to
    (logsumexp, label logit) per token (HIP slice kernel), the [N, 2] pairs are all-gathered over the mp group
    and combined locally (lse = logsumexp over ranks, label logit = sum: only the owning rank's is non-zero).
    The backward needs no collective: (exp(x - lse) - onehot) * g on the local slice with the global lse.
    Reference (3 all-reduces: max, sum-exp, label logit): mp_layers.py:744 ParallelCrossEntropy,
    c_softmax_with_cross_entropy."""

    @staticmethod
    def forward(ctx, logits, labels, group, ignore_index):
        # logits [N, V/mp] (any dtype), labels [N] global ids
        from ..ops.loss import ce_slice_stats
        n = _ws(group)
        per = logits.shape[-1]
        start = _rank(group) * per
        lg = logits.contiguous()
        lse_r, tgt_r = ce_slice_stats(lg, labels, start)
        mine = torch.stack([lse_r, tgt_r], -1).contiguous()       # [N, 2]
        allp = torch.empty((n,) + tuple(mine.shape), dtype=mine.dtype, device=mine.device)
        dist.all_gather_into_tensor(allp.view(-1), mine.view(-1), group=group.process_group)
        lse = torch.logsumexp(allp[..., 0], 0)
        tgt = allp[..., 1].sum(0)
        loss = (lse - tgt).masked_fill(labels == ignore_index, 0.0)
        ctx.save_for_backward(lg, labels, lse)
        ctx.start = start
        ctx.ignore_index = ignore_index
        return loss

    @staticmethod
    def backward(ctx, g):
        from ..ops.loss import ce_slice_grad
        lg, labels, lse = ctx.saved_tensors
        return ce_slice_grad(lg, labels, ctx.start, lse, g, ctx.ignore_index), None, None, None


def parallel_cross_entropy_raw(logits, labels, ignore_index=-100, group=None):
    g = group or _mp_group()
    V = logits.shape[-1]
    lf = logits.reshape(-1, V)
    lb = labels.reshape(-1).long()
    if _ws(g) == 1:
        return _ops.softmax_cross_entropy(lf, lb, ignore_index).view(labels.shape)
    return _ParallelCE.apply(lf, lb, g, ignore_index).view(labels.shape)


class ParallelCrossEntropy(nn.Layer):
    def __init__(self, mp_group=None, name=None, ignore_index=-100):
        super().__init__()
        self.group = mp_group or _mp_group()
        self.ignore_index = ignore_index

    def forward(self, input, label):
        lb = label._t
        if lb.dim() == input._t.dim():
            lb = lb.squeeze(-1)
        return _wrap(parallel_cross_entropy_raw(input._t, lb, self.ignore_index, self.group).unsqueeze(-1))


# ------------------------------------------------------------------------ RNG tracker
class RNGStatesTracker:
    """Named RNG streams so dropout inside TP regions differs per rank while replicated regions agree.
    Reference: fleet/meta_parallel/parallel_layers/random.py."""

    def __init__(self):
        self.states_ = {}
        self.seeds_ = set()

    def reset(self):
        self.states_ = {}
        self.seeds_ = set()

    def add(self, name, seed):
        if seed in self.seeds_:
            raise ValueError(f"seed {seed} already exists")
        if name in self.states_:
            raise ValueError(f"state {name} already exists")
        self.seeds_.add(seed)
        orig_cpu = torch.get_rng_state()
        orig_cuda = torch.cuda.get_rng_state() if torch.cuda.is_available() else None
        torch.manual_seed(seed)
        self.states_[name] = (torch.get_rng_state(), torch.cuda.get_rng_state() if torch.cuda.is_available() else None)
        torch.set_rng_state(orig_cpu)
        if orig_cuda is not None:
            torch.cuda.set_rng_state(orig_cuda)

    def get_states_tracker(self):
        return dict(self.states_)

    def set_states_tracker(self, states):
        self.states_ = dict(states)

    @contextlib.contextmanager
    def rng_state(self, name="model_parallel_rng"):
        if name not in self.states_:
            raise ValueError(f"state {name} does not exist")
        orig_cpu = torch.get_rng_state()
        orig_cuda = torch.cuda.get_rng_state() if torch.cuda.is_available() else None
        cpu, cuda = self.states_[name]
        torch.set_rng_state(cpu)
        if cuda is not None:
            torch.cuda.set_rng_state(cuda)
        try:
            yield
        finally:
            self.states_[name] = (torch.get_rng_state(),
                                  torch.cuda.get_rng_state() if torch.cuda.is_available() else None)
            torch.set_rng_state(orig_cpu)
            if orig_cuda is not None:
                torch.cuda.set_rng_state(orig_cuda)


_TRACKER = RNGStatesTracker()


def get_rng_state_tracker():
    return _TRACKER


def model_parallel_random_seed(seed=None):
    from ..distributed.fleet.topology import _get_hcg
    h = _get_hcg()
    rank = h.get_model_parallel_rank() if h else 0
    seed = seed or 1024
    _TRACKER.reset()
    _TRACKER.add("global_seed", seed)
    _TRACKER.add("model_parallel_rng", seed + 1 + rank * 100)
    torch.manual_seed(seed)
