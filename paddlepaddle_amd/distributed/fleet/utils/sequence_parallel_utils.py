"""Sequence parallelism helpers. Reference: python/paddle/distributed/fleet/utils/sequence_parallel_utils.py
(ScatterOp, GatherOp, AllGatherOp, ReduceScatterOp, ColumnSequenceParallelLinear,
RowSequenceParallelLinear, mark_as_sequence_parallel_parameter, register_sequence_parallel_allreduce_hooks).
Activations are split along axis 0 (sequence-major [S, B, H] layout, as in the reference)."""
from __future__ import annotations

import torch
import torch.distributed as dist

from .... import nn
from ....framework.tensor import _wrap
from ....parallel import tensor_parallel as tp
from .... import ops as _ops


def _g(group):
    return group or tp._mp_group()


def _scatter0(x, g):
    n = tp._ws(g)
    return x if n == 1 else x.chunk(n, 0)[tp._rank(g)].contiguous()


def _gather0(x, g):
    n = tp._ws(g)
    if n == 1:
        return x
    x = x.contiguous()
    out = torch.empty((n * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x, group=g.process_group)
    return out


def _rs0(x, g):
    n = tp._ws(g)
    if n == 1:
        return x
    x = x.contiguous()
    out = torch.empty((x.shape[0] // n,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.reduce_scatter_tensor(out, x, group=g.process_group)
    return out


class _Scatter(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g):
        ctx.g = g
        return _scatter0(x, g)

    @staticmethod
    def backward(ctx, d):
        return _gather0(d, ctx.g), None


class _Gather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g):
        ctx.g = g
        return _gather0(x, g)

    @staticmethod
    def backward(ctx, d):
        return _scatter0(d, ctx.g), None


class _AllGather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g):
        ctx.g = g
        return _gather0(x, g)

    @staticmethod
    def backward(ctx, d):
        return _rs0(d, ctx.g), None


class _ReduceScatter(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g):
        ctx.g = g
        return _rs0(x, g)

    @staticmethod
    def backward(ctx, d):
        return _gather0(d, ctx.g), None


class ScatterOp:
    @staticmethod
    def apply(x, group=None):
        return _wrap(_Scatter.apply(x._t, _g(group)))


class GatherOp:
    @staticmethod
    def apply(x, group=None):
        return _wrap(_Gather.apply(x._t, _g(group)))


class AllGatherOp:
    @staticmethod
    def apply(x, group=None):
        return _wrap(_AllGather.apply(x._t, _g(group)))


class ReduceScatterOp:
    @staticmethod
    def apply(x, group=None):
        return _wrap(_ReduceScatter.apply(x._t, _g(group)))


def scatter(x, group=None):
    return ScatterOp.apply(x, group)


def all_gather(x, group=None):
    return AllGatherOp.apply(x, group)


def reduce_scatter(x, group=None):
    return ReduceScatterOp.apply(x, group)


def mark_as_sequence_parallel_parameter(parameter):
    parameter.sequence_parallel = True


# the overlapped sequence-parallel linears and token-block collectives (parallel/sequence_parallel.py)
from ....parallel.sequence_parallel import (column_sp_linear, row_sp_linear, gather_tokens,  # noqa: E402,F401
                                            reduce_scatter_tokens, allreduce_sequence_parallel_grads)


def is_sequence_parallel_parameter(parameter):
    return getattr(parameter, "sequence_parallel", False)


def register_sequence_parallel_allreduce_hooks(model, accumulation_steps=1, fuse_sequence_parallel_allreduce=False):
    """LayerNorm / bias params that see only a sequence shard get their grads all-reduced over mp."""
    g = tp._mp_group()
    if tp._ws(g) == 1:
        return
    for p in model.parameters():
        if is_sequence_parallel_parameter(p):
            def hook(t, _g=g):
                dist.all_reduce(t.grad, group=_g.process_group)
            p._t.register_post_accumulate_grad_hook(hook)
            p._sp_hooked = True  # the optimizer-side flat all-reduce skips it


class ColumnSequenceParallelLinear(nn.Layer):
    """all-gather the sequence shard, then a column-parallel GEMM."""

    def __init__(self, in_features, out_features, weight_attr=None, has_bias=None, gather_output=False,
                 fuse_matmul_bias=False, mp_group=None, name=None):
        super().__init__()
        self.group = _g(mp_group)
        n = tp._ws(self.group)
        self.weight = self.create_parameter([in_features, out_features // n], attr=weight_attr)
        self.weight.is_distributed = n > 1
        self.bias = self.create_parameter([out_features // n], is_bias=True) if has_bias in (None, True) else None

    def forward(self, x):
        # all-gather of the sequence blocks overlapped with the GEMM of this rank's own block
        return _wrap(column_sp_linear(x._t, self.weight._t, None if self.bias is None else self.bias._t,
                                      group=self.group))


class RowSequenceParallelLinear(nn.Layer):
    """row-parallel GEMM followed by a reduce-scatter back to sequence shards."""

    def __init__(self, in_features, out_features, weight_attr=None, has_bias=True, input_is_parallel=True,
                 fuse_matmul_bias=False, mp_group=None, name=None):
        super().__init__()
        self.group = _g(mp_group)
        n = tp._ws(self.group)
        self.weight = self.create_parameter([in_features // n, out_features], attr=weight_attr)
        self.weight.is_distributed = n > 1
        self.bias = self.create_parameter([out_features], is_bias=True) if has_bias else None
        if self.bias is not None:
            mark_as_sequence_parallel_parameter(self.bias)

    def forward(self, x):
        y = row_sp_linear(x._t, self.weight._t, group=self.group)  # GEMM pipelined with the block reduces
        if self.bias is not None:
            y = y + self.bias._t
        return _wrap(y)
