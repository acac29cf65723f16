"""Segment (sequence / context) parallelism: every rank of the ``sep`` group holds the same parameters and
one contiguous segment of each sequence.

Reference: python/paddle/distributed/fleet/meta_parallel/segment_parallel.py:26 (SegmentParallel: broadcast
parameters over the sep / sharding / dp groups), fleet/utils/hybrid_parallel_util.py:249
(fused_allreduce_gradients: gradients summed over the sep group — "sep all reduce is not scaled" — and
averaged over dp, through the fused dp x sep group).

Attention across segments (MI355X design): Ulysses-style head/sequence exchange. Before attention one
all-to-all turns [B, S/P, H, D] segments into [B, S, H/P, D] (every rank gets the full sequence for 1/P of the
heads), the HIP flash-attention kernel runs causally over the whole sequence, and the inverse all-to-all
brings the output back to [B, S/P, H, D]. On an 8-GPU xGMI node every rank pair has its own link, so each
exchange is one hop per pair and moves 3 (+1) x B*S*H*D/P elements per rank — no ring of K/V blocks.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..autograd.engine import queue_callback as _queue_callback
from .. import nn
from ..distributed import collective as C
from ..framework.tensor import Tensor, _wrap


def _pg(group):
    return group.process_group if group is not None else None


def _a2a(x, group):
    out = torch.empty_like(x)
    dist.all_to_all_single(out, x, group=_pg(group))
    return out


class _SeqToHead(torch.autograd.Function):
    """[B, S/P, H, D] (my segment, all heads) -> [B, S, H/P, D] (all segments, my heads)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        P = group.nranks
        B, S, H, D = x.shape
        xs = x.reshape(B, S, P, H // P, D).permute(2, 0, 1, 3, 4).contiguous()  # chunk p -> rank p
        out = _a2a(xs, group)                                                   # [P(src segment), B, S, H/P, D]
        return out.permute(1, 0, 2, 3, 4).reshape(B, P * S, H // P, D)

    @staticmethod
    def backward(ctx, g):
        return _HeadToSeq.apply(g.contiguous(), ctx.group), None


class _HeadToSeq(torch.autograd.Function):
    """[B, S, H/P, D] (all segments, my heads) -> [B, S/P, H, D] (my segment, all heads)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        P = group.nranks
        B, S, Hl, D = x.shape
        xs = x.reshape(B, P, S // P, Hl, D).permute(1, 0, 2, 3, 4).contiguous()  # segment p -> rank p
        out = _a2a(xs, group)                                                    # [P(src head group), B, S/P, Hl, D]
        return out.permute(1, 2, 0, 3, 4).reshape(B, S // P, P * Hl, D)

    @staticmethod
    def backward(ctx, g):
        return _SeqToHead.apply(g.contiguous(), ctx.group), None


def seq_to_head(x, group):
    return _SeqToHead.apply(x, group) if group is not None and group.nranks > 1 else x


def head_to_seq(x, group):
    return _HeadToSeq.apply(x, group) if group is not None and group.nranks > 1 else x


def segment_attention(q, k, v, group, causal=True, scale=None):
    """Attention over the full sequence for segment-sharded q / k / v [B, S/P, H(kv), D] (torch tensors)."""
    from ..ops import attention as A
    if group is None or group.nranks == 1:
        return A.attention(q, k, v, causal=causal, scale=scale)
    P = group.nranks
    if q.shape[2] % P or k.shape[2] % P:
        raise ValueError(f"heads ({q.shape[2]}, kv {k.shape[2]}) must be divisible by the sep degree {P}")
    o = A.attention(seq_to_head(q, group), seq_to_head(k, group), seq_to_head(v, group), causal=causal, scale=scale)
    return head_to_seq(o, group)


def split_sequence(x, group, axis=1):
    """This rank's contiguous segment of ``x`` along ``axis``."""
    t = x._t if isinstance(x, Tensor) else x
    if group is None or group.nranks == 1:
        return x
    seg = t.chunk(group.nranks, axis)[group.rank]
    return _wrap(seg.contiguous()) if isinstance(x, Tensor) else seg.contiguous()


class SegmentParallel(nn.Layer):
    """Wraps a model for sep (x dp) training: parameters broadcast over the sep and dp groups; after
    backward, gradients are all-reduced over the fused dp x sep group in ~bucket_mb buckets (summed over sep,
    averaged over dp — reference fused_allreduce_gradients)."""

    def __init__(self, layers, hcg, strategy=None, bucket_mb=256):
        super().__init__()
        self._layers = layers
        self._hcg = hcg
        self._bucket = int(bucket_mb) << 20
        sep = hcg.get_sep_parallel_group()
        dp_n = hcg.get_data_parallel_world_size()
        with torch.no_grad():
            for g in (sep, hcg.get_data_parallel_group() if dp_n > 1 else None):
                if g is not None and g.nranks > 1:
                    for p in layers.parameters():
                        dist.broadcast(p._t.data, g.ranks[0], group=g.process_group)
        self._group = hcg.get_dp_sep_parallel_group()
        self._scale = 1.0 / dp_n
        self._queued = False
        for p in layers.parameters():
            if not p.stop_gradient:
                p._t.register_post_accumulate_grad_hook(self._on_grad)

    def _on_grad(self, t):
        if not self._queued:
            self._queued = True
            _queue_callback(self._sync)

    @torch.no_grad()
    def _sync(self):
        self._queued = False
        g = self._group
        if g is None or g.nranks <= 1:
            return
        grads = [p._t.grad for p in self._layers.parameters() if p._t.grad is not None]
        bucket, size = [], 0
        for gr in grads + [None]:
            if gr is not None:
                bucket.append(gr)
                size += gr.numel() * gr.element_size()
            if bucket and (gr is None or size >= self._bucket):
                flat = torch.cat([b.reshape(-1) for b in bucket])
                dist.all_reduce(flat, group=g.process_group)
                if self._scale != 1.0:
                    flat.mul_(self._scale)
                off = 0
                for b in bucket:
                    n = b.numel()
                    b.copy_(flat[off:off + n].view_as(b))
                    off += n
                bucket, size = [], 0

    def forward(self, *a, **k):
        return self._layers(*a, **k)

    def state_dict(self, *a, **k):
        return self._layers.state_dict(*a, **k)

    def set_state_dict(self, sd, use_structured_name=True):
        return self._layers.set_state_dict(sd, use_structured_name)

    def parameters(self, include_sublayers=True):
        return self._layers.parameters(include_sublayers)

    def named_parameters(self, prefix="", include_sublayers=True, remove_duplicate=True):
        return self._layers.named_parameters(prefix, include_sublayers, remove_duplicate)
