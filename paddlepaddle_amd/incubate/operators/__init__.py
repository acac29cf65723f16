"""paddle.incubate.operators. Reference: python/paddle/incubate/operators/__init__.py (graph_* ops,
softmax_mask_fuse(_upper_triangle), ResNetUnit)."""
from __future__ import annotations

import torch

from ...framework.tensor import Tensor, _wrap  # noqa: F401
from ...geometric import sample_neighbors as graph_sample_neighbors, reindex_graph as graph_reindex  # noqa: F401
from ...geometric import send_u_recv as _send_u_recv
from .resnet_unit import ResNetUnit, resnet_unit  # noqa: F401


def graph_send_recv(x, src_index, dst_index, pool_type="sum", out_size=None, name=None):
    return _send_u_recv(x, src_index, dst_index, pool_type, out_size)


def graph_khop_sampler(row, colptr, input_nodes, sample_sizes, sorted_eids=None, return_eids=False, name=None):
    from ...geometric import sample_neighbors, reindex_graph
    nodes = input_nodes
    all_src, all_dst = [], []
    frontier = input_nodes
    for k in sample_sizes:
        nb, cnt = sample_neighbors(row, colptr, frontier, k)[:2]
        all_src.append(nb)
        all_dst.append(torch.repeat_interleave(frontier._t, cnt._t.long()))
        frontier = _wrap(torch.unique(nb._t))
    src = torch.cat([s._t for s in all_src])
    dst = torch.cat(all_dst)
    uniq, inv = torch.unique(torch.cat([input_nodes._t, src, dst]), return_inverse=True)
    n0 = input_nodes._t.numel()
    es = inv[n0:n0 + src.numel()]
    ed = inv[n0 + src.numel():]
    return _wrap(es), _wrap(ed), _wrap(uniq), _wrap(inv[:n0])


def softmax_mask_fuse(x, mask, name=None):
    """softmax(x + mask) over the last axis (fused HIP softmax)."""
    from ... import ops
    return _wrap(ops.softmax(x._t + mask._t.to(x._t.dtype), -1))


def softmax_mask_fuse_upper_triangle(x):
    """Causal softmax: entries above the diagonal of the last two axes are masked."""
    from ... import ops
    t = x._t
    S, T = t.shape[-2], t.shape[-1]
    m = torch.ones(S, T, dtype=torch.bool, device=t.device).triu(T - S + 1)
    return _wrap(ops.softmax(t.masked_fill(m, float("-inf")), -1))
