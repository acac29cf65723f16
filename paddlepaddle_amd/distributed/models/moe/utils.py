"""MoE routing helpers. Reference: python/paddle/distributed/models/moe/utils.py (_number_count, _assign_pos,
_random_routing, _limit_by_capacity, _prune_gate_by_capacity)."""
from __future__ import annotations

import torch

from ....framework.tensor import Tensor, _wrap


def _t(x):
    return x._t if isinstance(x, Tensor) else x


def _number_count(numbers, upper_range):
    """Count of every value in [0, upper_range) (values outside are ignored)."""
    n = _t(numbers).reshape(-1).long()
    n = n[(n >= 0) & (n < upper_range)]
    return _wrap(torch.bincount(n, minlength=upper_range).to(torch.int64))


def _assign_pos(x, cum_count):
    """Positions of the tokens grouped by expert: out[cum_count[e - 1] .. cum_count[e]) are the indices i with
    x[i] == e (in the reference op's order: last occurrence first within an expert)."""
    xv = _t(x).reshape(-1).long()
    cc = _t(cum_count).reshape(-1).long()
    out = torch.empty(int(cc[-1].item()) if cc.numel() else 0, dtype=torch.int64, device=xv.device)
    fill = cc.clone()
    for i in range(xv.numel() - 1, -1, -1):
        e = int(xv[i])
        if e < 0:
            continue
        fill[e] -= 1
        out[int(fill[e])] = i
    return _wrap(out)


def _random_routing(topk_idx, topk_value, prob, topk=2):
    """Top-2 random routing: the second expert is dropped (-1) where 2 * value < prob."""
    if topk != 2:
        raise RuntimeError("only topk=2 is supported now")
    idx = _t(topk_idx).clone()
    keep = 2 * _t(topk_value)[:, 1] >= _t(prob).reshape(-1)
    idx[:, 1] = torch.where(keep, idx[:, 1], torch.full_like(idx[:, 1], -1))
    return _wrap(idx)


def _limit_by_capacity(expert_count, capacity, n_worker):
    """Per (worker, expert) counts clipped so every expert's total stays within its capacity, workers served in
    order."""
    ec = _t(expert_count).reshape(n_worker, -1).long()
    cap = _t(capacity).reshape(-1).long().clone()
    out = torch.zeros_like(ec)
    for w in range(n_worker):
        take = torch.minimum(ec[w], cap)
        out[w] = take
        cap -= take
    return _wrap(out.reshape(-1))


def _prune_gate_by_capacity(gate_idx, expert_count, n_expert, n_worker):
    """Tokens beyond their expert's remaining count get gate -1 (in token order)."""
    g = _t(gate_idx).reshape(-1).long().clone()
    left = _t(expert_count).reshape(-1).long().clone()
    for i in range(g.numel()):
        e = int(g[i])
        if e < 0:
            continue
        if left[e] > 0:
            left[e] -= 1
        else:
            g[i] = -1
    return _wrap(g)
