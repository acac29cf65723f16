"""global_scatter / global_gather: the MoE token exchange. Reference: python/paddle/distributed/utils/moe_utils.py:20
(global_scatter), :153 (global_gather) and the global_scatter / global_gather ops.

x rows are grouped in blocks i = card * n_expert + expert (local_count[i] rows each, block order = index order).
global_scatter sends block (card j, expert e) to card j and returns the received rows ordered expert-major
(for e: for source card j: global_count[j * n_expert + e] rows) — the order the reference op produces. Here it is
one variable-split all_to_all_single over RCCL (or gloo); global_gather is its inverse."""
from __future__ import annotations

import torch
import torch.distributed as dist

from ...framework.tensor import Tensor, _wrap


def _t(x):
    return x._t if isinstance(x, Tensor) else x


def _pg(group):
    if group is None:
        return None
    return getattr(group, "process_group", None) or getattr(group, "_pg", None) or group


def _world(group):
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(_pg(group))


def _blocks(counts):
    offs = [0]
    for c in counts:
        offs.append(offs[-1] + int(c))
    return offs


def _exchange(rows, send_counts, recv_counts, n_expert, world, group, send_expert_major):
    """send_counts / recv_counts: [world * n_expert] (index j * n_expert + e)."""
    soff = _blocks(send_counts)
    # send layout: for every destination card j, its experts in order
    if send_expert_major:  # rows are ordered (e, j): block index in the row order is e * world + j
        order = [e * world + j for j in range(world) for e in range(n_expert)]
        sizes = [int(send_counts[j * n_expert + e]) for e in range(n_expert) for j in range(world)]
        soff = _blocks(sizes)
        pieces = [rows[soff[k]:soff[k + 1]] for k in order]
    else:
        pieces = [rows[soff[i]:soff[i + 1]] for i in range(world * n_expert)]
    send = torch.cat(pieces) if pieces else rows[:0]
    in_split = [sum(int(send_counts[j * n_expert + e]) for e in range(n_expert)) for j in range(world)]
    out_split = [sum(int(recv_counts[j * n_expert + e]) for e in range(n_expert)) for j in range(world)]
    recv = rows.new_empty((sum(out_split),) + tuple(rows.shape[1:]))
    if world == 1:
        recv.copy_(send)
    else:
        dist.all_to_all_single(recv, send.contiguous(), out_split, in_split, group=_pg(group))
    return recv


def global_scatter(x, local_count, global_count, group=None, use_calc_stream=True):
    t = _t(x)
    lc = _t(local_count).tolist()
    gc = _t(global_count).tolist()
    world = _world(group)
    n_expert = len(lc) // world
    recv = _exchange(t, lc, gc, n_expert, world, group, send_expert_major=False)
    # received: for source card j, its blocks for my experts e in order -> reorder to expert-major
    roff = _blocks([gc[j * n_expert + e] for j in range(world) for e in range(n_expert)])
    out = [recv[roff[j * n_expert + e]:roff[j * n_expert + e + 1]] for e in range(n_expert) for j in range(world)]
    return _wrap(torch.cat(out) if out else recv)


def global_gather(x, local_count, global_count, group=None, use_calc_stream=True):
    """Inverse of global_scatter: x holds the expert outputs in global_scatter's output order; each block goes back
    to the card it came from, and the result has global_scatter's input layout."""
    t = _t(x)
    lc = _t(local_count).tolist()
    gc = _t(global_count).tolist()
    world = _world(group)
    n_expert = len(lc) // world
    # send back: x is (e, j)-ordered with global_count sizes; destination j gets its experts in order
    recv = _exchange(t, gc, lc, n_expert, world, group, send_expert_major=True)
    return _wrap(recv)
