"""fleet.utils.hybrid_parallel_util: gradient and parameter synchronisation helpers of hybrid-parallel dygraph
training. Reference: python/paddle/distributed/fleet/utils/hybrid_parallel_util.py (fused_allreduce_gradients
:249, broadcast_mp_parameters :213, broadcast_dp_parameters :225, broadcast_sharding_parameters :273,
broadcast_sep_parameters :287, broadcast_input_data :168).

Gradients are all-reduced in flat per-dtype buckets (``bucket_size`` bytes, default 128 MiB: few large RCCL
collectives over xGMI rather than one per parameter), each bucket scaled by 1 / nranks once; ``main_grad`` (fp32
master gradients of MixPrecisionLayer / fused gradient accumulation) is used where a parameter has one.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ....framework.tensor import Tensor, _wrap

_BUCKET = 128 * 1024 * 1024


def obtain_optimizer_parameters_list(optimizer):
    """Every parameter the optimizer updates (param groups flattened)."""
    plist = getattr(optimizer, "_parameter_list", None) or []
    if plist and isinstance(plist[0], dict):
        out = []
        for g in plist:
            out.extend(g["params"])
        return out
    return list(plist)


def _grad_of(p):
    mg = getattr(p, "main_grad", None)
    if mg is not None:
        return mg._t if isinstance(mg, Tensor) else mg
    return p._t.grad


def _pg(group):
    if group is None:
        return None
    return getattr(group, "process_group", group)


def _nranks(group):
    if group is None:
        return dist.get_world_size() if dist.is_initialized() else 1
    n = getattr(group, "nranks", None)
    return int(n) if n is not None else dist.get_world_size(group)


def _apply_collective_grads(parameters, comm_group, bucket_size=_BUCKET, scale=None):
    """All-reduce the parameters' gradients over ``comm_group`` in flat per-dtype buckets of about ``bucket_size``
    bytes (in reverse registration order, the order backward produces them), then multiply by ``scale`` (default
    1 / nranks). Gradients are copied back into their tensors."""
    n = _nranks(comm_group)
    if n <= 1 and scale is None:
        return
    scale = (1.0 / n) if scale is None else float(scale)
    grads = [g for g in (_grad_of(p) for p in reversed(list(parameters))) if g is not None]
    buckets, cur, cur_bytes = [], {}, {}
    for g in grads:
        dt = (g.dtype, g.device)
        cur.setdefault(dt, []).append(g)
        cur_bytes[dt] = cur_bytes.get(dt, 0) + g.numel() * g.element_size()
        if cur_bytes[dt] >= bucket_size:
            buckets.append(cur.pop(dt))
            cur_bytes[dt] = 0
    buckets.extend(v for v in cur.values() if v)
    pg = _pg(comm_group)
    with torch.no_grad():
        for b in buckets:
            flat = torch.cat([g.reshape(-1) for g in b]) if len(b) > 1 else b[0].reshape(-1).clone()
            if n > 1:
                dist.all_reduce(flat, group=pg)
            if scale != 1.0:
                flat.mul_(scale)
            o = 0
            for g in b:
                k = g.numel()
                g.copy_(flat[o:o + k].view_as(g))
                o += k


def fused_allreduce_gradients_with_group(parameter_list, group, bucket_size=_BUCKET, scale=None):
    _apply_collective_grads(parameter_list, group, bucket_size, scale)


def fused_allreduce_gradients(parameter_list, hcg):
    """Average the gradients over the data-parallel group (data x sep when sep parallelism is on)."""
    if hcg is None:
        group = None
    elif hcg.get_sep_parallel_world_size() > 1:
        group = hcg.get_dp_sep_parallel_group()
    else:
        group = hcg.get_data_parallel_group()
    _apply_collective_grads(parameter_list, group)


def sharding_reduce_gradients(parameter_list, hcg):
    """Average the gradients over the sharding group (every rank keeps the full averaged gradient)."""
    _apply_collective_grads(parameter_list, hcg.get_sharding_parallel_group())


def _broadcast_params(model, group, src_rank, skip_distributed, fuse_params=True):
    if group is None or _nranks(group) <= 1:
        return
    pg = _pg(group)
    tensors = []
    for p in model.parameters():
        if skip_distributed and getattr(p, "is_distributed", False):
            continue  # tensor-parallel shards differ by design
        tensors.append(p._t)
    for b in (model.buffers() if hasattr(model, "buffers") else []):
        t = getattr(b, "_t", b)
        if isinstance(t, torch.Tensor):
            tensors.append(t)
    with torch.no_grad():
        if not fuse_params:
            for t in tensors:
                dist.broadcast(t.data, src_rank, group=pg)
            return
        by = {}
        for t in tensors:
            by.setdefault((t.dtype, t.device), []).append(t)
        for ts in by.values():
            flat = torch.cat([t.detach().reshape(-1) for t in ts])
            dist.broadcast(flat, src_rank, group=pg)
            o = 0
            for t in ts:
                k = t.numel()
                t.data.copy_(flat[o:o + k].view_as(t))
                o += k


def sync_params_buffers(model, comm_group=None, src_rank=0, is_model_parallel=False, fuse_params=True):
    """Broadcast ``model``'s parameters and buffers from ``src_rank`` over ``comm_group`` (world when None), one
    flat broadcast per dtype when ``fuse_params``; with ``is_model_parallel`` the tensor-parallel shards
    (``is_distributed``) stay as they are (reference python/paddle/distributed/parallel.py sync_params_buffers)."""
    if comm_group is None:
        if not dist.is_initialized() or dist.get_world_size() <= 1:
            return
        from ...collective import _get_global_group
        comm_group = _get_global_group()
    _broadcast_params(model, comm_group, src_rank, is_model_parallel, fuse_params)


def broadcast_mp_parameters(model, hcg, fuse_params=True):
    g = hcg.get_model_parallel_group()
    _broadcast_params(model, g, hcg.get_model_parallel_group_src_rank(), True, fuse_params)


def broadcast_dp_parameters(model, hcg, fuse_params=True):
    g = hcg.get_data_parallel_group()
    _broadcast_params(model, g, hcg.get_data_parallel_group_src_rank(), False, fuse_params)


def broadcast_sharding_parameters(model, hcg, fuse_params=True):
    g = hcg.get_sharding_parallel_group()
    _broadcast_params(model, g, hcg.get_sharding_parallel_group_src_rank(), False, fuse_params)


def broadcast_sep_parameters(model, hcg, fuse_params=True):
    g = hcg.get_sep_parallel_group()
    _broadcast_params(model, g, hcg.get_sep_parallel_group_src_rank(), False, fuse_params)


def broadcast_input_data(hcg, *inputs, **kwargs):
    """Make the model-parallel ranks see the same batch: every tensor input is broadcast from the mp group's first
    rank (in place); returns (inputs, kwargs)."""
    g = hcg.get_model_parallel_group()
    if g is None or _nranks(g) <= 1:
        return inputs, kwargs
    src = hcg.get_model_parallel_group_src_rank()
    pg = _pg(g)

    def bc(v):
        t = v._t if isinstance(v, Tensor) else v
        if isinstance(t, torch.Tensor):
            dist.broadcast(t.data, src, group=pg)
        return v
    for v in inputs:
        bc(v)
    for v in kwargs.values():
        bc(v)
    return inputs, kwargs


def unwrap_optimizer(optimizer, optimizer_instances=()):
    """The innermost optimizer under wrappers (``_inner_opt`` chains) of the given classes."""
    opt = optimizer
    while isinstance(opt, tuple(optimizer_instances)) if optimizer_instances else hasattr(opt, "_inner_opt"):
        opt = opt._inner_opt
    return opt


__all__ = ["obtain_optimizer_parameters_list", "fused_allreduce_gradients", "fused_allreduce_gradients_with_group",
           "sharding_reduce_gradients", "broadcast_mp_parameters", "broadcast_dp_parameters",
           "broadcast_sharding_parameters", "broadcast_sep_parameters", "broadcast_input_data", "unwrap_optimizer"]
del _wrap
