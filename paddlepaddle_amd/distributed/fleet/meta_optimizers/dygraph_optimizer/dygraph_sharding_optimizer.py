"""DygraphShardingOptimizer (sharding stage 1 by parameter ownership) and DygraphShardingOptimizerV2 (stage 1 by
flat-buffer slices). Reference: python/paddle/distributed/fleet/meta_optimizers/dygraph_optimizer/
dygraph_sharding_optimizer.py (:54 V1, :586 V2).

V1: every parameter is owned by one sharding rank (greedy by size, largest first, as the reference's default
partition); the inner optimizer holds only the owned parameters, so its moments / master weights exist once per
group. reduce_gradients averages each gradient onto its owner — bucketed by (owner, dtype): one RCCL reduce per
bucket instead of one per parameter — and step() updates the owned parameters, then broadcasts every parameter
from its owner (bucketed the same way).

V2: the parameters of one dtype are laid out in one flat buffer padded to a multiple of the sharding degree; rank r
owns slice r. Gradients accumulate into a flat gradient buffer (each .grad is a view of it), reduce_gradients is one
reduce-scatter per buffer into the slice gradient, the inner optimizer steps one slice Parameter per buffer, and one
all-gather per buffer brings the parameters back. (The same layout as the flat-buffer ZeRO engine,
parallel/sharding.py, which fleet.distributed_model uses for sharding_degree > 1.)

The global-norm clip of the inner optimizer is made group-wide: sums of squares of the owned gradients (V1) /
slices (V2) are all-reduced over the sharding group.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .....framework.tensor import Parameter, Tensor
from ...utils.hybrid_parallel_util import obtain_optimizer_parameters_list


def _pg(group):
    return None if group is None else getattr(group, "process_group", group)


def _numel(p):
    return int(p._t.numel())


def _set_group_clip(opt, group, local_params_fn):
    clip = getattr(opt, "_grad_clip", None)
    if clip is None or not hasattr(clip, "_extra_sq_norm_fn") or group is None or group.nranks <= 1:
        return

    def _param_sq(params):
        from .....ops.optim import global_sq_norm
        ps = local_params_fn(params)
        gs = [p._t.grad for p in ps if p._t.grad is not None]
        dev = gs[0].device if gs else (params[0]._t.device if params else torch.device("cpu"))
        sq = (global_sq_norm(gs) if gs else torch.zeros((), device=dev)).reshape(1).float().clone()
        dist.all_reduce(sq, group=_pg(group))
        return sq[0]
    clip._param_sq_fn = _param_sq


class DygraphShardingOptimizer:
    def __init__(self, optimizer, hcg):
        plist = getattr(optimizer, "_parameter_list", None) or []
        if plist and isinstance(plist[0], dict):
            raise TypeError("DygraphShardingOptimizer does not take param_groups; pass a list of Parameters")
        self._inner_opt = optimizer
        self._hcg = hcg
        self._parameter_list = list(plist)
        self._origin_parameter_list = self._parameter_list
        self._group = hcg.get_sharding_parallel_group()
        self._sharding_world_size = hcg.get_sharding_parallel_world_size()
        self._sharding_rank = hcg.get_sharding_parallel_rank()
        self._rank2params = self._partition_parameters()
        self._param2rank = {id(p): r for r, ps in self._rank2params.items() for p in ps}
        local = self._rank2params[self._sharding_rank]
        optimizer._parameter_list = list(local)
        optimizer._param_groups = [{"params": list(local)}]
        own = {id(p) for p in local}
        _set_group_clip(optimizer, self._group, lambda ps: [p for p in ps if id(p) in own])

    def _partition_parameters(self):
        mapping = {r: [] for r in range(self._sharding_world_size)}
        sizes = [0] * self._sharding_world_size
        for p in sorted(self._parameter_list, key=_numel, reverse=True):
            r = sizes.index(min(sizes))
            mapping[r].append(p)
            sizes[r] += _numel(p)
        return mapping

    def filter_parameters(self, parameter_list, hcg):
        r = hcg.get_sharding_parallel_rank()
        return [p for p in parameter_list if self._param2rank.get(id(p)) == r]

    @staticmethod
    def _grad(p):
        mg = getattr(p, "main_grad", None)
        if mg is not None:
            return mg._t if isinstance(mg, Tensor) else mg
        return p._t.grad

    def _buckets(self, params, with_grads):
        by = {}
        for p in params:
            t = self._grad(p) if with_grads else p._t
            if t is None:
                continue
            by.setdefault((self._param2rank[id(p)], t.dtype, t.device), []).append(t)
        return by

    @torch.no_grad()
    def reduce_gradients(self, parameter_list, hcg):
        """Average every gradient onto the rank that owns its parameter (one reduce per (owner, dtype) bucket)."""
        n = self._sharding_world_size
        if n <= 1:
            return
        pg = _pg(self._group)
        for (owner, _dt, _dev), ts in self._buckets(parameter_list, True).items():
            flat = torch.cat([t.reshape(-1) for t in ts])
            flat.mul_(1.0 / n)
            dist.reduce(flat, self._group.ranks[owner], group=pg)
            o = 0
            for t in ts:
                k = t.numel()
                t.copy_(flat[o:o + k].view_as(t))
                o += k

    @torch.no_grad()
    def _sharding_sync_parameters(self):
        if self._sharding_world_size <= 1:
            return
        pg = _pg(self._group)
        for (owner, _dt, _dev), ts in self._buckets(self._parameter_list, False).items():
            flat = torch.cat([t.detach().reshape(-1) for t in ts])
            dist.broadcast(flat, self._group.ranks[owner], group=pg)
            o = 0
            for t in ts:
                k = t.numel()
                t.data.copy_(flat[o:o + k].view_as(t))
                o += k

    def step(self):
        self._inner_opt.step()
        self._sharding_sync_parameters()

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        loss.backward()
        self.reduce_gradients(self._parameter_list, self._hcg)
        self.step()

    def clear_grad(self, set_to_zero=True):
        for p in self._parameter_list:
            if getattr(p, "main_grad", None) is not None:
                if set_to_zero:
                    p.main_grad._t.zero_()
                else:
                    p.main_grad = None
            if p._t.grad is not None:
                if set_to_zero:
                    p._t.grad.zero_()
                else:
                    p._t.grad = None

    clear_gradients = clear_grad

    def state_dict(self):
        return self._inner_opt.state_dict()

    def set_state_dict(self, state_dict):
        return self._inner_opt.set_state_dict(state_dict)

    def __getattr__(self, item):
        return getattr(self._inner_opt, item)


class DygraphShardingOptimizerV2:
    def __init__(self, optimizer, hcg):
        self._inner_opt = optimizer
        self._hcg = hcg
        self._parameter_list = obtain_optimizer_parameters_list(optimizer)
        self._group = hcg.get_sharding_parallel_group()
        self._n = hcg.get_sharding_parallel_world_size()
        self._rank = hcg.get_sharding_parallel_rank()
        self._buffers = []
        by = {}
        for p in self._parameter_list:
            if p._t.requires_grad:
                by.setdefault((p._t.dtype, p._t.device), []).append(p)
        slices = []
        for (dt, dev), ps in by.items():
            total = sum(_numel(p) for p in ps)
            C = -(-total // self._n)
            flat = torch.zeros(C * self._n, dtype=dt, device=dev)
            gflat = torch.zeros(C * self._n, dtype=dt, device=dev)
            o = 0
            for p in ps:
                k = _numel(p)
                flat[o:o + k].copy_(p._t.detach().reshape(-1))
                v = flat[o:o + k].view(p._t.shape).requires_grad_(True)
                from .....framework.tensor import _PARAM_OF
                _PARAM_OF.pop(id(p._t), None)
                _PARAM_OF[id(v)] = p
                p._t = v
                v.grad = gflat[o:o + k].view(v.shape)  # autograd accumulates into the flat gradient
                o += k
            sp = Parameter(flat[self._rank * C:(self._rank + 1) * C], name=f"sharding_v2_slice_{len(self._buffers)}")
            sp._t = flat[self._rank * C:(self._rank + 1) * C]  # a view: the update lands in the parameters
            sp._t.requires_grad_(True)
            self._buffers.append({"flat": flat, "gflat": gflat, "C": C, "params": ps, "slice": sp,
                                  "sgrad": torch.empty(C, dtype=dt, device=dev)})
            slices.append(sp)
        optimizer._parameter_list = slices
        optimizer._param_groups = [{"params": slices}]
        _set_group_clip(optimizer, self._group, lambda ps: ps)

    @torch.no_grad()
    def reduce_gradients(self, parameter_list, hcg):
        """One reduce-scatter per flat buffer: slice r of the averaged gradient lands on sharding rank r."""
        for b in self._buffers:
            g = b["gflat"]
            if self._n > 1:
                g.mul_(1.0 / self._n)
                dist.reduce_scatter_tensor(b["sgrad"], g, group=_pg(self._group))
            else:
                b["sgrad"].copy_(g)
            b["slice"]._t.grad = b["sgrad"]

    @torch.no_grad()
    def _sharding_sync_parameters(self):
        for b in self._buffers:
            if self._n > 1:
                dist.all_gather_into_tensor(b["flat"], b["slice"]._t.detach().clone(), group=_pg(self._group))

    def step(self):
        if any(b["slice"]._t.grad is None for b in self._buffers):
            self.reduce_gradients(self._parameter_list, self._hcg)
        self._inner_opt.step()
        self._sharding_sync_parameters()
        for b in self._buffers:
            b["slice"]._t.grad = None

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        loss.backward()
        self.reduce_gradients(self._parameter_list, self._hcg)
        self.step()

    def clear_grad(self, set_to_zero=True):
        for b in self._buffers:
            b["gflat"].zero_()
            b["slice"]._t.grad = None
            for p in b["params"]:  # keep .grad the flat buffer's view
                k = p._t.numel()
                if p._t.grad is None or p._t.grad.data_ptr() < b["gflat"].data_ptr() or \
                        p._t.grad.data_ptr() >= b["gflat"].data_ptr() + b["gflat"].numel() * b["gflat"].element_size():
                    off = self._offset(b, p)
                    p._t.grad = b["gflat"][off:off + k].view(p._t.shape)

    clear_gradients = clear_grad

    @staticmethod
    def _offset(b, p):
        o = 0
        for q in b["params"]:
            if q is p:
                return o
            o += q._t.numel()
        raise KeyError(p)

    def state_dict(self):
        return self._inner_opt.state_dict()

    def set_state_dict(self, state_dict):
        return self._inner_opt.set_state_dict(state_dict)

    def __getattr__(self, item):
        return getattr(self._inner_opt, item)


__all__ = ["DygraphShardingOptimizer", "DygraphShardingOptimizerV2"]
