"""fleet.utils.tensor_fusion_helper: flat parameter / gradient storage and fused communication buffers.
Reference: python/paddle/distributed/fleet/utils/tensor_fusion_helper.py (assign_group_by_size :76,
flatten_dense_tensors :99, FusedCommBuffer :384, fused_parameters :925).

Parameters of one dtype are packed into one flat buffer (each parameter a view at a 256-byte aligned offset), their
gradients into a second one (fp32 with main_grad), so a data-parallel / sharding reduction of a whole group is one
collective. A FusedCommBuffer counts the gradients that arrive from backward (``add_grad``) and launches its
collective on the RCCL stream once every parameter has checked in ``acc_steps`` times (overlapped with the rest of
the backward); ``scale_grads`` waits for it and applies the 1 / nranks scale.
"""
from __future__ import annotations

import builtins
import collections

import torch
import torch.distributed as dist

from ....framework.tensor import Parameter, Tensor, _wrap


class HOOK_ACTION:
    ALL_REDUCE = 0
    REDUCE = 1
    REDUCE_SCATTER = 2


_ALIGN_BYTES = 256


def _numel(p):
    return int(p._t.numel())


def assign_group_by_size(parameters, group_size=128 * 1024 * 1024):
    """OrderedDict group index -> parameters: consecutive same-dtype parameters up to ``group_size`` bytes."""
    groups = collections.OrderedDict()
    cur, cur_bytes, cur_dt, gi = [], 0, None, 0
    for p in parameters:
        nb = _numel(p) * p._t.element_size()
        if cur and (p._t.dtype != cur_dt or cur_bytes + nb > group_size):
            groups[gi] = cur
            gi += 1
            cur, cur_bytes = [], 0
        cur.append(p)
        cur_bytes += nb
        cur_dt = p._t.dtype
    if cur:
        groups[gi] = cur
    return groups


def _offsets(parameters, elem):
    offs, o = {}, 0
    for p in parameters:
        offs[id(p)] = o
        k = _numel(p)
        pad = (-(k * elem)) % _ALIGN_BYTES // elem
        o += k + pad
    return offs, o


def flatten_dense_tensors(parameters, use_main_grad=False, fuse_param=True, warp_buffer=False, release_grad=False):
    """Pack ``parameters`` (one dtype) into flat storage: returns (param_storage, grad_storage) flat tensors (each
    parameter / gradient a view into them); release_grad: (None, buffer_size, {param name: offset})."""
    dt = parameters[0]._t.dtype
    dev = parameters[0]._t.device
    offs, size = _offsets(parameters, parameters[0]._t.element_size())
    if release_grad:
        return None, size, {p.name: offs[id(p)] for p in parameters}
    pstore = None
    if fuse_param:
        pstore = torch.zeros(size, dtype=dt, device=dev)
        from ....framework.tensor import _PARAM_OF
        for p in parameters:
            o, k = offs[id(p)], _numel(p)
            pstore[o:o + k].copy_(p._t.detach().reshape(-1))
            v = pstore[o:o + k].view(p._t.shape).requires_grad_(p._t.requires_grad)
            _PARAM_OF.pop(id(p._t), None)
            _PARAM_OF[id(v)] = p
            p._t = v
    gstore = torch.zeros(size, dtype=torch.float32 if use_main_grad else dt, device=dev)
    for p in parameters:
        o, k = offs[id(p)], _numel(p)
        view = gstore[o:o + k].view(p._t.shape)
        if use_main_grad:
            p.main_grad = _wrap(view)
        else:
            p._t.grad = view
    return pstore, gstore


class FusedCommBuffer:
    def __init__(self, id, params, comm_group, acc_steps=1, act=None, dst=-1, use_main_grad=None, fuse_param=False,
                 scale_after_comm=True, release_grads=False, use_reduce_avg=False, free_grads_in_comm=False):
        if act not in (HOOK_ACTION.ALL_REDUCE, HOOK_ACTION.REDUCE, HOOK_ACTION.REDUCE_SCATTER):
            raise ValueError("FusedCommBuffer act must be ALL_REDUCE, REDUCE or REDUCE_SCATTER")
        if act == HOOK_ACTION.REDUCE and dst == -1:
            raise ValueError("FusedCommBuffer REDUCE needs a dst rank")
        self._id, id = id, builtins.id  # the reference's parameter name shadows the builtin
        self._params = list(params)
        self._comm_group = comm_group
        self._acc_steps = int(acc_steps)
        self._act = act
        self._dst = dst
        self._scale_after_comm = scale_after_comm
        self.use_main_grad = use_main_grad if use_main_grad is not None else hasattr(self._params[0], "main_grad")
        self._nranks = comm_group.nranks if comm_group is not None else (dist.get_world_size()
                                                                         if dist.is_initialized() else 1)
        self.param_storage, self.grad_storage = flatten_dense_tensors(self._params, self.use_main_grad, fuse_param)
        self._task = None
        self._steps = {id(p): 0 for p in self._params}
        self._checked_in = 0
        if act == HOOK_ACTION.REDUCE_SCATTER:
            n = self._nranks
            pad = (-self.grad_storage.numel()) % n
            if pad:
                self.grad_storage = torch.cat([self.grad_storage, self.grad_storage.new_zeros(pad)])
                self._rebind_grads()
            self._shard = self.grad_storage.new_empty(self.grad_storage.numel() // n)

    def _rebind_grads(self):
        offs, _ = _offsets(self._params, self._params[0]._t.element_size())
        for p in self._params:
            o, k = offs[id(p)], _numel(p)
            view = self.grad_storage[o:o + k].view(p._t.shape)
            if self.use_main_grad:
                p.main_grad = _wrap(view)
            else:
                p._t.grad = view

    @property
    def _pg(self):
        return getattr(self._comm_group, "process_group", self._comm_group)

    def add_grad(self, param, use_comm=True):
        """Called once per backward per parameter (e.g. from a post-accumulate hook); the collective starts when
        every parameter of the buffer has checked in acc_steps times."""
        self._steps[id(param)] += 1
        if self._steps[id(param)] == self._acc_steps:
            self._checked_in += 1
        if self._checked_in == len(self._params):
            if use_comm:
                self.comm_grads()
            for k in self._steps:
                self._steps[k] = 0
            self._checked_in = 0

    @torch.no_grad()
    def comm_grads(self):
        g = self.grad_storage
        if not self._scale_after_comm:
            g.mul_(1.0 / self._nranks)
        if self._nranks <= 1:
            self._task = None
            return
        if self._act == HOOK_ACTION.ALL_REDUCE:
            self._task = dist.all_reduce(g, group=self._pg, async_op=True)
        elif self._act == HOOK_ACTION.REDUCE:
            self._task = dist.reduce(g, self._dst, group=self._pg, async_op=True)
        else:
            self._task = dist.reduce_scatter_tensor(self._shard, g, group=self._pg, async_op=True)

    @torch.no_grad()
    def scale_grads(self):
        if self._task is not None:
            self._task.wait()
            self._task = None
        if self._scale_after_comm:
            target = self._shard if self._act == HOOK_ACTION.REDUCE_SCATTER else self.grad_storage
            target.mul_(1.0 / self._nranks)

    def sharded_grad(self):
        return self._shard if self._act == HOOK_ACTION.REDUCE_SCATTER else self.grad_storage


def filter_params(params, is_fp32, is_distributed, need_clip):
    return [p for p in params if (p._t.dtype == torch.float32) == is_fp32
            and bool(getattr(p, "is_distributed", False)) == is_distributed
            and bool(getattr(p, "need_clip", True)) == need_clip]


def fused_parameters(parameters, use_main_grad=False, fuse_param=True, comm_overlap=False, comm_group=None, act=None,
                     dst=-1, acc_step=1, scale_after_comm=False, group_params=False, apply_decay_param_fun=None,
                     use_reduce_avg=False, group_size=256 * 1024 * 1024):
    """Fuse the parameters (and their gradients) group by group. Returns (decay_fused, all_fused, comm_buffers):
    a fused stand-in Parameter per group (its storage is the flat parameter buffer), the decay subset of them
    (``apply_decay_param_fun`` on the member names), and FusedCommBuffers when comm_overlap is on."""
    act = HOOK_ACTION.REDUCE if act is None else act
    if group_params:
        raise NotImplementedError("fused_parameters(group_params=True)")
    decay_fused, all_fused, buffers = [], [], []
    groups = []
    for dec in (True, False):
        sel = [p for p in parameters if apply_decay_param_fun is None or bool(apply_decay_param_fun(p.name)) == dec]
        if apply_decay_param_fun is None and not dec:
            break
        for g in assign_group_by_size(sel, group_size).values():
            groups.append((dec, g))
    for i, (dec, g) in enumerate(groups):
        if comm_overlap:
            buf = FusedCommBuffer(i, g, comm_group, acc_step, act, dst, use_main_grad, fuse_param, scale_after_comm)
            buffers.append(buf)
            pstore = buf.param_storage
        else:
            pstore, _ = flatten_dense_tensors(g, use_main_grad, fuse_param)
        if pstore is None:
            continue
        fp = Parameter(pstore, name=f"fused_param_{i}")
        fp._t = pstore
        all_fused.append(fp)
        if dec:
            decay_fused.append(fp)
    return decay_fused, all_fused, buffers


__all__ = ["HOOK_ACTION", "assign_group_by_size", "flatten_dense_tensors", "FusedCommBuffer", "fused_parameters",
           "filter_params"]
del Tensor
