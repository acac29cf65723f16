"""Process groups and collectives.

Reference: python/paddle/distributed/communication/*.py, python/paddle/distributed/collective.py,
paddle/phi/core/distributed/nccl_comm_context.cc.

One process per GPU; backend "nccl" on a HIP build IS RCCL (rings over the xGMI point-to-point
links of the MI355X node); "gloo" on CPU. All collectives take/return paddle Tensors and operate
in place on their device buffers, like paddle's.
"""
from __future__ import annotations

import datetime
import os
import pickle

import numpy as np
import torch
import torch.distributed as dist

from ..framework.tensor import Tensor, _wrap


class ReduceOp:
    SUM = 0
    MAX = 1
    MIN = 2
    PROD = 3
    AVG = 4


_TORCH_OP = {ReduceOp.SUM: dist.ReduceOp.SUM, ReduceOp.MAX: dist.ReduceOp.MAX, ReduceOp.MIN: dist.ReduceOp.MIN,
             ReduceOp.PROD: dist.ReduceOp.PRODUCT, ReduceOp.AVG: dist.ReduceOp.AVG}


class Group:
    """A communication group (paddle.distributed.collective.Group)."""

    def __init__(self, rank_in_group, id, ranks, pg=None, name=None):  # noqa: A002 - reference keyword
        self.rank = rank_in_group
        self.id = id
        self.ranks = list(ranks)
        self.nranks = len(ranks)
        self.process_group = pg
        self.name = name

    @property
    def world_size(self):
        return self.nranks

    def is_member(self):
        return self.rank >= 0

    def get_group_rank(self, rank):
        return self.ranks.index(rank) if rank in self.ranks else -1

    @property
    def backend(self):
        return dist.get_backend(self.process_group) if self.process_group is not None else "gloo"

    def __repr__(self):
        return f"Group(rank={self.rank}, nranks={self.nranks}, id={self.id}, ranks={self.ranks})"


_groups = {}
_default_group = None
_next_gid = [1]


class _Task:
    def __init__(self, work=None, post=None):
        self._work = work
        self._post = post

    def wait(self):
        if self._work is not None:
            self._work.wait()
        if self._post is not None:
            self._post()
            self._post = None
        return True

    def is_completed(self):
        return self._work is None or self._work.is_completed()


def is_available():
    return dist.is_available()


def is_initialized():
    return dist.is_available() and dist.is_initialized()


def get_rank(group=None):
    if group is not None:
        return group.rank
    if is_initialized():
        return dist.get_rank()
    return int(os.environ.get("PADDLE_TRAINER_ID", os.environ.get("RANK", "0")))


def get_world_size(group=None):
    if group is not None:
        return group.nranks
    if is_initialized():
        return dist.get_world_size()
    return int(os.environ.get("PADDLE_TRAINERS_NUM", os.environ.get("WORLD_SIZE", "1")))


def get_backend(group=None):
    if not is_initialized():
        return None
    return dist.get_backend(None if group is None else group.process_group).upper()


class ParallelEnv:
    @property
    def rank(self):
        return get_rank()

    @property
    def world_size(self):
        return get_world_size()

    @property
    def local_rank(self):
        return int(os.environ.get("LOCAL_RANK", "0"))

    @property
    def nranks(self):
        return get_world_size()

    @property
    def device_id(self):
        return self.local_rank

    dev_id = device_id

    @property
    def trainer_endpoints(self):
        return os.environ.get("PADDLE_TRAINER_ENDPOINTS", "").split(",")

    @property
    def current_endpoint(self):
        return os.environ.get("PADDLE_CURRENT_ENDPOINT", "")


def init_parallel_env(backend=None, timeout_s=1800):
    """Initialise the default group from torchrun/paddle-launch environment variables."""
    global _default_group
    if _default_group is not None:
        return _default_group
    if "RANK" not in os.environ and "PADDLE_TRAINER_ID" in os.environ:
        os.environ["RANK"] = os.environ["PADDLE_TRAINER_ID"]
        os.environ["WORLD_SIZE"] = os.environ.get("PADDLE_TRAINERS_NUM", "1")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    use_gpu = torch.cuda.is_available() and os.environ.get("PADDLE_AMD_FORCE_CPU", "0") != "1"
    if backend is None or backend == "auto":
        backend = "nccl" if use_gpu else "gloo"
    backend = {"rccl": "nccl", "xccl": "nccl", "bkcl": "nccl"}.get(backend, backend)
    if use_gpu:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local % torch.cuda.device_count())
        from ..framework.place import set_device
        set_device(f"gpu:{local % torch.cuda.device_count()}")
    if not dist.is_initialized():
        kw = {}
        if backend == "nccl" and use_gpu:
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
        wd = os.environ.get("PADDLE_AMD_COMM_WATCHDOG")
        if wd:
            from .watchdog import enable_comm_watchdog
            enable_comm_watchdog(timeout_s=float(wd), report_dir=os.environ.get("PADDLE_AMD_COMM_WATCHDOG_DIR"))
        from .collective_check import maybe_enable_from_env
        maybe_enable_from_env()
    ws = dist.get_world_size()
    _default_group = Group(dist.get_rank(), 0, list(range(ws)), None, "_default_pg")
    _groups[0] = _default_group
    return _default_group


def _pg(group):
    if group is None:
        return None
    return group.process_group


def new_group(ranks=None, backend=None, timeout=None, nccl_comm_init_option=0):
    if not is_initialized():
        init_parallel_env()
    ws = dist.get_world_size()
    ranks = list(range(ws)) if ranks is None else sorted(ranks)
    kw = {}
    if timeout is not None:
        kw["timeout"] = timeout
    pg = dist.new_group(ranks=ranks, backend=backend if backend in ("gloo", "nccl") else None, **kw)
    me = dist.get_rank()
    gid = _next_gid[0]
    _next_gid[0] += 1
    g = Group(ranks.index(me) if me in ranks else -1, gid, ranks, pg)
    _groups[gid] = g
    return g


def get_group(id=0):
    return _groups.get(id)


def _get_global_group():
    if _default_group is None:
        init_parallel_env()
    return _default_group


def destroy_process_group(group=None):
    global _default_group
    if group is None:
        if dist.is_initialized():
            dist.destroy_process_group()
        _default_group = None
        _groups.clear()
    else:
        dist.destroy_process_group(group.process_group)
        _groups.pop(group.id, None)


def barrier(group=None):
    if is_initialized():
        if dist.get_backend(_pg(group)) == "nccl":
            dist.barrier(group=_pg(group), device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier(group=_pg(group))


def _ret(work, sync_op, post=None):
    if sync_op:
        if work is not None:
            work.wait()
        if post is not None:
            post()
        return None
    return _Task(work, post)


def _all_reduce_raw(t, op=ReduceOp.SUM, group=None, async_op=False):
    if not is_initialized() or get_world_size(group) == 1:
        return None
    return dist.all_reduce(t, op=_TORCH_OP[op], group=_pg(group), async_op=async_op)


def _static_comm(tensor, name, fn, meta=None):
    """Inside a static program being built: record the collective as one in-place "comm" node (replayed on
    the executor's communication stream, static/program.py _Streams). Returns True when recorded."""
    from ..framework.trace_hook import _active_program
    prog = _active_program()
    t = tensor._t if hasattr(tensor, "_t") else tensor
    if prog is None or not prog._is_traced(t):
        return False
    from ..static.program import OpNode

    def run(x):
        fn(x)
        return None
    run._pa_comm = meta  # (kind, op, group) for the fuse_all_reduce pass
    prog._append(OpNode(run, (prog._template(t),), {}, None, kind="comm", name="c:" + name))
    return True


def all_reduce(tensor, op=ReduceOp.SUM, group=None, sync_op=True, use_calc_stream=False):
    if is_initialized() and get_world_size(group) > 1 and _static_comm(
            tensor, "all_reduce", lambda x: dist.all_reduce(x, op=_TORCH_OP[op], group=_pg(group)),
            ("all_reduce", op, group)):
        return _ret(None, sync_op)
    if not is_initialized() or get_world_size(group) == 1:
        return _ret(None, sync_op)
    w = dist.all_reduce(tensor._t, op=_TORCH_OP[op], group=_pg(group), async_op=not sync_op)
    return _ret(w, sync_op)


def all_gather(tensor_list, tensor, group=None, sync_op=True):
    n = get_world_size(group)
    t = tensor._t
    if not is_initialized() or n == 1:
        tensor_list.clear() if isinstance(tensor_list, list) else None
        tensor_list.append(_wrap(t.clone()))
        return _ret(None, sync_op)
    out = torch.empty(n * t.numel(), dtype=t.dtype, device=t.device)
    w = dist.all_gather_into_tensor(out, t.contiguous().view(-1), group=_pg(group), async_op=not sync_op)

    def post():
        o = out.view((n,) + tuple(t.shape))
        tensor_list.clear()
        tensor_list.extend(_wrap(o[i]) for i in range(n))
    return _ret(w, sync_op, post)


def all_gather_into_tensor(out_tensor, tensor, group=None, sync_op=True):
    if not is_initialized() or get_world_size(group) == 1:
        out_tensor._t.copy_(tensor._t.reshape(out_tensor._t.shape))
        return _ret(None, sync_op)
    w = dist.all_gather_into_tensor(out_tensor._t, tensor._t.contiguous(), group=_pg(group), async_op=not sync_op)
    return _ret(w, sync_op)


def all_gather_object(object_list, obj, group=None):
    n = get_world_size(group)
    out = [None] * n
    if not is_initialized() or n == 1:
        out = [obj]
    else:
        dist.all_gather_object(out, obj, group=_pg(group))
    object_list.clear()
    object_list.extend(out)


def broadcast(tensor, src, group=None, sync_op=True):
    if is_initialized() and get_world_size(group) > 1 and _static_comm(
            tensor, "broadcast", lambda x: dist.broadcast(x, src=src, group=_pg(group))):
        return _ret(None, sync_op)
    if not is_initialized() or get_world_size(group) == 1:
        return _ret(None, sync_op)
    w = dist.broadcast(tensor._t, src=src, group=_pg(group), async_op=not sync_op)
    return _ret(w, sync_op)


def broadcast_object_list(object_list, src, group=None):
    if not is_initialized() or get_world_size(group) == 1:
        return
    dist.broadcast_object_list(object_list, src=src, group=_pg(group))


def reduce(tensor, dst, op=ReduceOp.SUM, group=None, sync_op=True):
    if not is_initialized() or get_world_size(group) == 1:
        return _ret(None, sync_op)
    w = dist.reduce(tensor._t, dst=dst, op=_TORCH_OP[op], group=_pg(group), async_op=not sync_op)
    return _ret(w, sync_op)


def reduce_scatter(tensor, tensor_list, op=ReduceOp.SUM, group=None, sync_op=True):
    if not is_initialized() or get_world_size(group) == 1:
        tensor._t.copy_(tensor_list[0]._t)
        return _ret(None, sync_op)
    inp = torch.cat([t._t.reshape(-1) for t in tensor_list]).contiguous()
    w = dist.reduce_scatter_tensor(tensor._t.view(-1), inp, op=_TORCH_OP[op], group=_pg(group),
                                   async_op=not sync_op)
    return _ret(w, sync_op)


def reduce_scatter_tensor(out_tensor, in_tensor, op=ReduceOp.SUM, group=None, sync_op=True):
    if not is_initialized() or get_world_size(group) == 1:
        out_tensor._t.copy_(in_tensor._t.reshape(out_tensor._t.shape))
        return _ret(None, sync_op)
    w = dist.reduce_scatter_tensor(out_tensor._t, in_tensor._t.contiguous(), op=_TORCH_OP[op], group=_pg(group),
                                   async_op=not sync_op)
    return _ret(w, sync_op)


def scatter(tensor, tensor_list=None, src=0, group=None, sync_op=True):
    if not is_initialized() or get_world_size(group) == 1:
        tensor._t.copy_(tensor_list[0]._t)
        return _ret(None, sync_op)
    me = dist.get_rank()
    sl = [t._t.contiguous() for t in tensor_list] if me == src else None
    w = dist.scatter(tensor._t, sl, src=src, group=_pg(group), async_op=not sync_op)
    return _ret(w, sync_op)


def scatter_object_list(out_object_list, in_object_list=None, src=0, group=None):
    if not is_initialized() or get_world_size(group) == 1:
        out_object_list.clear()
        out_object_list.append(in_object_list[0])
        return
    out = [None]
    dist.scatter_object_list(out, in_object_list, src=src, group=_pg(group))
    out_object_list.clear()
    out_object_list.extend(out)


def gather(tensor, gather_list=None, dst=0, group=None, sync_op=True):
    n = get_world_size(group)
    if not is_initialized() or n == 1:
        if gather_list is not None:
            gather_list.clear()
            gather_list.append(_wrap(tensor._t.clone()))
        return _ret(None, sync_op)
    me = dist.get_rank()
    bufs = [torch.empty_like(tensor._t) for _ in range(n)] if me == dst else None
    w = dist.gather(tensor._t, bufs, dst=dst, group=_pg(group), async_op=not sync_op)

    def post():
        if me == dst and gather_list is not None:
            gather_list.clear()
            gather_list.extend(_wrap(b) for b in bufs)
    return _ret(w, sync_op, post)


def alltoall(out_tensor_list, in_tensor_list, group=None, sync_op=True):
    n = get_world_size(group)
    if not is_initialized() or n == 1:
        out_tensor_list.clear()
        out_tensor_list.extend(_wrap(t._t.clone()) for t in in_tensor_list)
        return _ret(None, sync_op)
    ins = [t._t.contiguous() for t in in_tensor_list]
    if all(t.shape == ins[0].shape for t in ins):
        # one all_to_all_single over a packed buffer (single RCCL launch; also what gloo supports)
        send = torch.cat([t.reshape(-1) for t in ins])
        recv = torch.empty_like(send)
        w = dist.all_to_all_single(recv, send, group=_pg(group), async_op=not sync_op)
        outs = list(recv.view((n,) + tuple(ins[0].shape)).unbind(0))
    else:
        outs = [torch.empty_like(t) for t in ins]
        w = dist.all_to_all(outs, ins, group=_pg(group), async_op=not sync_op)

    def post():
        out_tensor_list.clear()
        out_tensor_list.extend(_wrap(o) for o in outs)
    return _ret(w, sync_op, post)


def alltoall_single(out_tensor, in_tensor, in_split_sizes=None, out_split_sizes=None, group=None, sync_op=True):
    if not is_initialized() or get_world_size(group) == 1:
        out_tensor._t.copy_(in_tensor._t)
        return _ret(None, sync_op)
    w = dist.all_to_all_single(out_tensor._t, in_tensor._t.contiguous(), out_split_sizes, in_split_sizes,
                               group=_pg(group), async_op=not sync_op)
    return _ret(w, sync_op)


def send(tensor, dst=0, group=None, sync_op=True):
    w = dist.isend(tensor._t.contiguous(), dst=dst, group=_pg(group))
    return _ret(w, sync_op)


def recv(tensor, src=0, group=None, sync_op=True):
    w = dist.irecv(tensor._t, src=src, group=_pg(group))
    return _ret(w, sync_op)


def isend(tensor, dst, group=None):
    return send(tensor, dst, group, False)


def irecv(tensor, src=None, group=None):
    return recv(tensor, src, group, False)


class P2POp:
    def __init__(self, op, tensor, peer, group=None):
        self.op, self.tensor, self.peer, self.group = op, tensor, peer, group


def batch_isend_irecv(p2p_op_list):
    ops = []
    for p in p2p_op_list:
        fn = dist.isend if p.op in (isend, dist.isend, send) else dist.irecv
        ops.append(dist.P2POp(fn, p.tensor._t, p.peer, group=_pg(p.group)))
    works = dist.batch_isend_irecv(ops)
    return [_Task(w) for w in works]


def wait(tensor, group=None, use_calc_stream=True):
    if tensor._t.is_cuda:
        torch.cuda.current_stream().synchronize()


def get_global_rank(group, group_rank):
    return group.ranks[group_rank]
