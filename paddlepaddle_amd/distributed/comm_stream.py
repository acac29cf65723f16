"""paddle.distributed.stream / paddle.distributed.communication.stream: collectives with explicit stream
semantics (reference python/paddle/distributed/communication/stream/*.py).

On this framework RCCL runs each collective on the process group's communication stream (torch c10d
ProcessGroupNCCL over RCCL/xGMI); `work.wait()` makes the *current* (calculation) stream wait on it
without blocking the host. The three modes map onto that:
  * ``sync_op=False``: the collective is issued and its task returned; the caller orders it with
    ``task.wait()`` (a stream dependency, not a host sync) — compute issued meanwhile overlaps it.
  * ``sync_op=True, use_calc_stream=False``: issued, then the calculation stream waits on it; the finished
    task is returned.
  * ``sync_op=True, use_calc_stream=True``: the collective is ordered on the calculation stream (issued and
    waited at once); returns None, as the reference does — no task object to keep alive.
``use_calc_stream=True`` with ``sync_op=False`` is rejected like in the reference. All-gather /
reduce-scatter / all-to-all accept either a tensor list or one concatenated tensor."""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor, _wrap
from . import collective as C
from .collective import ReduceOp


def _finish(task, sync_op, use_calc_stream):
    if not sync_op and use_calc_stream:
        raise RuntimeError("use_calc_stream can only be true in sync op behavior.")
    if not sync_op:
        return task
    task.wait()
    return None if use_calc_stream else task


def _check(sync_op, use_calc_stream):
    if not sync_op and use_calc_stream:
        raise RuntimeError("use_calc_stream can only be true in sync op behavior.")


def all_reduce(tensor, op=ReduceOp.SUM, group=None, sync_op=True, use_calc_stream=False):
    _check(sync_op, use_calc_stream)
    return _finish(C.all_reduce(tensor, op, group, sync_op=False) or C._Task(), sync_op, use_calc_stream)


def all_gather(tensor_or_tensor_list, tensor, group=None, sync_op=True, use_calc_stream=False):
    _check(sync_op, use_calc_stream)
    if isinstance(tensor_or_tensor_list, list):
        task = C.all_gather(tensor_or_tensor_list, tensor, group, sync_op=False)
    else:
        task = C.all_gather_into_tensor(tensor_or_tensor_list, tensor, group, sync_op=False)
    return _finish(task or C._Task(), sync_op, use_calc_stream)


def reduce_scatter(tensor, tensor_or_tensor_list, op=ReduceOp.SUM, group=None, sync_op=True, use_calc_stream=False):
    _check(sync_op, use_calc_stream)
    src = tensor_or_tensor_list
    if isinstance(src, Tensor):  # one concatenated input: split along dim 0
        n = C.get_world_size(group)
        src = [_wrap(c) for c in src._t.chunk(n, 0)]
    return _finish(C.reduce_scatter(tensor, src, op, group, sync_op=False) or C._Task(), sync_op, use_calc_stream)


def alltoall(out_tensor_or_tensor_list, in_tensor_or_tensor_list, group=None, sync_op=True, use_calc_stream=False):
    _check(sync_op, use_calc_stream)
    if isinstance(in_tensor_or_tensor_list, Tensor):
        task = C.alltoall_single(out_tensor_or_tensor_list, in_tensor_or_tensor_list, group=group, sync_op=False)
    else:
        task = C.alltoall(out_tensor_or_tensor_list, in_tensor_or_tensor_list, group, sync_op=False)
    return _finish(task or C._Task(), sync_op, use_calc_stream)


def alltoall_single(out_tensor, in_tensor, out_split_sizes=None, in_split_sizes=None, group=None, sync_op=True,
                    use_calc_stream=False):
    _check(sync_op, use_calc_stream)
    task = C.alltoall_single(out_tensor, in_tensor, in_split_sizes, out_split_sizes, group, sync_op=False)
    return _finish(task or C._Task(), sync_op, use_calc_stream)


def broadcast(tensor, src, group=None, sync_op=True, use_calc_stream=False):
    _check(sync_op, use_calc_stream)
    return _finish(C.broadcast(tensor, src, group, sync_op=False) or C._Task(), sync_op, use_calc_stream)


def reduce(tensor, dst=0, op=ReduceOp.SUM, group=None, sync_op=True, use_calc_stream=False):
    _check(sync_op, use_calc_stream)
    return _finish(C.reduce(tensor, dst, op, group, sync_op=False) or C._Task(), sync_op, use_calc_stream)


def scatter(tensor, tensor_or_tensor_list=None, src=0, group=None, sync_op=True, use_calc_stream=False):
    _check(sync_op, use_calc_stream)
    lst = tensor_or_tensor_list
    if isinstance(lst, Tensor):
        n = C.get_world_size(group)
        lst = [_wrap(c) for c in lst._t.chunk(n, 0)]
    return _finish(C.scatter(tensor, lst, src, group, sync_op=False) or C._Task(), sync_op, use_calc_stream)


def gather(tensor, gather_list=None, dst=0, group=None, sync_op=True, use_calc_stream=False):
    _check(sync_op, use_calc_stream)
    return _finish(C.gather(tensor, gather_list, dst, group, sync_op=False) or C._Task(), sync_op, use_calc_stream)


def send(tensor, dst=0, group=None, sync_op=True, use_calc_stream=False):
    _check(sync_op, use_calc_stream)
    return _finish(C.send(tensor, dst, group, sync_op=False) or C._Task(), sync_op, use_calc_stream)


def recv(tensor, src=0, group=None, sync_op=True, use_calc_stream=False):
    _check(sync_op, use_calc_stream)
    return _finish(C.recv(tensor, src, group, sync_op=False) or C._Task(), sync_op, use_calc_stream)


__all__ = ["all_reduce", "all_gather", "reduce_scatter", "alltoall", "alltoall_single", "broadcast", "reduce",
           "scatter", "gather", "send", "recv"]
del torch
