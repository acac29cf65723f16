"""paddle.incubate.multiprocessing: the standard multiprocessing API with Tensor pickling through shared memory.

Reference: python/paddle/incubate/multiprocessing/__init__.py + reductions.py:235 (init_reductions registers
ForkingPickler reducers so a Tensor sent to another process travels as a shared-memory / IPC handle instead of a
copy). A paddle Tensor is reduced to its torch storage, which torch.multiprocessing's reducers share (CPU: shared
memory file descriptors; GPU: IPC handles)."""
from __future__ import annotations

import multiprocessing
from multiprocessing import *  # noqa: F401,F403
from multiprocessing.reduction import ForkingPickler

import torch.multiprocessing  # noqa: F401  (registers the torch.Tensor reducers)

from ..framework.tensor import Tensor

__all__ = []


def _rebuild_tensor(t, stop_gradient):
    out = Tensor(t)
    out.stop_gradient = stop_gradient
    return out


def _reduce_tensor(x):
    return _rebuild_tensor, (x._t.detach(), x.stop_gradient)


def init_reductions():
    ForkingPickler.register(Tensor, _reduce_tensor)


init_reductions()
_ = multiprocessing
