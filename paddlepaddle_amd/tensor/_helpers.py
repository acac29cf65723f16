"""Argument normalisation shared by the tensor op modules."""
from __future__ import annotations

import numpy as np
import torch

from ..framework import dtype as _dt
from ..framework.tensor import Tensor, _unwrap, _wrap


def T(x):
    """Unwrap a paddle Tensor to its device buffer; numpy arrays become torch tensors."""
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, np.ndarray):
        return torch.from_numpy(x)
    return x


def TT(x, like=None):
    """Unwrap and force a torch tensor (python scalars become 0-d tensors on like's device)."""
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, torch.Tensor):
        return x
    if isinstance(x, np.ndarray):
        t = torch.from_numpy(x)
    else:
        t = torch.as_tensor(x)
    if like is not None:
        t = t.to(like.device)
    return t


def axis_arg(axis):
    if axis is None:
        return None
    if isinstance(axis, Tensor):
        axis = axis._t.tolist()
    if isinstance(axis, torch.Tensor):
        axis = axis.tolist()
    if isinstance(axis, (list, tuple)):
        if len(axis) == 0:
            return None
        return tuple(int(a) for a in axis)
    return int(axis)


def shape_arg(shape):
    if isinstance(shape, Tensor):
        return tuple(int(v) for v in shape._t.tolist())
    if isinstance(shape, torch.Tensor):
        return tuple(int(v) for v in shape.tolist())
    if isinstance(shape, (int, np.integer)):
        return (int(shape),)
    return tuple(int(v._t.item()) if isinstance(v, Tensor) else int(v) for v in shape)


def dtype_arg(dtype):
    return None if dtype is None else _dt.to_torch_dtype(dtype)


def wrap(t):
    return _wrap(t)


def wraps(seq):
    return [_wrap(t) for t in seq]


def scalar(x):
    if isinstance(x, Tensor):
        return x._t.item()
    if isinstance(x, torch.Tensor):
        return x.item()
    return x
