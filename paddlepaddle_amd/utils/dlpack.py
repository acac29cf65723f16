"""Reference: python/paddle/utils/dlpack.py."""
from __future__ import annotations

import torch.utils.dlpack as _dl

from ..framework.tensor import _wrap


def to_dlpack(x):
    return _dl.to_dlpack(x._t)


def from_dlpack(dlpack):
    if hasattr(dlpack, "__dlpack__"):
        import torch
        return _wrap(torch.from_dlpack(dlpack))
    return _wrap(_dl.from_dlpack(dlpack))
