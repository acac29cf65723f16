"""paddle.incubate.tensor. Reference: python/paddle/incubate/tensor/{math,manipulation}.py (segment_* reductions,
_npu_identity, async offload / reload of tensors to pinned host memory on a side stream)."""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor, _wrap
from ..geometric import segment_sum, segment_mean, segment_max, segment_min  # noqa: F401


def _npu_identity(x, format=-1):
    """Identity (the reference's NPU storage-format cast; formats do not exist on this device)."""
    return x


class _AsyncLoad:
    """Side stream + events for async_offload / async_reload (reference manipulation.py:102 create_async_load)."""

    def __init__(self):
        self.stream = torch.cuda.Stream() if torch.cuda.is_available() else None

    def _run(self, src, fn):
        if self.stream is None:
            return fn(src), None
        ev = torch.cuda.Event()
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            out = fn(src)
            ev.record(self.stream)
        src.record_stream(self.stream)
        return out, ev


class _Task:
    def __init__(self, event):
        self._event = event

    def wait(self):
        if self._event is not None:
            torch.cuda.current_stream().wait_event(self._event)

    def cpu_wait(self):
        if self._event is not None:
            self._event.synchronize()

    def is_completed(self):
        return self._event is None or self._event.query()


def create_async_load():
    return _AsyncLoad()


def async_offload(src_tensor, async_load):
    """Copy a device tensor to pinned host memory on the loader's stream: (host tensor, task)."""
    t = src_tensor._t if isinstance(src_tensor, Tensor) else src_tensor

    def cp(s):
        h = torch.empty(s.shape, dtype=s.dtype, pin_memory=s.is_cuda)
        h.copy_(s, non_blocking=True)
        return h
    out, ev = async_load._run(t, cp)
    return _wrap(out), _Task(ev)


def async_reload(src_tensor, async_load):
    """Copy a (pinned) host tensor back to the current device on the loader's stream: (device tensor, task)."""
    t = src_tensor._t if isinstance(src_tensor, Tensor) else src_tensor
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    out, ev = async_load._run(t, lambda s: s.to(dev, non_blocking=True))
    return _wrap(out), _Task(ev)
