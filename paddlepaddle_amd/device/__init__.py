"""paddle.device. Reference: python/paddle/device/__init__.py. 'gpu' = HIP device (MI355X)."""
from __future__ import annotations

import torch

from ..framework.place import (set_device, get_device, is_compiled_with_cuda, is_compiled_with_rocm,  # noqa: F401
                               is_compiled_with_xpu, is_compiled_with_ipu, is_compiled_with_cinn,
                               is_compiled_with_custom_device, CPUPlace, CUDAPlace)
from . import cuda  # noqa: F401
from . import pinned  # noqa: F401
from .cuda import Stream, current_stream, stream_guard, synchronize  # noqa: F401
from .cuda import Event as _CudaEvent


class Event(_CudaEvent):
    """paddle.device.Event: the device comes first (reference device/__init__.py Event(device, enable_timing,
    blocking, interprocess)); paddle.device.cuda.Event keeps (enable_timing, blocking, interprocess)."""

    def __init__(self, device=None, enable_timing=False, blocking=False, interprocess=False):
        super().__init__(enable_timing, blocking, interprocess)
        self.device = device


def get_all_device_type():
    return ["cpu", "gpu"] if torch.cuda.is_available() else ["cpu"]


def get_all_custom_device_type():
    return []


def get_available_device():
    return ["cpu"] + [f"gpu:{i}" for i in range(torch.cuda.device_count())]


def get_available_custom_device():
    return []


def get_cudnn_version():
    return None


def device_count():
    return torch.cuda.device_count()


def is_compiled_with_distribute():
    """RCCL (torch.distributed 'nccl' backend) and gloo are built in."""
    import torch.distributed as dist
    return dist.is_available()


def set_stream(stream=None):
    """Make ``stream`` the current stream of its device; returns the previous one."""
    prev = current_stream()
    if stream is not None:
        torch.cuda.set_stream(getattr(stream, "_s", stream))
    return prev


class XPUPlace:
    def __init__(self, *a, **k):
        raise RuntimeError("XPU devices are not supported by this MI355X framework")


class IPUPlace:
    def __init__(self, *a, **k):
        raise RuntimeError("IPU devices are not supported by this MI355X framework")
