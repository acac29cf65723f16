"""Device places. Reference: paddle/phi/common/place.h, python/paddle/device/__init__.py.

On MI355X a "GPU place" is a HIP device (one process per GPU). CUDAPlace is kept as the public
name for API compatibility with paddle code; it denotes a HIP device here.
"""
from __future__ import annotations

import os

import torch


class Place:
    __slots__ = ()

    def is_cpu_place(self):
        return False

    def is_gpu_place(self):
        return False

    def is_cuda_pinned_place(self):
        return False

    def is_custom_place(self):
        return False

    def __eq__(self, other):
        return isinstance(other, Place) and repr(self) == repr(other)

    def __hash__(self):
        return hash(repr(self))


class CPUPlace(Place):
    __slots__ = ()

    def is_cpu_place(self):
        return True

    def __repr__(self):
        return "Place(cpu)"

    @property
    def torch_device(self):
        return torch.device("cpu")


class CUDAPlace(Place):
    __slots__ = ("_id",)

    def __init__(self, id=0):
        self._id = int(id)

    def is_gpu_place(self):
        return True

    def get_device_id(self):
        return self._id

    def gpu_device_id(self):
        return self._id

    def __repr__(self):
        return f"Place(gpu:{self._id})"

    @property
    def torch_device(self):
        return torch.device("cuda", self._id)


class CUDAPinnedPlace(Place):
    __slots__ = ()

    def is_cuda_pinned_place(self):
        return True

    def __repr__(self):
        return "Place(gpu_pinned)"

    @property
    def torch_device(self):
        return torch.device("cpu")


class XPUPlace(CPUPlace):  # not supported on this hardware, kept for import compatibility
    def __init__(self, dev_id=0):
        super().__init__()
        self._dev_id = int(dev_id)

    def get_device_id(self):
        return self._dev_id


class CustomPlace(CPUPlace):
    def __init__(self, dev_type="custom", dev_id=0):
        super().__init__()
        self._dev_type, self._dev_id = dev_type, int(dev_id)

    def get_device_id(self):
        return self._dev_id

    def get_device_type(self):
        return self._dev_type


IPUPlace = CPUPlace


def is_compiled_with_cuda():
    """True on a ROCm build (the HIP device plays the CUDA role in the paddle API)."""
    return torch.version.hip is not None or torch.cuda.is_available()


def is_compiled_with_rocm():
    return torch.version.hip is not None


def is_compiled_with_xpu():
    return False


def is_compiled_with_ipu():
    return False


def is_compiled_with_cinn():
    return False


def is_compiled_with_distribute():
    return True


def is_compiled_with_custom_device(device_type=None):
    return False


_current_place = None


def _default_place():
    if torch.cuda.is_available() and os.environ.get("PADDLE_AMD_FORCE_CPU", "0") != "1":
        # launcher-assigned device id (``--devices 4,5``) wins over the local rank
        idx = int(os.environ.get("PADDLE_AMD_DEVICE_ID", os.environ.get("LOCAL_RANK", "0")))
        idx %= max(torch.cuda.device_count(), 1)
        return CUDAPlace(idx)
    return CPUPlace()


def _get_current_place():
    global _current_place
    if _current_place is None:
        _current_place = _default_place()
    return _current_place


def _get_torch_device():
    return _get_current_place().torch_device


def set_device(device):
    """paddle.set_device('cpu' | 'gpu' | 'gpu:N'). Returns the new place."""
    global _current_place
    if isinstance(device, Place):
        _current_place = device
    else:
        d = str(device).lower()
        if d == "cpu":
            _current_place = CPUPlace()
        elif d.startswith("gpu") or d.startswith("cuda") or d.startswith("hip"):
            idx = int(d.split(":")[1]) if ":" in d else 0
            if not torch.cuda.is_available():
                raise ValueError("no HIP device is available; cannot set_device('gpu')")
            _current_place = CUDAPlace(idx)
        else:
            raise ValueError(f"unsupported device {device!r}")
    if isinstance(_current_place, CUDAPlace):
        torch.cuda.set_device(_current_place.get_device_id())
    return _current_place


def get_device():
    p = _get_current_place()
    if isinstance(p, CUDAPlace):
        return f"gpu:{p.get_device_id()}"
    return "cpu"


def place_from_torch_device(dev) -> Place:
    if dev.type == "cuda":
        return CUDAPlace(dev.index or 0)
    return CPUPlace()


def to_torch_device(place):
    if place is None:
        return _get_torch_device()
    if isinstance(place, Place):
        return place.torch_device
    if isinstance(place, str):
        p = place.lower()
        if p == "cpu":
            return torch.device("cpu")
        if p.startswith(("gpu", "cuda")):
            idx = int(p.split(":")[1]) if ":" in p else 0
            return torch.device("cuda", idx)
    if isinstance(place, torch.device):
        return place
    raise ValueError(f"unsupported place {place!r}")
