"""paddle.device.cuda on HIP: streams, events, memory stats, graphs.
Reference: python/paddle/device/cuda/{__init__,streams,graphs}.py."""
from __future__ import annotations

import contextlib

import torch

from . import graphs  # noqa: F401


def device_count():
    return torch.cuda.device_count()


def synchronize(device=None):
    if torch.cuda.is_available():
        torch.cuda.synchronize(_dev(device))


def _dev(device):
    if device is None:
        return None
    if isinstance(device, int):
        return device
    if hasattr(device, "get_device_id"):
        return device.get_device_id()
    if isinstance(device, str):
        return int(device.split(":")[1]) if ":" in device else 0
    return device


class Stream:
    def __init__(self, device=None, priority=2, stream_base=None, blocking=False):
        if stream_base is not None:  # wrap an existing stream (ours or a torch one)
            self._s = stream_base._s if isinstance(stream_base, Stream) else stream_base
            return
        self._s = torch.cuda.Stream(device=_dev(device), priority=-1 if priority == 1 else 0)

    @property
    def stream_base(self):
        return self._s

    @property
    def cuda_stream(self):
        return self._s.cuda_stream

    def synchronize(self):
        self._s.synchronize()

    def wait_event(self, event):
        self._s.wait_event(event._e)

    def wait_stream(self, stream):
        self._s.wait_stream(stream._s)

    def record_event(self, event=None):
        event = event or Event()
        event.record(self)
        return event

    def query(self):
        return self._s.query()


class Event:
    def __init__(self, enable_timing=False, blocking=False, interprocess=False):
        self._e = torch.cuda.Event(enable_timing=enable_timing, blocking=blocking, interprocess=interprocess)

    def record(self, stream=None):
        self._e.record(None if stream is None else stream._s)

    def query(self):
        return self._e.query()

    def synchronize(self):
        self._e.synchronize()

    def elapsed_time(self, end_event):
        return self._e.elapsed_time(end_event._e)


def current_stream(device=None):
    s = Stream.__new__(Stream)
    s._s = torch.cuda.current_stream(_dev(device))
    return s


def default_stream(device=None):
    s = Stream.__new__(Stream)
    s._s = torch.cuda.default_stream(_dev(device))
    return s


@contextlib.contextmanager
def stream_guard(stream):
    with torch.cuda.stream(stream._s):
        yield


def set_stream(stream):
    torch.cuda.set_stream(stream._s)
    return stream


def _native():
    from .. import allocator as A
    return A if A.is_enabled() else None


def _idx(device):
    d = _dev(device)
    return d.index if isinstance(d, torch.device) and d.index is not None else (
        d if isinstance(d, int) else torch.cuda.current_device())


def max_memory_allocated(device=None):
    A = _native()
    if A is not None:
        return A.stats(_idx(device))["peak_allocated"]
    return torch.cuda.max_memory_allocated(_dev(device))


def max_memory_reserved(device=None):
    A = _native()
    if A is not None:
        return A.stats(_idx(device))["peak_reserved"]
    return torch.cuda.max_memory_reserved(_dev(device))


def memory_allocated(device=None):
    A = _native()
    if A is not None:
        return A.stats(_idx(device))["allocated"]
    return torch.cuda.memory_allocated(_dev(device))


def memory_reserved(device=None):
    A = _native()
    if A is not None:
        return A.stats(_idx(device))["reserved"]
    return torch.cuda.memory_reserved(_dev(device))


def reset_max_memory_allocated(device=None):
    A = _native()
    if A is not None:
        A.reset_peak(_idx(device))
        return
    torch.cuda.reset_peak_memory_stats(_dev(device))


def empty_cache():
    A = _native()
    if A is not None:
        for i in range(torch.cuda.device_count()):
            A.empty_cache(i)
        return
    torch.cuda.empty_cache()


def get_device_properties(device=None):
    return torch.cuda.get_device_properties(_dev(device) or 0)


def get_device_name(device=None):
    return torch.cuda.get_device_name(_dev(device) or 0)


def get_device_capability(device=None):
    return torch.cuda.get_device_capability(_dev(device) or 0)
