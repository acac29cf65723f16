"""Pinned (page-locked) host memory from the native pool ``_C_runtime.PinnedPool``
(csrc/runtime/pinned_pool.cpp: auto-growth best-fit chunks of hipHostMalloc memory).

Reference: paddle/phi/core/memory/allocation/{pinned_allocator.cc, auto_growth_best_fit_allocator.cc}
and ``Tensor.pin_memory`` / DataLoader's pinned staging (python/paddle/io/dataloader).

A pooled buffer is exposed as a CPU torch tensor that shares the pool's memory (``torch.frombuffer``
keeps the owner alive through every view). When the last view dies the block goes back to the pool —
but not while an asynchronous host->device copy may still read it: ``copy_to_device`` records an
event on the copying stream and the block is only recycled once that event has completed (checked
lazily on the next allocation and by ``reclaim()``).
"""
from __future__ import annotations

import ctypes
import threading
import weakref

import torch

_lock = threading.Lock()
_pool = None
_pending = []  # (event, ptr) blocks whose release waits for a device copy
_LIVE = weakref.WeakValueDictionary()  # block address -> live _Block (pooled tensors' storage start)


def pool():
    """The process-wide native pinned pool (None when the runtime module is not built)."""
    global _pool
    if _pool is None:
        from ..utils import native
        m = native.module()
        if m is None or not hasattr(m, "PinnedPool"):
            return None
        # resolve hipHostMalloc only when a HIP device is usable; otherwise page-aligned host memory
        _pool = m.PinnedPool(64 << 20, 256, bool(torch.cuda.is_available()))
    return _pool


class _Block:
    """Owner of one pool block; returned to the pool when the last tensor view is gone."""

    __slots__ = ("ptr", "event", "__weakref__")

    def __init__(self, ptr):
        self.ptr = ptr
        self.event = None

    def __del__(self):
        p = _pool
        if p is None or self.ptr is None:
            return
        ev, self.event = self.event, None
        if ev is not None and not ev.query():
            with _lock:
                _pending.append((ev, self.ptr))
        else:
            p.deallocate(self.ptr)
        self.ptr = None


def reclaim():
    """Recycle blocks whose pending device copies have completed; returns how many were freed."""
    p = _pool
    if p is None:
        return 0
    with _lock:
        done = [(e, q) for e, q in _pending if e.query()]
        for item in done:
            _pending.remove(item)
    for _, q in done:
        p.deallocate(q)
    return len(done)


def empty(shape, dtype=torch.float32):
    """Uninitialised pinned CPU tensor from the pool (falls back to torch's pinned allocator)."""
    p = pool()
    shape = tuple(int(s) for s in shape)
    if p is None:
        t = torch.empty(shape, dtype=dtype)
        return t.pin_memory() if torch.cuda.is_available() else t
    if _pending:
        reclaim()
    n = 1
    for s in shape:
        n *= s
    nbytes = max(1, n * torch.empty((), dtype=dtype).element_size())
    ptr = p.allocate(nbytes)
    buf = (ctypes.c_uint8 * nbytes).from_address(ptr)
    blk = _Block(ptr)
    buf._pa_owner = blk  # torch.frombuffer keeps buf (hence the block) alive through every view
    _LIVE[ptr] = blk
    return torch.frombuffer(buf, dtype=torch.uint8, count=nbytes).view(dtype)[:n].view(shape)


def is_pooled(t):
    return _LIVE.get(t.untyped_storage().data_ptr()) is not None


def pin(t):
    """Copy a CPU tensor into pooled pinned memory (Tensor.pin_memory)."""
    out = empty(t.shape, t.dtype)
    out.copy_(t)
    return out


def copy_to_device(t, device, stream=None):
    """Asynchronous H2D copy of a pinned tensor. The block the source lives in is kept out of the pool
    until the copy has completed (event on the copying stream)."""
    dev_t = t.to(device, non_blocking=True)
    if torch.cuda.is_available() and device.type == "cuda":
        ev = torch.cuda.Event()
        ev.record(stream or torch.cuda.current_stream(device))
        owner = _LIVE.get(t.untyped_storage().data_ptr())
        if owner is not None:
            owner.event = ev
    return dev_t


def stats():
    p = pool()
    s = dict(p.stats()) if p is not None else {}
    s["pending_copies"] = len(_pending)
    return s


def release_idle():
    """Free fully idle pool chunks back to the system (paddle.device.cuda.empty_cache analogue)."""
    reclaim()
    p = pool()
    return p.release_idle() if p is not None else 0
