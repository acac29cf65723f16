"""Native device allocator (csrc/runtime/allocator.h, HIP backend allocator_hip.cpp -> _C_alloc.so).

Reference: paddle/phi/core/memory/allocation/auto_growth_best_fit_allocator.cc, stream_safe_cuda_allocator.cc,
FLAGS_allocator_strategy. It replaces PyTorch's caching allocator for every device buffer of the process
(torch.cuda.memory.CUDAPluggableAllocator): auto-growth 64 MiB+ chunks from hipMalloc, best-fit blocks with
splitting and neighbour coalescing, per-stream pools with event-ordered cross-stream reuse, free chunks
released on OOM / empty_cache. paddle.device.cuda.memory_* report its counters while it is active.

It must be installed before the first device allocation: ``enable()`` early in the program, or set
``PADDLE_AMD_ALLOCATOR=auto_growth`` (or FLAGS_allocator_strategy=auto_growth_best_fit) in the environment,
which the package honours at import. PyTorch's hipGraph memory pools need its own allocator, so graph
capture is unavailable while this one is installed.
"""
from __future__ import annotations

import ctypes
import os

import torch

_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C_alloc.so")
_LIB = None
_ACTIVE = False
_FIELDS = ("allocated", "reserved", "peak_allocated", "peak_reserved", "n_alloc", "n_free", "n_chunks",
           "n_raw_alloc", "n_raw_free", "n_cross_stream", "n_oom_release")


def _lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(_PATH):
            raise RuntimeError(f"native allocator library missing: {_PATH} (run tools/build_native.py)")
        _LIB = ctypes.CDLL(_PATH)
        _LIB.pa_alloc_stats.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]
        _LIB.pa_alloc_empty_cache.argtypes = [ctypes.c_int]
        _LIB.pa_alloc_empty_cache.restype = ctypes.c_int64
        _LIB.pa_alloc_reset_peak.argtypes = [ctypes.c_int]
        _LIB.pa_alloc_set_min_chunk.argtypes = [ctypes.c_int64]
    return _LIB


def enable(min_chunk_mb=64):
    """Install the native allocator for this process (before any device tensor exists)."""
    global _ACTIVE
    if _ACTIVE:
        return True
    lib = _lib()
    lib.pa_alloc_set_min_chunk(int(min_chunk_mb) << 20)
    # a pluggable allocator gets no record_stream calls: let the process groups keep their tensors alive
    # until the collective is waited on instead (stream-ordered reuse stays safe)
    os.environ.setdefault("TORCH_NCCL_AVOID_RECORD_STREAMS", "1")
    alloc = torch.cuda.memory.CUDAPluggableAllocator(_PATH, "pa_malloc", "pa_free")
    torch.cuda.memory.change_current_allocator(alloc)
    _ACTIVE = True
    return True


def is_enabled():
    return _ACTIVE


def stats(device=0):
    out = (ctypes.c_int64 * len(_FIELDS))()
    _lib().pa_alloc_stats(int(device), out)
    return dict(zip(_FIELDS, [int(v) for v in out]))


def empty_cache(device=0):
    return int(_lib().pa_alloc_empty_cache(int(device)))


def reset_peak(device=0):
    _lib().pa_alloc_reset_peak(int(device))


def _env_requested():
    v = os.environ.get("PADDLE_AMD_ALLOCATOR", "") or os.environ.get("FLAGS_allocator_strategy", "")
    return v.lower() in ("auto_growth", "auto_growth_best_fit", "native")
