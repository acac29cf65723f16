"""HIP graph capture / replay. Reference: python/paddle/device/cuda/graphs.py (CUDAGraph: capture_begin,
capture_end, replay, reset, print_to_dot_files; wrap_cuda_graph), paddle/phi/backends/gpu/cuda/cuda_graph.cc.

MI355X design: the capture itself is the HIP runtime's stream capture driven natively
(csrc/runtime/allocator_hip.cpp: pa_graph_begin -> hipStreamBeginCapture, pa_graph_end -> hipStreamEndCapture +
hipGraphInstantiate, pa_graph_launch -> hipGraphLaunch, hipGraphDebugDotPrint). Memory touched by the captured
work must stay reserved for the replays, so allocations made while capturing go to a private memory pool of
the active device allocator: the framework's native allocator (device/allocator.py, graph pools in
csrc/runtime/allocator.h) when it is installed, otherwise PyTorch's caching allocator through its pool API.
A pool may be shared by several graphs (``pool_id``) and is released by ``reset()``.
Launch-bound inner loops (decode steps, small-batch training steps) are captured once and replayed — the
replacement for a tracing compiler."""
from __future__ import annotations

import ctypes
import itertools
import os

import torch

_MODES = {"global": 0, "thread_local": 1, "relaxed": 2}
_POOL_IDS = itertools.count(1)
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        from .. import allocator as A
        lib = ctypes.CDLL(A._PATH)
        vp = ctypes.c_void_p
        lib.pa_graph_begin.argtypes = [vp, ctypes.c_int]
        lib.pa_graph_end.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        lib.pa_graph_launch.argtypes = [vp, vp]
        lib.pa_graph_num_nodes.argtypes = [vp, ctypes.POINTER(ctypes.c_size_t)]
        lib.pa_graph_dot.argtypes = [vp, ctypes.c_char_p]
        lib.pa_graph_destroy.argtypes = [vp, vp]
        lib.pa_alloc_begin_pool.argtypes = [ctypes.c_int, vp, ctypes.c_uint64]
        lib.pa_alloc_end_pool.argtypes = [ctypes.c_int, vp]
        lib.pa_alloc_release_pool.argtypes = [ctypes.c_int, ctypes.c_uint64]
        _LIB = lib
    return _LIB


def is_cuda_graph_supported():
    return torch.cuda.is_available()


def _native_alloc():
    from .. import allocator as A
    return A.is_enabled()


class CUDAGraph:
    def __init__(self, place=None, mode="thread_local", pool_id=None):
        if mode not in _MODES:
            raise ValueError(f"mode must be one of {list(_MODES)}")
        self._mode = _MODES[mode]
        self._pool = pool_id
        self._graph = self._exec = None
        self._stream = None
        self._ctx = None
        self._dev = None
        self._native = None

    def capture_begin(self):
        if self._exec is not None:
            raise RuntimeError("graph already captured; reset() before capturing again")
        self._dev = torch.cuda.current_device()
        self._stream = torch.cuda.Stream()
        self._stream.wait_stream(torch.cuda.current_stream())
        self._ctx = torch.cuda.stream(self._stream)
        self._ctx.__enter__()
        sp = ctypes.c_void_p(self._stream.cuda_stream)
        self._native = _native_alloc()
        if self._native:
            if self._pool is None:
                self._pool = next(_POOL_IDS)
            _lib().pa_alloc_begin_pool(self._dev, sp, self._pool)
        else:
            if self._pool is None:
                self._pool = torch.cuda.graph_pool_handle()
            torch._C._cuda_beginAllocateCurrentStreamToPool(self._dev, self._pool)
        # the native allocator may grow its graph pool with hipMalloc during the capture, which only the
        # relaxed capture mode permits
        rc = _lib().pa_graph_begin(sp, 2 if self._native else self._mode)
        if rc != 0:
            self._end_pool()
            self._ctx.__exit__(None, None, None)
            raise RuntimeError(f"hipStreamBeginCapture failed ({rc})")

    def _end_pool(self):
        if self._native:
            _lib().pa_alloc_end_pool(self._dev, ctypes.c_void_p(self._stream.cuda_stream))
        else:
            torch._C._cuda_endAllocateToPool(self._dev, self._pool)

    def capture_end(self):
        g, x = ctypes.c_void_p(), ctypes.c_void_p()
        rc = _lib().pa_graph_end(ctypes.c_void_p(self._stream.cuda_stream), ctypes.byref(g), ctypes.byref(x))
        self._end_pool()
        self._ctx.__exit__(None, None, None)
        torch.cuda.current_stream().wait_stream(self._stream)
        if rc != 0:
            raise RuntimeError(f"hipStreamEndCapture / hipGraphInstantiate failed ({rc})")
        self._graph, self._exec = g.value, x.value

    def replay(self):
        if self._exec is None:
            raise RuntimeError("replay() before capture_end()")
        rc = _lib().pa_graph_launch(ctypes.c_void_p(self._exec), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        if rc != 0:
            raise RuntimeError(f"hipGraphLaunch failed ({rc})")

    def num_nodes(self):
        n = ctypes.c_size_t()
        _lib().pa_graph_num_nodes(ctypes.c_void_p(self._graph), ctypes.byref(n))
        return int(n.value)

    def reset(self):
        if self._exec is not None or self._graph is not None:
            torch.cuda.current_stream().synchronize()
            _lib().pa_graph_destroy(ctypes.c_void_p(self._graph), ctypes.c_void_p(self._exec))
        self._graph = self._exec = None
        if self._pool is not None and self._dev is not None:
            if self._native:
                _lib().pa_alloc_release_pool(self._dev, self._pool)
            else:
                torch._C._cuda_releasePool(self._dev, self._pool)

    def pool(self):
        return self._pool

    def print_to_dot_files(self, dirname, flags=None):
        os.makedirs(str(dirname), exist_ok=True)
        path = os.path.join(str(dirname), "graph.dot")
        rc = _lib().pa_graph_dot(ctypes.c_void_p(self._graph), path.encode())
        if rc != 0:
            raise RuntimeError(f"hipGraphDebugDotPrint failed ({rc})")
        return path

    def __del__(self):
        try:
            if self._exec is not None:
                self.reset()
        except Exception:  # pragma: no cover - interpreter shutdown
            pass


class capture:
    """``with capture(g): ...`` == g.capture_begin() ... g.capture_end()."""

    def __init__(self, graph):
        self.graph = graph

    def __enter__(self):
        self.graph.capture_begin()
        return self.graph

    def __exit__(self, *exc):
        self.graph.capture_end()
        return False


def wrap_cuda_graph(function, mode="thread_local", memory_pool="default"):
    """Run ``function`` eagerly once (warm-up), capture it on the second call with the same input shapes,
    then replay: inputs are copied into the captured static buffers and the captured outputs are returned
    (reference: paddle.device.cuda.graphs.wrap_cuda_graph)."""
    from ...framework.tensor import Tensor, _wrap
    state = {"n": 0, "graph": None, "ins": None, "out": None, "key": None}

    def flat(args):
        return [a._t if isinstance(a, Tensor) else a for a in args]

    def wrapper(*args):
        ts = flat(args)
        key = tuple((tuple(t.shape), t.dtype) if isinstance(t, torch.Tensor) else ("c", t) for t in ts)
        if not torch.cuda.is_available() or not all(not isinstance(t, torch.Tensor) or t.is_cuda for t in ts):
            return function(*args)
        if state["graph"] is not None and key == state["key"]:
            for dst, src in zip(state["ins"], ts):
                if isinstance(dst, torch.Tensor):
                    dst.copy_(src)
            state["graph"].replay()
            return state["out"]
        state["n"] += 1
        if state["n"] < 2 or state["graph"] is not None:
            return function(*args)
        static = [t.clone() if isinstance(t, torch.Tensor) else t for t in ts]
        g = CUDAGraph(mode=mode)
        g.capture_begin()
        try:
            out = function(*[_wrap(t) if isinstance(t, torch.Tensor) else t for t in static])
        finally:
            g.capture_end()
        state.update(graph=g, ins=static, out=out, key=key)
        g.replay()
        return out

    return wrapper
