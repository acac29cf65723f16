"""HIP graph capture/replay. Reference: python/paddle/device/cuda/graphs.py (CUDAGraph).
On MI355X: hipGraph via the runtime's graph API — the replacement for a tracing compiler
for launch-bound inner loops."""
from __future__ import annotations

import torch


def is_cuda_graph_supported():
    return torch.cuda.is_available()


class CUDAGraph:
    def __init__(self, place=None, mode="thread_local", pool_id=None):
        self._g = torch.cuda.CUDAGraph()
        self._stream = None
        self._ctx = None
        self._pool = pool_id

    def capture_begin(self):
        self._stream = torch.cuda.Stream()
        self._stream.wait_stream(torch.cuda.current_stream())
        self._ctx = torch.cuda.stream(self._stream)
        self._ctx.__enter__()
        self._g.capture_begin(pool=self._pool)

    def capture_end(self):
        self._g.capture_end()
        self._ctx.__exit__(None, None, None)
        torch.cuda.current_stream().wait_stream(self._stream)

    def replay(self):
        self._g.replay()

    def reset(self):
        self._g.reset()

    def pool(self):
        return self._g.pool()

    def print_to_dot_files(self, dirname, flags=None):
        self._g.debug_dump(str(dirname) + "/graph.dot")


def wrap_cuda_graph(function, mode="thread_local", memory_pool="default"):
    return function
