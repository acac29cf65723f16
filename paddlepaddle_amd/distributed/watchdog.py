"""Collective-communication watchdog (failure / hang detection).

Reference: paddle/phi/core/distributed/comm_task_manager.cc + comm_task.h (CommTaskManager: background
thread over the outstanding comm tasks' events; timeouts are reported with op / rank / group / size and
can abort the job).

``enable_comm_watchdog()`` wraps the torch.distributed collectives that every layer of this framework
calls (DataParallel buckets, the sharding engine's all-gather / reduce-scatter, pipeline p2p, the
paddle.distributed API): a GPU collective gets a HIP event recorded on the stream that consumes its
result (for async ops: when the work is waited on), a CPU (gloo) collective is tracked from entry to
return. The native thread in ``_C_runtime.comm_watchdog`` polls the events and reports every collective
still pending after the timeout (stderr + ``<report_dir>/comm_watchdog.rank<r>.txt``); with
``abort=True`` it aborts the process so the launcher's failure detection restarts the job.
Auto-enabled by ``PADDLE_AMD_COMM_WATCHDOG=<timeout seconds>`` at init_parallel_env.
"""
from __future__ import annotations

import functools
import os

import torch
import torch.distributed as dist

_OPS = ("all_reduce", "all_gather", "all_gather_into_tensor", "reduce_scatter_tensor", "reduce_scatter",
        "broadcast", "reduce", "all_to_all", "all_to_all_single", "send", "recv", "isend", "irecv", "barrier",
        "gather", "scatter")
_ORIG = {}
_STATE = {"on": False}


def _native():
    from ..utils import native
    m = native.module()
    if m is None or not hasattr(m, "comm_watchdog"):
        raise RuntimeError("native runtime (_C_runtime) with comm_watchdog is not built")
    return m.comm_watchdog


def _first_tensor(args, kwargs):
    for a in list(args) + list(kwargs.values()):
        if isinstance(a, torch.Tensor):
            return a
        if isinstance(a, (list, tuple)) and a and isinstance(a[0], torch.Tensor):
            return a[0]
    return None


def _nbytes(args, kwargs):
    n = 0
    for a in list(args) + list(kwargs.values()):
        if isinstance(a, torch.Tensor):
            n += a.numel() * a.element_size()
        elif isinstance(a, (list, tuple)):
            n += sum(x.numel() * x.element_size() for x in a if isinstance(x, torch.Tensor))
    return n


def _gname(kwargs):
    g = kwargs.get("group")
    if g is None:
        return "world"
    try:
        return f"group[{','.join(str(r) for r in dist.get_process_group_ranks(g))}]"
    except Exception:  # pragma: no cover
        return "group"


class _WorkProxy:
    """Async work handle: tracking starts when the caller waits (the point from which the current
    stream depends on the collective)."""

    def __init__(self, work, op, group, nbytes, dev):
        self._w, self._op, self._g, self._n, self._dev = work, op, group, nbytes, dev

    def wait(self, *a, **k):
        r = self._w.wait(*a, **k)
        if self._dev:
            _native().track(self._op, self._g, self._n, torch.cuda.current_stream().cuda_stream, 0)
        return r

    def __getattr__(self, k):
        return getattr(self._w, k)


def _wrap(name, fn):
    @functools.wraps(fn)
    def w(*args, **kwargs):
        if not _STATE["on"]:
            return fn(*args, **kwargs)
        wd = _native()
        t = _first_tensor(args, kwargs)
        dev = t is not None and t.is_cuda
        nbytes = _nbytes(args, kwargs)
        gname = _gname(kwargs)
        is_async = kwargs.get("async_op", False) or name in ("isend", "irecv")
        if dev:
            work = fn(*args, **kwargs)
            if is_async and work is not None:
                return _WorkProxy(work, name, gname, nbytes, True)
            wd.track(name, gname, nbytes, torch.cuda.current_stream().cuda_stream, 0)
            return work
        tid = wd.track_host(name, gname, nbytes, 0)
        try:
            work = fn(*args, **kwargs)
        except BaseException:
            wd.finish(tid)
            raise
        if is_async and work is not None:
            orig_wait = work.wait

            def wait(*a, **k):
                try:
                    return orig_wait(*a, **k)
                finally:
                    wd.finish(tid)
            try:
                work.wait = wait
            except AttributeError:
                wd.finish(tid)
            return work
        wd.finish(tid)
        return work
    return w


def enable_comm_watchdog(timeout_s=600.0, poll_ms=500, abort=False, report_dir=None):
    """Start the native watchdog and route torch.distributed collectives through it."""
    rank = dist.get_rank() if dist.is_initialized() else int(os.environ.get("RANK", "0"))
    _native().start(rank, int(timeout_s * 1000), int(poll_ms), bool(abort), report_dir or "")
    if not _ORIG:
        for n in _OPS:
            f = getattr(dist, n, None)
            if f is not None:
                _ORIG[n] = f
                setattr(dist, n, _wrap(n, f))
    _STATE["on"] = True


def disable_comm_watchdog():
    _STATE["on"] = False
    for n, f in _ORIG.items():
        setattr(dist, n, f)
    _ORIG.clear()
    try:
        _native().stop()
    except RuntimeError:
        pass


def status():
    """(pending tasks, timeouts so far, ops that timed out)."""
    wd = _native()
    return wd.pending(), wd.timeouts(), list(wd.timed_out_ops())
