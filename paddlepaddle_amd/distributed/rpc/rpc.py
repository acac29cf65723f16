"""Remote procedure calls between named workers.

Reference: python/paddle/distributed/rpc/rpc.py (init_rpc over a TCPStore rendezvous at
``master_endpoint`` — env PADDLE_TRAINER_ID / PADDLE_TRAINERS_NUM / PADDLE_MASTER_ENDPOINT — then
rpc_sync / rpc_async of a pickled Python callable on worker ``to``, FutureWrapper.wait(), WorkerInfo
name/rank/ip/port, shutdown() as a never-timing-out barrier) and paddle/fluid/distributed/rpc/ (a
brpc agent).

Here the transport is torch's TensorPipe agent: it moves CPU tensors without pickling their storage,
runs incoming calls on a thread pool (so a parameter server answers several trainers at once) and
its shutdown already joins every worker. Timeouts are in seconds; <= 0 means none (the reference's
convention). Like the reference, calls execute arbitrary Python on the peer: use on a trusted network.
"""
from __future__ import annotations

import os
import socket
from dataclasses import dataclass

import torch.distributed.rpc as _trpc

_DEFAULT_RPC_TIMEOUT = -1
_MAX_TIMEOUT_S = 7 * 24 * 3600
_STATE = {"name": None, "rank": None, "world": None}


@dataclass(frozen=True)
class WorkerInfo:
    name: str
    rank: int
    ip: str
    port: int

    def __repr__(self):
        return f"{{name: {self.name}, rank: {self.rank}, ip: {self.ip}, port: {self.port}}}"


class FutureWrapper:
    """Result handle of rpc_async (reference rpc.py _FutureWrapper): ``wait()`` returns fn's result or
    re-raises its exception."""

    def __init__(self, fut):
        self._fut = fut

    def wait(self):
        return self._fut.wait()

    def done(self):
        return self._fut.done()


def _timeout(timeout):
    return float(_MAX_TIMEOUT_S) if timeout is None or timeout <= 0 else float(timeout)


def init_rpc(name: str, rank: int | None = None, world_size: int | None = None,
             master_endpoint: str | None = None, num_worker_threads: int = 16) -> None:
    """Join the RPC group as ``name``. Blocks until all ``world_size`` workers have joined."""
    if _STATE["name"] is not None:
        raise RuntimeError("init_rpc called twice without shutdown()")
    rank = int(os.environ["PADDLE_TRAINER_ID"]) if rank is None else int(rank)
    world_size = int(os.environ["PADDLE_TRAINERS_NUM"]) if world_size is None else int(world_size)
    master_endpoint = master_endpoint or os.environ["PADDLE_MASTER_ENDPOINT"]
    addr, port = master_endpoint.rsplit(":", 1)
    timeout = int(os.getenv("FLAGS_stop_check_timeout", "900"))
    opts = _trpc.TensorPipeRpcBackendOptions(num_worker_threads=num_worker_threads, rpc_timeout=timeout,
                                             init_method=f"tcp://{addr}:{int(port)}")
    # CPU-only transports: tensors crossing RPC are host buffers (device tensors are staged by callers)
    opts._transports = ["uv"]
    opts._channels = ["basic"]
    _trpc.init_rpc(name, rank=rank, world_size=world_size, rpc_backend_options=opts)
    _STATE.update(name=name, rank=rank, world=world_size)


def _check():
    if _STATE["name"] is None:
        raise RuntimeError("rpc is not initialised: call paddle.distributed.rpc.init_rpc first")


def rpc_async(to: str, fn, args=None, kwargs=None, timeout: int = _DEFAULT_RPC_TIMEOUT) -> FutureWrapper:
    _check()
    return FutureWrapper(_trpc.rpc_async(to, fn, args=tuple(args or ()), kwargs=dict(kwargs or {}),
                                         timeout=_timeout(timeout)))


def rpc_sync(to: str, fn, args=None, kwargs=None, timeout: int = _DEFAULT_RPC_TIMEOUT):
    return rpc_async(to, fn, args, kwargs, timeout).wait()


def _info(w) -> WorkerInfo:
    # TensorPipe exposes names and ids; the endpoint is what this host would bind for the worker
    ip = os.getenv("POD_IP", "127.0.0.1")
    return WorkerInfo(w.name, int(w.id), ip, 0)


def get_worker_info(name: str) -> WorkerInfo:
    _check()
    return _info(_trpc.get_worker_info(name))


def get_all_worker_infos() -> list[WorkerInfo]:
    _check()
    agent = _trpc.api._get_current_rpc_agent()
    return sorted((_info(w) for w in agent.get_worker_infos()), key=lambda i: i.rank)


def get_current_worker_info() -> WorkerInfo:
    _check()
    return _info(_trpc.get_worker_info())


def shutdown() -> None:
    """Wait for every worker to reach shutdown and for all outstanding calls to finish, then stop."""
    if _STATE["name"] is None:
        return
    _trpc.shutdown(graceful=True)
    _STATE.update(name=None, rank=None, world=None)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
