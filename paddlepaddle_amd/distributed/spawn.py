"""paddle.distributed.spawn. Reference: python/paddle/distributed/spawn.py.
One process per GPU (the MI355X execution model): each child gets RANK / WORLD_SIZE / LOCAL_RANK /
MASTER_ADDR / MASTER_PORT (+ the PADDLE_* equivalents) and initialises RCCL on first collective."""
from __future__ import annotations

import os
import socket

import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, func, args, world, port, env):
    os.environ.update(env)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), PADDLE_TRAINER_ID=str(rank), PADDLE_TRAINERS_NUM=str(world),
                      PADDLE_LOCAL_RANK=str(rank), HSA_ENABLE_IPC_MODE_LEGACY="0")
    if "HIP_VISIBLE_DEVICES" not in env and os.environ.get("PADDLE_AMD_FORCE_CPU") != "1":
        os.environ.setdefault("PADDLE_AMD_DEVICE_ID", str(rank))
    func(*args)


class MultiprocessContext:
    def __init__(self, ctx):
        self._ctx = ctx

    def join(self, timeout=None):
        return self._ctx.join(timeout)

    @property
    def processes(self):
        return self._ctx.processes


def spawn(func, args=(), nprocs=-1, join=True, daemon=False, **options):
    if nprocs == -1:
        import torch
        nprocs = max(torch.cuda.device_count(), 1)
    port = int(options.get("master_port", _free_port()))
    env = {k: v for k, v in os.environ.items() if k.startswith(("PADDLE_", "HIP_", "HSA_", "FLAGS_"))}
    ctx = mp.start_processes(_entry, args=(func, tuple(args), nprocs, port, env), nprocs=nprocs, join=join,
                             daemon=daemon, start_method="spawn")
    return MultiprocessContext(ctx) if ctx is not None else None
