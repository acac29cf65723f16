"""paddle.distributed.rpc. Reference: python/paddle/distributed/rpc/__init__.py."""
from .rpc import (get_all_worker_infos, get_current_worker_info, get_worker_info, init_rpc, rpc_async,  # noqa: F401
                  rpc_sync, shutdown, WorkerInfo, FutureWrapper)

__all__ = ["init_rpc", "shutdown", "rpc_async", "rpc_sync", "get_worker_info", "get_all_worker_infos",
           "get_current_worker_info"]
