"""paddle.distributed.communication (reference python/paddle/distributed/communication/): the collective
API re-exported, plus the ``stream`` namespace (sync_op / use_calc_stream variants)."""
from .collective import *  # noqa: F401,F403
from .collective import (all_reduce, all_gather, broadcast, reduce, reduce_scatter, scatter, gather,  # noqa: F401
                         alltoall, alltoall_single, send, recv, isend, irecv, ReduceOp)


def is_avg_reduce_op_supported():
    """ReduceOp.AVG runs natively on RCCL (the DP / sharding paths use it; gloo gets SUM + scale)."""
    return True


from . import comm_stream as stream  # noqa: E402  (explicit sync_op / use_calc_stream semantics)

import sys as _sys  # noqa: E402
_sys.modules[__name__ + ".stream"] = stream
__path__ = []  # submodules above are importable by dotted name
