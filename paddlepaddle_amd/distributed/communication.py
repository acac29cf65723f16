"""paddle.distributed.communication (reference python/paddle/distributed/communication/): the collective
API re-exported, plus the ``stream`` namespace (sync_op / use_calc_stream variants)."""
from .collective import *  # noqa: F401,F403
from .collective import (all_reduce, all_gather, broadcast, reduce, reduce_scatter, scatter, gather,  # noqa: F401
                         alltoall, alltoall_single, send, recv, isend, irecv, ReduceOp)


class stream:
    """communication.stream.*: same collectives; ``sync_op=False`` returns the async task."""
    all_reduce = staticmethod(all_reduce)
    all_gather = staticmethod(all_gather)
    broadcast = staticmethod(broadcast)
    reduce = staticmethod(reduce)
    reduce_scatter = staticmethod(reduce_scatter)
    scatter = staticmethod(scatter)
    gather = staticmethod(gather)
    alltoall = staticmethod(alltoall)
    alltoall_single = staticmethod(alltoall_single)
    send = staticmethod(send)
    recv = staticmethod(recv)
