"""paddle.distributed.ps: parameter-server training (sparse / dense tables on server processes).

Reference: python/paddle/distributed/ps/{the_one_ps.py,coordinator.py,utils/}. See the_one_ps.py for the
design; ``DistributedEmbedding`` is the eager-mode lookup layer (static.nn.sparse_embedding uses it).
"""
from .the_one_ps import (PsRuntime, PsClient, Communicator, sparse_lookup, get_runtime,  # noqa: F401
                         set_runtime)
from .layers import DistributedEmbedding, PsOptimizer  # noqa: F401

TheOnePSRuntime = PsRuntime

__all__ = ["PsRuntime", "TheOnePSRuntime", "PsClient", "Communicator", "DistributedEmbedding", "PsOptimizer",
           "sparse_lookup"]
