"""paddle.distributed.fleet. Reference: python/paddle/distributed/fleet/__init__.py."""
from .recompute import recompute, recompute_sequential, recompute_hybrid  # noqa: F401
from .fleet import fleet, DistributedStrategy, HybridParallelOptimizer, TensorParallel  # noqa: F401
from .topology import CommunicateTopology, HybridCommunicateGroup, ParallelMode  # noqa: F401
from . import meta_parallel, layers, utils  # noqa: F401

init = fleet.init
distributed_model = fleet.distributed_model
distributed_optimizer = fleet.distributed_optimizer
distributed_scaler = fleet.distributed_scaler
get_hybrid_communicate_group = fleet.get_hybrid_communicate_group
worker_index = fleet.worker_index
worker_num = fleet.worker_num
is_first_worker = fleet.is_first_worker
barrier_worker = fleet.barrier_worker
local_rank = fleet.local_rank
save_persistables = fleet.save_persistables
save_inference_model = fleet.save_inference_model


class UserDefinedRoleMaker:
    def __init__(self, *a, **k):
        pass


class PaddleCloudRoleMaker:
    def __init__(self, is_collective=True, **k):
        self.is_collective = is_collective


class Role:
    WORKER = 1
    SERVER = 2
    HETER_WORKER = 3
    ALL = 4
    COORDINATOR = 5
