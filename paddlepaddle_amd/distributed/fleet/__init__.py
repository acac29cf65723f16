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
is_server = fleet.is_server
is_worker = fleet.is_worker
init_server = fleet.init_server
run_server = fleet.run_server
init_worker = fleet.init_worker
stop_worker = fleet.stop_worker
server_num = fleet.server_num
server_index = fleet.server_index
server_endpoints = fleet.server_endpoints
load_model = fleet.load_model
shrink = fleet.shrink


class PaddleCloudRoleMaker:
    """Role from the environment (reference fleet/base/role_maker.py PaddleCloudRoleMaker): collective mode
    uses the torch.distributed env; PS mode reads TRAINING_ROLE, PADDLE_PSERVERS_IP_PORT_LIST,
    PADDLE_TRAINERS_NUM, PADDLE_TRAINER_ID, POD_IP / PADDLE_PORT (parsed by distributed.ps.PsRuntime)."""

    def __init__(self, is_collective=False, **k):
        self.is_collective = is_collective
        self._kwargs = k


class UserDefinedRoleMaker(PaddleCloudRoleMaker):
    """Explicit role (reference UserDefinedRoleMaker): current_id, role (Role.WORKER / Role.SERVER),
    worker_num, server_endpoints."""

    def __init__(self, is_collective=False, init_gloo=False, current_id=0, role=None, worker_num=1,
                 server_endpoints=None, worker_endpoints=None, **k):
        super().__init__(is_collective=is_collective, **k)
        self._current_id = int(current_id)
        self._role = "PSERVER" if role == Role.SERVER else "TRAINER"
        self._worker_num = int(worker_num)
        self._server_endpoints = ",".join(server_endpoints or [])
        self._worker_endpoints = list(worker_endpoints or [])


class Role:
    WORKER = 1
    SERVER = 2
    HETER_WORKER = 3
    ALL = 4
    COORDINATOR = 5


class UtilBase:
    """fleet.util: all_reduce / barrier / all_gather helpers over the default group (reference
    fleet/base/util_factory.py UtilBase)."""

    def all_reduce(self, input, mode="sum", comm_world="worker"):
        import numpy as np
        import torch
        import torch.distributed as dist
        t = torch.as_tensor(np.asarray(input), dtype=torch.float64)
        if dist.is_initialized():
            op = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[mode]
            dist.all_reduce(t, op=op)
        return t.numpy()

    def barrier(self, comm_world="worker"):
        import torch.distributed as dist
        if dist.is_initialized():
            dist.barrier()

    def all_gather(self, input, comm_world="worker"):
        import torch.distributed as dist
        if not dist.is_initialized():
            return [input]
        out = [None] * dist.get_world_size()
        dist.all_gather_object(out, input)
        return out

    def get_file_shard(self, files):
        import torch.distributed as dist
        r, n = (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)
        return files[r::n]

    def print_on_rank(self, message, rank_id):
        import torch.distributed as dist
        if (dist.get_rank() if dist.is_initialized() else 0) == rank_id:
            print(message)


util = UtilBase()
Fleet = type(fleet)


class MultiSlotDataGenerator:
    """PS data generator (reference fleet/data_generator): subclasses implement generate_sample(line)
    returning an iterator of [(slot_name, [values...]), ...]; run_from_memory / run_from_stdin print the
    MultiSlot text format."""

    def __init__(self):
        self._proto_info = None
        self.batch_size_ = 32

    def set_batch(self, batch_size):
        self.batch_size_ = batch_size

    def generate_sample(self, line):
        raise NotImplementedError

    def generate_batch(self, samples):
        def it():
            for s in samples:
                yield s
        return it

    def _format(self, sample):
        out = []
        for name, vals in sample:
            out.append(str(len(vals)))
            out.extend(str(v) for v in vals)
        return " ".join(out)

    def run_from_memory(self, lines=None):
        res = []
        for line in lines or []:
            for s in self.generate_sample(line)():
                res.append(self._format(s))
        return res

    def run_from_stdin(self):
        import sys
        for line in sys.stdin:
            for s in self.generate_sample(line)():
                sys.stdout.write(self._format(s) + "\n")


class MultiSlotStringDataGenerator(MultiSlotDataGenerator):
    pass
