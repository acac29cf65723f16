"""paddle.distributed. Reference: python/paddle/distributed/__init__.py."""
from .collective import (ReduceOp, Group, ParallelEnv, init_parallel_env, get_rank, get_world_size,  # noqa: F401
                         is_initialized, is_available, new_group, get_group, barrier, destroy_process_group,
                         all_reduce, all_gather, all_gather_object, all_gather_into_tensor, broadcast,
                         broadcast_object_list, reduce, reduce_scatter, scatter, scatter_object_list, gather,
                         alltoall, alltoall_single, send, recv, isend, irecv, P2POp, batch_isend_irecv, wait,
                         get_backend, get_global_rank)
from .auto_parallel import (ProcessMesh, Shard, Replicate, Partial, Placement, ReduceType, shard_tensor,  # noqa
                            dtensor_from_local, dtensor_from_fn, reshard, unshard_dtensor, shard_layer,
                            shard_optimizer, shard_scaler, ShardingStage1, ShardingStage2, ShardingStage3,
                            shard_dataloader, Strategy, DistModel, to_static, get_mesh, set_mesh)
from . import auto_parallel  # noqa: F401
from .auto_parallel.intermediate import (parallelize, ColWiseParallel, RowWiseParallel,  # noqa: F401,E402
                                         PrepareLayerInput, PrepareLayerOutput, SequenceParallelBegin,
                                         SequenceParallelEnd, SequenceParallelEnable, SequenceParallelDisable,
                                         SplitPoint)
from ..parallel.data_parallel import DataParallel  # noqa: F401,E402
from .fleet.utils.hybrid_parallel_util import sync_params_buffers  # noqa: F401,E402
from .extras import *  # noqa: F401,F403,E402
from . import communicator  # noqa: F401,E402
from .watchdog import enable_comm_watchdog, disable_comm_watchdog  # noqa: F401,E402
from .collective_check import (enable_collective_check, disable_collective_check, check_collectives,  # noqa: F401,E402
                               CollectiveMismatchError)


def __getattr__(name):
    # heavier subsystems are imported on first use (fleet pulls in pipeline/TP layers)
    import importlib
    if name in ("fleet", "sharding", "checkpoint", "launch", "spawn_mod", "utils", "communication", "rpc", "ps",
                "elastic"):
        mod = importlib.import_module(f".{name}", __name__)
        globals()[name] = mod
        return mod
    if name == "stream":  # paddle.distributed.stream: collectives with sync_op / use_calc_stream semantics
        from . import communication
        globals()["stream"] = communication.stream
        return communication.stream
    if name in ("save_state_dict", "load_state_dict"):
        from . import checkpoint
        return getattr(checkpoint, name)
    if name == "spawn":
        from .spawn import spawn
        return spawn
    if name == "group_sharded_parallel":
        from ..parallel.sharding import group_sharded_parallel
        return group_sharded_parallel
    raise AttributeError(name)
