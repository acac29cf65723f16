"""paddle.distributed. Reference: python/paddle/distributed/__init__.py."""
from .collective import (ReduceOp, Group, ParallelEnv, init_parallel_env, get_rank, get_world_size,  # noqa: F401
                         is_initialized, is_available, new_group, get_group, barrier, destroy_process_group,
                         all_reduce, all_gather, all_gather_object, all_gather_into_tensor, broadcast,
                         broadcast_object_list, reduce, reduce_scatter, scatter, scatter_object_list, gather,
                         alltoall, alltoall_single, send, recv, isend, irecv, P2POp, batch_isend_irecv, wait,
                         get_backend, get_global_rank)
