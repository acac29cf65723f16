"""paddle.distributed.auto_parallel (semi-automatic SPMD parallelism)."""
from .placement_type import Shard, Replicate, Partial, Placement, ReduceType  # noqa: F401
from .process_mesh import ProcessMesh, get_mesh, set_mesh, get_current_process_mesh  # noqa: F401
from .api import (shard_tensor, dtensor_from_local, dtensor_to_local, dtensor_from_fn, reshard,  # noqa: F401
                  unshard_dtensor, shard_layer, shard_optimizer, shard_scaler, ShardingStage1, ShardingStage2,
                  ShardingStage3, shard_dataloader, ShardDataloader, Strategy, DistModel, to_static,
                  in_auto_parallel_align_mode)
from .intermediate import (parallelize, parallelize_model, parallelize_optimizer, ColWiseParallel,  # noqa: F401,E402
                           RowWiseParallel, PrepareLayerInput, PrepareLayerOutput, SequenceParallelBegin,
                           SequenceParallelEnd, SequenceParallelEnable, SequenceParallelDisable, SplitPoint)
from .interface import recompute, exclude_ops_in_recompute  # noqa: F401,E402
