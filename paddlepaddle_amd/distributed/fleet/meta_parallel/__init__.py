"""fleet.meta_parallel. Reference: python/paddle/distributed/fleet/meta_parallel/__init__.py."""
from ....parallel.pipeline import (LayerDesc, SharedLayerDesc, PipelineLayer, PipelineParallel, SegmentLayers,  # noqa: F401
                                   PipelineParallelWithInterleave, PipelineParallelWithInterleaveFthenB,
                                   PipelineParallelZeroBubble, PipelineParallelZeroBubbleVPP)
from ....parallel.segment_parallel import SegmentParallel  # noqa: F401
from ....parallel.tensor_parallel import (ColumnParallelLinear, RowParallelLinear, VocabParallelEmbedding,  # noqa: F401
                                          ParallelCrossEntropy, get_rng_state_tracker, model_parallel_random_seed)
from ..fleet import TensorParallel  # noqa: F401
from ....parallel.sharding import GroupShardedModel as ShardingParallel  # noqa: F401
