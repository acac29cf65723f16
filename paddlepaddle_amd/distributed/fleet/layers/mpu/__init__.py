"""fleet.layers.mpu. Reference: python/paddle/distributed/fleet/layers/mpu/."""
from .....parallel.tensor_parallel import (ColumnParallelLinear, RowParallelLinear, VocabParallelEmbedding,  # noqa: F401
                                           ParallelCrossEntropy, get_rng_state_tracker, RNGStatesTracker,
                                           model_parallel_random_seed)
from . import mp_ops, random  # noqa: F401
