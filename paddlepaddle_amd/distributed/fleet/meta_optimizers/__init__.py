"""fleet.meta_optimizers. Reference: python/paddle/distributed/fleet/meta_optimizers/ (the dygraph wrappers that
PaddleNLP imports directly)."""
from .dygraph_optimizer import (DygraphShardingOptimizer, DygraphShardingOptimizerV2,  # noqa: F401
                                HybridParallelOptimizer)
