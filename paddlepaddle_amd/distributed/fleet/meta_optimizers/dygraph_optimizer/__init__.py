"""fleet.meta_optimizers.dygraph_optimizer. Reference: python/paddle/distributed/fleet/meta_optimizers/
dygraph_optimizer/__init__.py."""
from .dygraph_sharding_optimizer import DygraphShardingOptimizer, DygraphShardingOptimizerV2  # noqa: F401
from .hybrid_parallel_optimizer import HybridParallelOptimizer  # noqa: F401
