"""HybridParallelOptimizer at its reference import path (python/paddle/distributed/fleet/meta_optimizers/
dygraph_optimizer/hybrid_parallel_optimizer.py); the implementation is fleet.fleet.HybridParallelOptimizer (what
fleet.distributed_optimizer returns): group-wide global-norm clip over mp / pp / sharding, sequence-parallel
gradient reduction."""
from ...fleet import HybridParallelOptimizer  # noqa: F401

__all__ = ["HybridParallelOptimizer"]
