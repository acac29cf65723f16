"""paddle.geometric.sampling. Reference: python/paddle/geometric/sampling/__init__.py."""
from .. import sample_neighbors, weighted_sample_neighbors  # noqa: F401

__all__ = []
