"""paddle.distributed.sharding. Reference: python/paddle/distributed/sharding/group_sharded.py."""
from ..parallel.sharding import group_sharded_parallel, save_group_sharded_model  # noqa: F401
