"""fleet.utils. Reference: python/paddle/distributed/fleet/utils/."""
from ..recompute import recompute  # noqa: F401
from . import sequence_parallel_utils  # noqa: F401
from .fs import LocalFS, HDFSClient, DistributedInfer  # noqa: F401,E402
