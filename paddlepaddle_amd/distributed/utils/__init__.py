"""paddle.distributed.utils. Reference: python/paddle/distributed/utils/ (moe_utils, log_utils, launch_utils,
nccl_utils, stream_utils)."""
from . import launch_utils, log_utils, moe_utils, nccl_utils, stream_utils  # noqa: F401
from .moe_utils import global_gather, global_scatter  # noqa: F401

__all__ = []
