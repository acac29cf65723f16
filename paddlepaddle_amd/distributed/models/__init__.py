"""paddle.distributed.models. Reference: python/paddle/distributed/models/__init__.py."""
from . import moe  # noqa: F401
