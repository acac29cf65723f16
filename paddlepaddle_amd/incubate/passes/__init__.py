"""paddle.incubate.passes. Reference: python/paddle/incubate/passes/__init__.py."""
from . import fuse_resnet_unit_pass  # noqa: F401
