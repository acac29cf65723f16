"""paddle.incubate.checkpoint. Reference: python/paddle/incubate/checkpoint/__init__.py."""
from . import auto_checkpoint  # noqa: F401

__all__ = []
