"""paddle.geometric.message_passing. Reference: python/paddle/geometric/message_passing/__init__.py."""
from .. import send_u_recv, send_ue_recv, send_uv  # noqa: F401

__all__ = []
