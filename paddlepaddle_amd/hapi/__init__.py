"""paddle.hapi: high-level Model API, callbacks, summary, flops."""
from .model import Model  # noqa: F401
from .model_summary import summary, flops  # noqa: F401
from . import callbacks  # noqa: F401
