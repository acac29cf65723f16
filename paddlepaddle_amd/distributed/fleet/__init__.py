"""paddle.distributed.fleet (filled in by fleet.py)."""
from .recompute import recompute, recompute_sequential, recompute_hybrid  # noqa: F401
