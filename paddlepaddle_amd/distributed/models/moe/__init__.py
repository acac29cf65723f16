"""paddle.distributed.models.moe. Reference: python/paddle/distributed/models/moe/."""
from . import utils  # noqa: F401
from ....parallel.moe import MoELayer, BaseGate, NaiveGate, GShardGate, SwitchGate  # noqa: F401
