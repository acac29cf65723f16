"""paddle.incubate.distributed.models.moe (re-export of parallel/moe.py)."""
from ....parallel.moe import (MoELayer, BaseGate, NaiveGate, GShardGate, SwitchGate, GroupedExperts,  # noqa: F401
                              ClipGradForMOEByGlobalNorm)
