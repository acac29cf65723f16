"""paddle.incubate.distributed.models.moe (re-export of parallel/moe.py)."""
from ....parallel.moe import (MoELayer, BaseGate, NaiveGate, GShardGate, SwitchGate,  # noqa: F401
                              ClipGradForMOEByGlobalNorm)
