from . import models  # noqa: F401


class fleet:  # paddle.incubate.distributed.fleet: recompute helpers (reference incubate/distributed/fleet)
    from ...distributed.fleet.recompute import recompute_sequential, recompute_hybrid  # noqa: F401


import sys as _sys  # noqa: E402
_sys.modules[__name__ + ".fleet"] = fleet
