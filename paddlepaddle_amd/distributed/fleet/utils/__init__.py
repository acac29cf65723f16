"""fleet.utils. Reference: python/paddle/distributed/fleet/utils/."""
from ..recompute import recompute  # noqa: F401
from . import sequence_parallel_utils  # noqa: F401
from .fs import LocalFS, HDFSClient, DistributedInfer  # noqa: F401,E402
from . import hybrid_parallel_util  # noqa: F401,E402
from . import mix_precision_utils  # noqa: F401,E402
from . import tensor_fusion_helper  # noqa: F401,E402
