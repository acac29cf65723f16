"""paddle.distributed.passes: pass framework + registered program passes (reference
python/paddle/distributed/passes/__init__.py). See pass_base.py and program_passes.py."""
from .pass_base import PassBase, PassContext, PassManager, PassType, new_pass, register_pass  # noqa: F401
from .program_passes import (  # noqa: F401
    AMPPass, DeadCodeEliminationPass, FP16Pass, FuseGemmEpiloguePass, GradientMergePass,
)
from . import pipeline_scheduler  # noqa: F401  (pipeline_scheduler_* passes)
from . import fusion_passes  # noqa: F401  (fused_feedforward / fused_attention / ... and auto-parallel passes)
from . import conv_passes  # noqa: F401  (fuse_relu_depthwise_conv / fuse_resunit)

__all__ = ["new_pass", "PassManager", "PassContext"]
