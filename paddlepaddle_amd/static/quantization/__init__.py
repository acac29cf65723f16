"""paddle.static.quantization. Reference: python/paddle/static/quantization/__init__.py (post-training
quantization, quant_aware / convert, weight quantization). The graph passes of the reference
(QuantizationTransformPass, ... — IrGraph rewrites) are what quant_aware / convert / quantize() perform on this
framework's Program nodes; the oneDNN int8 passes are CPU-inference specific and not provided."""
from .post_training_quantization import (PostTrainingQuantization, PostTrainingQuantizationProgram,  # noqa: F401
                                         WeightQuantization)
from .quanter import convert, quant_aware  # noqa: F401
from . import quant_ops  # noqa: F401
