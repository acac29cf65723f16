"""fleet.layers.mpu. Reference: python/paddle/distributed/fleet/layers/mpu/."""
from .....parallel.tensor_parallel import (ColumnParallelLinear, RowParallelLinear, VocabParallelEmbedding,  # noqa: F401
                                           ParallelCrossEntropy, get_rng_state_tracker, RNGStatesTracker,
                                           model_parallel_random_seed)
from . import mp_ops, random  # noqa: F401


def is_fused_matmul_bias_supported():
    """The linear layers' bias add runs in the GEMM epilogue on MI355X (reference mp_layers.py)."""
    return True


def is_fused_linear_param_grad_add_supported():
    """Weight gradients accumulate into main_grad inside the wgrad GEMM (FLAGS_fused_grad_accumulation)."""
    return True
