"""paddle.incubate. Reference: python/paddle/incubate/__init__.py (LookAhead, ModelAverage,
softmax_mask_fuse(_upper_triangle), graph_* / segment_* ops, identity_loss, nn, asp, autograd,
distributed.models.moe)."""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor, _wrap
from . import nn  # noqa: F401
from .optimizer import LookAhead, ModelAverage  # noqa: F401
from . import optimizer, asp, autograd, autotune  # noqa: F401
from . import distributed  # noqa: F401
from .operators import (graph_khop_sampler, graph_reindex, graph_sample_neighbors, graph_send_recv,  # noqa: F401
                        softmax_mask_fuse, softmax_mask_fuse_upper_triangle, ResNetUnit)
from .tensor import segment_sum, segment_mean, segment_max, segment_min  # noqa: F401
from . import operators, layers, framework, checkpoint, jit, multiprocessing, tensor, xpu, passes  # noqa: F401
from .framework import get_rng_state, set_rng_state, register_rng_state_as_index  # noqa: F401
from .checkpoint import auto_checkpoint  # noqa: F401
from .jit import inference  # noqa: F401,F811
from .passes import fuse_resnet_unit_pass  # noqa: F401


def identity_loss(x, reduction="none"):
    t = x._t
    if reduction in ("mean", 1):
        return _wrap(t.mean())
    if reduction in ("sum", 0):
        return _wrap(t.sum())
    return x
