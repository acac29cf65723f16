"""paddle.incubate.layers. Reference: python/paddle/incubate/layers/__init__.py."""
from . import nn  # noqa: F401
from .nn import (_pull_box_sparse, _pull_gpups_sparse, batch_fc, correlation, fused_bn_add_act,  # noqa: F401
                 fused_seqpool_cvm, partial_concat, partial_sum, pow2_decay_with_linear_warmup, rank_attention,
                 search_pyramid_hash, shuffle_batch, tdm_child, tdm_sampler)

__all__ = []
