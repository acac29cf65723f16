"""paddle.nn.functional. Reference: python/paddle/nn/functional/__init__.py."""
from .activation import *  # noqa: F401,F403
from .common import *  # noqa: F401,F403
from .conv import *  # noqa: F401,F403
from .distance import *  # noqa: F401,F403
from .flash_attention import (flash_attention, scaled_dot_product_attention, flash_attn_unpadded,  # noqa: F401
                              flash_attn_qkvpacked, flash_attention_with_sparse_mask,
                              calc_reduced_attention_scores)
from .loss import *  # noqa: F401,F403
from .norm import *  # noqa: F401,F403
from .pooling import *  # noqa: F401,F403
from .vision import *  # noqa: F401,F403
from ...tensor.math import sigmoid, tanh  # noqa: F401
from ...tensor.manipulation import unfold as _tensor_unfold  # noqa: F401
from .common import unfold  # noqa: F401,E402
from .extension import *  # noqa: F401,F403,E402
