"""Hot-op layer: hand-written CDNA4 HIP kernels with autograd, plus the CPU reference paths.

Every function here takes/returns *device buffers* (torch tensors) — the paddle Tensor wrapper is
applied by the callers in ``nn.functional`` / ``incubate``. On a HIP device the kernel in
``csrc/kernels`` runs (see ``_loader.hip_enabled_for``); on CPU the reference math runs.
"""
from __future__ import annotations

from .activation import gelu, silu, swiglu, softmax, bias_gelu  # noqa: F401
from .norm import rms_norm, rms_norm_residual, layer_norm, layer_norm_residual, add_rms_norm  # noqa: F401
from .loss import softmax_cross_entropy  # noqa: F401
from .attention import flash_attention, attention_bhsd, flash_attention_qkvpacked, qkv_rope_attention, attention_reference, paged_decode_attention, dense_decode_attention  # noqa: F401,E501
from .rope import apply_rotary, decode_rope_cache  # noqa: F401
from .linear import fused_linear, colsum, linear_nt, ffn_gelu  # noqa: F401
from .lm_head import lm_head_cross_entropy  # noqa: F401
from .dropout import dropout_add  # noqa: F401
from . import optim  # noqa: F401
from ._loader import has as has_kernel, hip_enabled_for, LIB_PATH  # noqa: F401
from .bn import batch_norm_act_nhwc  # noqa: F401
from . import conv, gemm, dwconv, quant  # noqa: F401,E402
