"""Layout autotune (FLAGS_layout_autotune; paddle.incubate.autotune.set_config({"layout": {"enable": True}})).

Reference: paddle/fluid/imperative/layout_autotune.cc, paddle/fluid/eager/eager_layout_auto_tune.h:127 — under
autotune the reference rewrites NCHW convolution inputs to NHWC once, keeps layout-agnostic ops in NHWC and
transposes back at layout-sensitive ops.

MI355X design: the conv / batch-norm / max-pool HIP kernels are NHWC-native (csrc/kernels/gemm*.hip, bn.hip,
pool.hip). With autotune on, an NCHW-facing call on a device tensor keeps the tensor's LOGICAL shape NCHW but
gives it channels-last strides (one relayout at the first convolution), runs the NHWC kernel on the
zero-copy NHWC view, and hands back a logical-NCHW view of the NHWC result. Elementwise ops preserve
channels-last strides, so the activations stay channels-last from layer to layer without any transpose; a
layout-sensitive op (reshape / flatten / a kernel that needs contiguous NCHW) simply sees a strided NCHW tensor
and PyTorch-ROCm copies it where the op requires contiguity. User-visible shapes and semantics never change.
"""
from __future__ import annotations

import torch

from .flags import get_flags

_FLAG = "FLAGS_layout_autotune"


def enabled():
    try:
        return bool(get_flags(_FLAG)[_FLAG])
    except Exception:  # pragma: no cover
        return False


def applies(t, ndim=4):
    """Autotune this NCHW call: flag on, a 4-D floating device tensor."""
    return (isinstance(t, torch.Tensor) and t.dim() == ndim and t.is_cuda and t.is_floating_point()
            and enabled())


def to_nhwc_view(t):
    """Logical NCHW -> the NHWC view of its channels-last storage (relayout only if not channels-last yet)."""
    if t is None:
        return None
    if not t.is_contiguous(memory_format=torch.channels_last):
        t = t.contiguous(memory_format=torch.channels_last)
    return t.permute(0, 2, 3, 1)


def to_nchw_view(t):
    """NHWC -> logical NCHW with channels-last strides (no copy)."""
    return t.permute(0, 3, 1, 2)
