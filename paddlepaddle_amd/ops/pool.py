"""Max pooling over channels-last activations (csrc/kernels/pool.hip).

Reference: paddle/phi/kernels/funcs/pooling.cu (max_pool2d / max_pool2d_with_index). ResNet's stem pool
(3x3, stride 2, padding 1 on [N, 112, 112, 64] NHWC) is the target shape: the forward stores the window
offset of each maximum (uint8) and the backward gathers dy per input pixel (no zero-fill, no scatter).
"""
from __future__ import annotations

import torch

from . import _loader as L


class _MaxPoolNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        N, H, W, C = x.shape
        Ho = (H + 2 * p - k) // s + 1
        Wo = (W + 2 * p - k) // s + 1
        y = torch.empty(N, Ho, Wo, C, dtype=x.dtype, device=x.device)
        arg = torch.empty(N, Ho, Wo, C, dtype=torch.uint8, device=x.device)
        L.call("pa_maxpool_nhwc_fwd", L.ptr(x), L.ptr(y), L.ptr(arg), N, H, W, C, Ho, Wo, k, s, p, L.dcode(x),
               L.stream_ptr())
        ctx.save_for_backward(arg)
        ctx.cfg = (N, H, W, C, Ho, Wo, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        N, H, W, C, Ho, Wo, k, s, p = ctx.cfg
        dy = dy.contiguous()
        dx = torch.empty(N, H, W, C, dtype=dy.dtype, device=dy.device)
        L.call("pa_maxpool_nhwc_bwd", L.ptr(dy), L.ptr(arg), L.ptr(dx), N, H, W, C, Ho, Wo, k, s, p, L.dcode(dy),
               L.stream_ptr())
        return dx, None, None, None


def maxpool2d_nhwc_supported(x, k, s, p, dilation=1, ceil_mode=False, return_mask=False):
    return (isinstance(k, int) and isinstance(s, int) and isinstance(p, int) and dilation == 1 and not ceil_mode
            and not return_mask and x.dim() == 4 and x.is_contiguous() and x.dtype in (torch.bfloat16, torch.float16)
            and x.shape[3] % 8 == 0 and 1 <= k and k * k <= 255 and s >= 1 and 0 <= 2 * p <= k
            and L.has("pa_maxpool_nhwc_fwd") and L.hip_enabled_for(x))


def maxpool2d_nhwc(x, k, s, p):
    """x [N, H, W, C] -> [N, Ho, Wo, C]."""
    return _MaxPoolNHWC.apply(x, k, s, p)
