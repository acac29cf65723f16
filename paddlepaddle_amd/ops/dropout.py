"""Fused dropout (+ residual add) with a counter-based RNG.

Reference: paddle/phi/kernels/fusion/gpu/fused_dropout_add_kernel.cu,
python/paddle/incubate/nn/functional/fused_dropout_add.py.
The keep-mask is a pure function of (seed, element index): forward draws a 64-bit seed from the
host generator (captured/restored by activation recompute like any RNG state) and the backward
regenerates the mask from it — no mask tensor is stored (saves 1 byte/element of activation memory).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _loader as L
from ..framework.trace_hook import static_op


def _seed():
    return int(torch.randint(0, 2 ** 62, (1,)).item())


class _DropoutAddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, p):
        xc = x.contiguous()
        rc = res.contiguous().to(x.dtype) if res is not None else None
        out = torch.empty_like(xc)
        seed = _seed()
        L.call("pa_dropout_add_fwd", L.ptr(xc), L.ptr(rc), L.ptr(out), xc.numel(), float(p), seed, L.dcode(xc),
               L.stream_ptr())
        ctx.seed, ctx.p, ctx.has_res = seed, p, res is not None
        return out

    @staticmethod
    def backward(ctx, dy):
        dyc = dy.contiguous()
        dx = torch.empty_like(dyc)
        L.call("pa_dropout_bwd", L.ptr(dyc), L.ptr(dx), dyc.numel(), float(ctx.p), ctx.seed, L.dcode(dyc),
               L.stream_ptr())
        return dx, (dy if ctx.has_res else None), None


@static_op
def dropout_add(x, residual, p, training=True):
    """residual + dropout(x, p) (upscale_in_train)."""
    if not training or p == 0.0:
        return x + residual if residual is not None else x
    if L.hip_enabled_for(x) and x.dtype in L._DT and x.numel() % 8 == 0 and \
            (residual is None or residual.shape == x.shape):
        return _DropoutAddFn.apply(x, residual, float(p))
    y = F.dropout(x, p, True)
    return y + residual if residual is not None else y
