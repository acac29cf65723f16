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


# Bias-gradient fusion: the gradient a dropout backward produces is, in a transformer block, the output gradient
# of the linear (out-proj / FFN2) whose output was dropped out, and that linear's backward needs its column sums.
# Once a linear backward has met such a gradient (key recorded here), the dropout backward of that key writes the
# column partials as it goes (pa_dropout_bwd_colsum) and the linear only folds them (ops/linear.py).
_WANT_CS: set = set()


def take_colsum(g):
    """(partials, nparts) written for ``g`` (or the tensor it views) by the dropout backward, else None."""
    t = g if hasattr(g, "_pa_cs_key") else g._base
    if t is None or not hasattr(t, "_pa_cs_key"):
        return None
    if t.data_ptr() != g.data_ptr() or t.numel() != g.numel() or t.shape[-1] != g.shape[-1]:
        return None
    rec = t._pa_cs
    if rec is None or rec[2] != t._version:
        _WANT_CS.add(t._pa_cs_key)
        return None
    t._pa_cs = None
    return rec[0], rec[1]


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
        cols = dyc.shape[-1] if dyc.dim() else 1
        rows = dyc.numel() // max(cols, 1)
        key = (rows, cols, dyc.dtype)
        cs = None
        if key in _WANT_CS and cols % 8 == 0 and L.has("pa_dropout_bwd_colsum"):
            nparts = int(L.lib().pa_colsum_nparts(rows))
            ws = torch.empty(nparts * cols, dtype=torch.float32, device=dyc.device)
            L.call("pa_dropout_bwd_colsum", L.ptr(dyc), L.ptr(dx), L.ptr(ws), rows, cols, float(ctx.p), ctx.seed,
                   L.dcode(dyc), L.stream_ptr())
            cs = (ws, nparts, dx._version)
        else:
            L.call("pa_dropout_bwd", L.ptr(dyc), L.ptr(dx), dyc.numel(), float(ctx.p), ctx.seed, L.dcode(dyc),
                   L.stream_ptr())
        dx._pa_cs_key, dx._pa_cs = key, cs
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
