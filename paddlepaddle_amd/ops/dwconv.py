"""Depthwise 2-D convolution on NHWC tensors (groups == C_in == C_out) with the HIP kernels of
csrc/kernels/dwconv.hip: forward, data gradient and split weight gradient (fp32 lane partials folded by
pa_reduce_parts), bias gradient by the column-sum kernel. Reference: paddle/phi/kernels/gpu/depthwise_conv.h.
Chosen per shape against MIOpen by measured time (ops/gemm.py choose), like the other hand-written convs."""
from __future__ import annotations

import torch

from . import _loader as L
from . import gemm as G
from .linear import colsum

__all__ = ["eligible", "depthwise_conv2d_nhwc"]


def eligible(x, w, groups):
    if not (L.hip_enabled_for(x) and L.has("pa_dwconv_fwd") and x.dtype in L._DT and w.dtype == x.dtype):
        return False
    if x.dim() != 4 or w.dim() != 4 or not x.is_contiguous():
        return False
    C = x.shape[3]
    return groups == C and w.shape[0] == C and w.shape[1] == 1 and C % 8 == 0 and x.numel() > 0


def _shape(x, w, stride, pad, dil, relu=False):
    N, H, W, C = x.shape
    KH, KW = int(w.shape[2]), int(w.shape[3])
    Ho = (H + 2 * pad[0] - dil[0] * (KH - 1) - 1) // stride[0] + 1
    Wo = (W + 2 * pad[1] - dil[1] * (KW - 1) - 1) // stride[1] + 1
    return torch.tensor([N, H, W, C, Ho, Wo, KH, KW, stride[0], stride[1], pad[0], pad[1], dil[0], dil[1],
                         int(bool(relu))], dtype=torch.int32), Ho, Wo


class _DWConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad, dil, relu=False):
        N, H, W, C = x.shape
        shp, Ho, Wo = _shape(x, w, stride, pad, dil, relu)
        wt = w.reshape(C, -1).t().contiguous()  # [KH*KW, C]: one tap's 8 channel weights per vector load
        y = torch.empty(N, Ho, Wo, C, dtype=x.dtype, device=x.device)
        L.call("pa_dwconv_fwd", L.ptr(x), L.ptr(wt), L.ptr(None if b is None else b.contiguous()), L.ptr(y),
               L.ptr(shp), L.dcode(x), L.stream_ptr())
        ctx.save_for_backward(x, wt)
        ctx.shp, ctx.wshape, ctx.has_b = shp, w.shape, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wt = ctx.saved_tensors
        shp = ctx.shp
        dy = dy.contiguous().to(x.dtype)
        C = x.shape[3]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            L.call("pa_dwconv_dgrad", L.ptr(dy), L.ptr(wt), L.ptr(x), L.ptr(dx), L.ptr(shp), L.dcode(x),
                   L.stream_ptr())
        if ctx.needs_input_grad[1]:
            pp = torch.zeros(4, dtype=torch.int32)
            L.call("pa_dwconv_wgrad_parts", L.ptr(shp), L.ptr(pp))
            nparts = int(pp[0])
            taps = wt.shape[0]
            part = torch.empty(nparts, taps * C, dtype=torch.float32, device=x.device)
            L.call("pa_dwconv_wgrad", L.ptr(x), L.ptr(dy), L.ptr(part), L.ptr(shp), L.dcode(x), L.stream_ptr())
            out = torch.empty(taps * C, dtype=x.dtype, device=x.device)
            L.call("pa_reduce_parts", L.ptr(part), L.ptr(None), L.ptr(out), L.ptr(None), nparts, taps * C,
                   L._DT[x.dtype], 0, L.stream_ptr())
            dw = out.view(taps, C).t().reshape(ctx.wshape)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = colsum(dy.view(-1, C))
        return dx, dw, db, None, None, None, None


def depthwise_conv2d_nhwc(x, w, b, stride, pad, dil, fallback, pre_relu=False):
    """NHWC depthwise convolution on the HIP kernels when they measured faster than MIOpen for this shape
    (``fallback(x, w)`` is the MIOpen path); None means: use the fallback. ``pre_relu``: convolve relu(x) (the
    ReLU applied on the kernels' loads and its mask in the data gradient; the fallback gets relu(x))."""
    key = ("dwconv", tuple(x.shape), tuple(w.shape), tuple(stride), tuple(pad), tuple(dil), b is not None,
           x.requires_grad or w.requires_grad, bool(pre_relu))
    if pre_relu:
        plain = fallback
        fallback = lambda xx, ww: plain(torch.relu(xx), ww)  # noqa: E731

    def run(xx, ww):
        return _DWConv.apply(xx, ww, b, tuple(stride), tuple(pad), tuple(dil), bool(pre_relu))

    def bench(fn):
        def go():
            xx = x.detach().requires_grad_(x.requires_grad)
            ww = w.detach().requires_grad_(w.requires_grad)
            with torch.enable_grad():
                y = fn(xx, ww)
                if y.requires_grad:
                    y.backward(torch.ones_like(y))
        return go
    if not G.known(key) and not G._capturing() and L.flag("FLAGS_gemm_backend", "auto") == "auto":
        G.choose(key, {"hip": bench(run), "blas": bench(fallback)})
    if G.choose(key, {"hip": None, "blas": None}) == "hip":
        return run(x, w)
    return None
