"""GELU / SiLU / SwiGLU / softmax with HIP kernels.

Reference: paddle/phi/kernels/gpu/{gelu,softmax}_kernel.cu, incubate swiglu,
fusion/gpu/fused_bias_act_kernel.cu. Kernels: csrc/kernels/act.hip, csrc/kernels/softmax.hip.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _loader as L
from ..framework.trace_hook import static_op


class _GeluHIP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, approximate):
        xc = x.contiguous()
        y = torch.empty_like(xc)
        L.call("pa_gelu_fwd", L.ptr(xc), L.ptr(y), xc.numel(), int(approximate), L.dcode(xc), L.stream_ptr())
        ctx.save_for_backward(xc)
        ctx.approximate = approximate
        return y

    @staticmethod
    def backward(ctx, dy):
        (xc,) = ctx.saved_tensors
        dyc = dy.contiguous().to(xc.dtype)
        dx = torch.empty_like(xc)
        L.call("pa_gelu_bwd", L.ptr(xc), L.ptr(dyc), L.ptr(dx), xc.numel(), int(ctx.approximate), L.dcode(xc),
               L.stream_ptr())
        return dx, None


@static_op
def gelu(x, approximate=False):
    if L.hip_enabled_for(x) and x.dtype in L._DT and x.numel() % 8 == 0:
        return _GeluHIP.apply(x, bool(approximate))
    return F.gelu(x, approximate="tanh" if approximate else "none")


class _BiasGeluHIP(torch.autograd.Function):
    """y = gelu(x + bias) over [rows, cols]; saves x+bias pre-activation recomputed in bwd."""

    @staticmethod
    def forward(ctx, x, bias):
        cols = x.shape[-1]
        xc = x.contiguous().view(-1, cols)
        bc = bias.contiguous().to(x.dtype)
        y = torch.empty_like(xc)
        L.call("pa_bias_gelu_fwd", L.ptr(xc), L.ptr(bc), L.ptr(y), xc.shape[0], cols, L.dcode(xc), L.stream_ptr())
        ctx.save_for_backward(xc, bc)
        ctx.shape = x.shape
        ctx.b_dtype = bias.dtype
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        xc, bc = ctx.saved_tensors
        h = xc + bc
        dyc = dy.contiguous().view_as(xc).to(xc.dtype)
        dh = torch.empty_like(h)
        L.call("pa_gelu_bwd", L.ptr(h), L.ptr(dyc), L.ptr(dh), h.numel(), 1, L.dcode(h), L.stream_ptr())
        db = dh.float().sum(0).to(ctx.b_dtype)
        return dh.view(ctx.shape), db


@static_op
def bias_gelu(x, bias):
    """gelu_tanh(x + bias) (GPT MLP epilogue)."""
    if L.hip_enabled_for(x) and x.dtype in L._DT and x.shape[-1] % 8 == 0:
        return _BiasGeluHIP.apply(x, bias)
    return F.gelu(x + bias, approximate="tanh")


@static_op
def silu(x):
    return F.silu(x)


class _SwigluHIP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        cols = a.shape[-1]
        shape = a.shape
        a2 = a.reshape(-1, cols)
        b2 = b.reshape(-1, cols)
        # allow a/b to be halves of one [rows, 2*cols] buffer (chunk views) — same row stride
        if a2.stride(1) != 1 or b2.stride(1) != 1 or a2.stride(0) != b2.stride(0):
            a2, b2 = a2.contiguous(), b2.contiguous()
        stride = a2.stride(0)
        rows = a2.shape[0]
        y = torch.empty(rows, cols, dtype=a.dtype, device=a.device)
        L.call("pa_swiglu_fwd", L.ptr(a2), L.ptr(b2), L.ptr(y), rows, cols, stride, L.dcode(a2), L.stream_ptr())
        ctx.save_for_backward(a2, b2)
        ctx.shape = shape
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        a2, b2 = ctx.saved_tensors
        rows, cols = a2.shape[0], a2.shape[1]
        dyc = dy.contiguous().view(rows, cols).to(a2.dtype)
        dab = torch.empty(rows, 2 * cols, dtype=a2.dtype, device=a2.device)
        da, db = dab[:, :cols], dab[:, cols:]
        L.call("pa_swiglu_bwd", L.ptr(a2), L.ptr(b2), L.ptr(dyc), L.ptr(da), L.ptr(db), rows, cols,
               a2.stride(0) | (dab.stride(0) << 32), L.dcode(a2), L.stream_ptr())
        return da.reshape(ctx.shape), db.reshape(ctx.shape)


class _SwigluPackedHIP(torch.autograd.Function):
    """x [.., 2f] = [gate | up] (one projection's output) -> silu(gate) * up [.., f]. The gradient is one [.., 2f]
    buffer written by the backward kernel: the gate/up halves never go through a chunk + cat in autograd."""

    @staticmethod
    def forward(ctx, x):
        f = x.shape[-1] // 2
        x2 = x.reshape(-1, 2 * f)
        if x2.stride(1) != 1 or x2.stride(0) % 8 or x2.data_ptr() % 16:
            x2 = x2.contiguous()
        rows = x2.shape[0]
        y = torch.empty(rows, f, dtype=x.dtype, device=x.device)
        a2, b2 = x2[:, :f], x2[:, f:]
        L.call("pa_swiglu_fwd", L.ptr(a2), L.ptr(b2), L.ptr(y), rows, f, x2.stride(0), L.dcode(x2), L.stream_ptr())
        ctx.save_for_backward(x2)
        ctx.shape = x.shape
        return y.view(*x.shape[:-1], f)

    @staticmethod
    def backward(ctx, dy):
        (x2,) = ctx.saved_tensors
        rows, f = x2.shape[0], x2.shape[1] // 2
        dyc = dy.contiguous().view(rows, f).to(x2.dtype)
        dx = torch.empty(rows, 2 * f, dtype=x2.dtype, device=x2.device)
        L.call("pa_swiglu_bwd", L.ptr(x2[:, :f]), L.ptr(x2[:, f:]), L.ptr(dyc), L.ptr(dx[:, :f]), L.ptr(dx[:, f:]),
               rows, f, x2.stride(0) | (dx.stride(0) << 32), L.dcode(x2), L.stream_ptr())
        return dx.view(ctx.shape)


@static_op
def swiglu(a, b=None):
    """silu(a) * b; with ``b`` None, ``a`` is [.., 2f] = [gate | up] (Reference:
    python/paddle/incubate/nn/functional/swiglu.py:22 — one-input form splits the last dim)."""
    if b is None:
        if L.hip_enabled_for(a) and a.dtype in L._DT and a.shape[-1] % 16 == 0:
            return _SwigluPackedHIP.apply(a)
        g, u = a.chunk(2, -1)
        return F.silu(g) * u
    if L.hip_enabled_for(a) and a.dtype in L._DT and a.shape[-1] % 8 == 0 and a.shape == b.shape:
        return _SwigluHIP.apply(a, b)
    return F.silu(a) * b


class _SoftmaxHIP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        cols = x.shape[-1]
        x2 = x.contiguous().view(-1, cols)
        y = torch.empty_like(x2)
        L.call("pa_softmax_fwd", L.ptr(x2), L.ptr(y), x2.shape[0], cols, L.dcode(x2), L.stream_ptr())
        ctx.save_for_backward(y)
        ctx.shape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy2 = dy.contiguous().view_as(y).to(y.dtype)
        dx = torch.empty_like(y)
        L.call("pa_softmax_bwd", L.ptr(y), L.ptr(dy2), L.ptr(dx), y.shape[0], y.shape[1], L.dcode(y),
               L.stream_ptr())
        return dx.view(ctx.shape)


@static_op
def softmax(x, axis=-1):
    nd = x.dim()
    if nd == 0:
        return torch.ones_like(x)
    ax = axis % nd
    if ax == nd - 1 and L.hip_enabled_for(x) and x.dtype in L._DT and x.shape[-1] % 8 == 0 \
            and x.shape[-1] <= 65536:
        return _SoftmaxHIP.apply(x)
    if x.dtype in (torch.float16, torch.bfloat16):
        return F.softmax(x.float(), ax).to(x.dtype)
    return F.softmax(x, ax)
