"""MoE building blocks on the device: token routing and the grouped (all-experts) linear layer.

Reference: paddle/phi/kernels/fusion/cutlass/fused_moe_kernel.cu, python/paddle/incubate/nn/functional/
fused_moe.py:20, python/paddle/incubate/distributed/models/moe/moe_layer.py.

``route(eid, E)`` turns the expert id of every (token, slot) entry into per-expert offsets and a stable
permutation (csrc/kernels/grouped_gemm.hip pa_moe_route — two small kernels, no host sync).
``grouped_linear(x, w, offs, bias)`` computes y[rows of e] = x[rows of e] . w[e] (+ bias[e]) for every expert
in one launch and has a backward made of the same grouped kernel (dX = dY . W_e^T, dW_e = X_e^T . dY_e);
bias gradients are per-expert segment sums. Everything is shape-static, so the MoE layer can be captured
in a hipGraph. On CPU (and for non-bf16 inputs) the same math runs per expert with torch.
"""
from __future__ import annotations

import torch

from . import _loader as L

_ZERO = {}


def _zero_page(dev):
    z = _ZERO.get(dev)
    if z is None:
        z = _ZERO[dev] = torch.zeros(64, dtype=torch.uint8, device=dev)
    return z


def _hip(t):
    return L.hip_enabled_for(t) and L.has("pa_grouped_gemm")


def route(eid, num_experts):
    """eid [n] int (negative = dropped entry) -> (offs [E + 1] int32, perm [n] int64 whose first offs[E]
    entries list the kept entries grouped by expert, in entry order)."""
    eid = eid.reshape(-1)
    n = eid.numel()
    dev = eid.device
    if L.hip_enabled_for(eid) and L.has("pa_moe_route") and n > 0:
        e32 = eid.to(torch.int32).contiguous()
        counts = torch.empty(num_experts, dtype=torch.int32, device=dev)
        offs = torch.empty(num_experts + 1, dtype=torch.int32, device=dev)
        perm = torch.zeros(n, dtype=torch.int32, device=dev)
        L.call("pa_moe_route", L.ptr(e32), n, num_experts, L.ptr(counts), L.ptr(offs), L.ptr(perm), L.stream_ptr())
        return offs, perm.long()
    key = torch.where(eid < 0, torch.full_like(eid, num_experts), eid)
    perm = torch.argsort(key, stable=True)
    counts = torch.bincount(key, minlength=num_experts + 1)[:num_experts]
    offs = torch.zeros(num_experts + 1, dtype=torch.int32, device=dev)
    offs[1:] = torch.cumsum(counts, 0).to(torch.int32)
    return offs, perm


def expert_of_rows(offs, rows):
    """Expert index of every sorted row (rows past offs[-1] get E)."""
    r = torch.arange(rows, device=offs.device, dtype=torch.int32)
    return torch.searchsorted(offs[1:].contiguous(), r, right=True)


def _gg(mode, a, b, c, bias, offs, E, rows, M, N, K, lda, ldb, ldc, flags):
    L.call("pa_grouped_gemm", mode, L.ptr(a), L.ptr(b), L.ptr(c), L.ptr(bias), L.ptr(offs),
           L.ptr(_zero_page(a.device)), E, rows, M, N, K, lda, ldb, ldc, flags, L.stream_ptr())


def _fallback(x, w, offs, bias):
    out = x.new_zeros(x.shape[0], w.shape[2])
    o = offs.tolist()
    for e in range(w.shape[0]):
        s, t = o[e], o[e + 1]
        if t > s:
            y = x[s:t] @ w[e]
            if bias is not None:
                y = y + bias[e]
            out[s:t] = y
    return out


class _GroupedLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, offs, bias):
        T, K = x.shape
        E, _, N = w.shape
        x, w = x.contiguous(), w.contiguous()
        b = bias.contiguous() if bias is not None else None
        y = torch.zeros(T, N, dtype=x.dtype, device=x.device)
        rows_alive = T  # rows past offs[E] are never written: zero them for a defined output
        _gg(0, x, w, y, b, offs, E, rows_alive, 0, N, K, K, N, N, 1 if b is not None else 0)
        ctx.save_for_backward(x, w, offs)
        ctx.has_bias = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, offs = ctx.saved_tensors
        T, K = x.shape
        E, _, N = w.shape
        dy = dy.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.zeros_like(x)
            _gg(1, dy, w, dx, None, offs, E, T, 0, K, N, N, N, K, 0)
        if ctx.needs_input_grad[1]:
            dw = torch.empty_like(w)
            _gg(2, x, dy, dw, None, offs, E, T, K, N, 0, K, N, N, 0)
        if ctx.has_bias and ctx.needs_input_grad[3]:
            eo = expert_of_rows(offs, T).long()
            db = torch.zeros(E + 1, N, dtype=torch.float32, device=dy.device)
            db.index_add_(0, eo, dy.float())
            db = db[:E].to(dy.dtype)
        return dx, dw, None, db


def grouped_linear(x, w, offs, bias=None):
    """x [T, K] rows sorted by expert (rows offs[e]:offs[e+1] -> expert e; rows past offs[E] give 0),
    w [E, K, N], bias [E, N] -> y [T, N]."""
    ok = (_hip(x) and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.shape[1] % 64 == 0
          and w.shape[2] % 64 == 0 and (bias is None or bias.dtype == torch.bfloat16))
    if not ok:
        return _fallback(x, w, offs, bias)
    y = _GroupedLinear.apply(x, w, offs.to(torch.int32).contiguous(), bias)
    return y
