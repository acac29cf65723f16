"""Flash attention forward/backward (HIP, MFMA bf16) in paddle's [batch, seq, heads, head_dim] layout.

Reference: paddle/phi/kernels/gpu/flash_attn_kernel.cu, flash_attn_grad_kernel.cu,
python/paddle/nn/functional/flash_attention.py:364 (flash_attention), :1145 (sdpa).
Kernel: csrc/kernels/flash_attn.hip — per workgroup a 64-row (or 128-row) Q block, K/V tiles
streamed through LDS, S = QKᵀ and O += PV on v_mfma_f32_16x16x32_bf16, online softmax with the
running max/sum in registers, LSE written for the backward. GQA via kv-head = head / (H/Hk).
Backward recomputes P from Q, K and LSE (no S×S materialisation): dV, dK accumulated per key block,
dQ accumulated in fp32.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import _loader as L
from ..framework.trace_hook import static_op


def attention_reference(q, k, v, causal=False, scale=None, mask=None, dropout=0.0, training=False):
    """Plain math reference in fp32; q,k,v [B,S,H,D]."""
    B, Sq, H, D = q.shape
    Hk = k.shape[2]
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    qf, kf, vf = q.float().transpose(1, 2), k.float().transpose(1, 2), v.float().transpose(1, 2)
    if Hk != H:
        kf = kf.repeat_interleave(H // Hk, 1)
        vf = vf.repeat_interleave(H // Hk, 1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    Sk = k.shape[1]
    if causal:
        cm = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).tril(Sk - Sq)
        s = s.masked_fill(~cm, float("-inf"))
    if mask is not None:
        m = mask
        if m.dtype == torch.bool:
            s = s.masked_fill(~m, float("-inf"))
        else:
            s = s + m.float()
    p = torch.softmax(s, -1)
    if dropout > 0 and training:
        p = F.dropout(p, dropout)
    o = torch.matmul(p, vf)
    return o.transpose(1, 2).to(q.dtype)


def _sdpa(q, k, v, causal, scale, mask, dropout, training):
    """ATen SDPA path (used on CPU and for shapes the HIP kernel does not cover)."""
    qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
    H, Hk = q.shape[2], k.shape[2]
    if Hk != H:
        kt = kt.repeat_interleave(H // Hk, 1)
        vt = vt.repeat_interleave(H // Hk, 1)
    am = mask
    if causal and q.shape[1] != k.shape[1]:
        Sq, Sk = q.shape[1], k.shape[1]
        am = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).tril(Sk - Sq)
        causal = False
    o = F.scaled_dot_product_attention(qt, kt, vt, attn_mask=am, dropout_p=dropout if training else 0.0,
                                       is_causal=causal and am is None, scale=scale)
    return o.transpose(1, 2)


def _strides(t):
    st = t.stride()
    return [st[0], st[1], st[2]]


def _i64arr(vals):
    import ctypes
    return (ctypes.c_int64 * len(vals))(*[int(v) for v in vals])


def _fa_fwd(q, k, v, causal, scale):
    B, Sq, H, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    o = torch.empty(B, Sq, H, D, dtype=q.dtype, device=q.device)
    lse = torch.empty(B, H, Sq, dtype=torch.float32, device=q.device)
    st = _i64arr(_strides(q) + _strides(k) + _strides(v) + _strides(o))
    L.call("pa_flash_attn_fwd", L.ptr(q), L.ptr(k), L.ptr(v), L.ptr(o), L.ptr(lse), st, B, Sq, Sk, H, Hk, D,
           float(scale), int(causal), L.stream_ptr())
    return o, lse


def _fa_bwd(q, k, v, o, lse, do, dq, dk, dv, causal, scale):
    B, Sq, H, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    dq_acc = torch.empty(B, Sq, H, D, dtype=torch.float32, device=q.device)
    delta = torch.empty(B, H, Sq, dtype=torch.float32, device=q.device)
    st = _i64arr(_strides(q) + _strides(k) + _strides(v) + _strides(o) + _strides(do) + _strides(dq)
                 + _strides(dk) + _strides(dv))
    L.call("pa_flash_attn_bwd", L.ptr(q), L.ptr(k), L.ptr(v), L.ptr(o), L.ptr(do), L.ptr(lse), L.ptr(dq),
           L.ptr(dk), L.ptr(dv), L.ptr(dq_acc), L.ptr(delta), st, B, Sq, Sk, H, Hk, D, float(scale), int(causal),
           L.stream_ptr())


def _lastdim_contig(t):
    return t.stride(-1) == 1 and t.data_ptr() % 16 == 0 and all(s % 8 == 0 for s in t.stride()[:-1])


class _FlashAttnHIP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        q, k, v = [t if _lastdim_contig(t) else t.contiguous() for t in (q, k, v)]
        o, lse = _fa_fwd(q, k, v, causal, scale)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        B, Sq, H, D = q.shape
        Sk, Hk = k.shape[1], k.shape[2]
        do = do.to(q.dtype)
        if not _lastdim_contig(do):
            do = do.contiguous()
        dq = torch.empty(B, Sq, H, D, dtype=q.dtype, device=q.device)
        dk = torch.empty(B, Sk, H, D, dtype=q.dtype, device=q.device)
        dv = torch.empty(B, Sk, H, D, dtype=q.dtype, device=q.device)
        _fa_bwd(q, k, v, o, lse, do, dq, dk, dv, ctx.causal, ctx.scale)
        if Hk != H:
            g = H // Hk
            dk = dk.view(B, Sk, Hk, g, D).sum(3)
            dv = dv.view(B, Sk, Hk, g, D).sum(3)
        return dq, dk, dv, None, None


class _FlashAttnQKVPackedHIP(torch.autograd.Function):
    """qkv [B, S, H, 3, D] (PaddleNLP fused-QKV layout) -> o [B, S, H, D]; grad is one dqkv buffer."""

    @staticmethod
    def forward(ctx, qkv, causal, scale):
        q, k, v = qkv[:, :, :, 0], qkv[:, :, :, 1], qkv[:, :, :, 2]
        o, lse = _fa_fwd(q, k, v, causal, scale)
        ctx.save_for_backward(qkv, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        do = do.to(qkv.dtype)
        if not _lastdim_contig(do):
            do = do.contiguous()
        dqkv = torch.empty_like(qkv)
        q, k, v = qkv[:, :, :, 0], qkv[:, :, :, 1], qkv[:, :, :, 2]
        _fa_bwd(q, k, v, o, lse, do, dqkv[:, :, :, 0], dqkv[:, :, :, 1], dqkv[:, :, :, 2], ctx.causal, ctx.scale)
        return dqkv, None, None


@static_op
def flash_attention_qkvpacked(qkv, causal=True, scale=None, dropout=0.0, training=True):
    """qkv [B,S,H,3,D] -> [B,S,H,D]."""
    D = qkv.shape[-1]
    scale = 1.0 / math.sqrt(D) if scale is None else float(scale)
    q, k, v = qkv[:, :, :, 0], qkv[:, :, :, 1], qkv[:, :, :, 2]
    if _hip_ok(q, k, v, None, dropout, training) and _lastdim_contig(qkv):
        return _FlashAttnQKVPackedHIP.apply(qkv, bool(causal), scale)
    return flash_attention(q, k, v, causal=causal, scale=scale, dropout=dropout, training=training)


def _hip_ok(q, k, v, mask, dropout, training):
    if not L.hip_enabled_for(q) or not L.has("pa_flash_attn_fwd"):
        return False
    if mask is not None or (dropout > 0 and training):
        return False
    if q.dtype not in (torch.bfloat16, torch.float16) or k.dtype != q.dtype or v.dtype != q.dtype:
        return False
    D = q.shape[-1]
    if D not in (64, 128) or k.shape[-1] != D:
        return False
    if q.shape[2] % k.shape[2] != 0:
        return False
    return True


@static_op
def flash_attention(q, k, v, causal=False, scale=None, mask=None, dropout=0.0, training=True):
    """Attention over [B,S,H,D] tensors; returns [B,Sq,H,D]."""
    D = q.shape[-1]
    scale = 1.0 / math.sqrt(D) if scale is None else float(scale)
    if _hip_ok(q, k, v, mask, dropout, training):
        return _FlashAttnHIP.apply(q, k, v, bool(causal), scale)
    return _sdpa(q, k, v, causal, scale, mask, dropout, training)
