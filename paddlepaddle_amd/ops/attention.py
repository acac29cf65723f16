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


class _FlashAttnHIP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        B, Sq, H, D = q.shape
        Sk, Hk = k.shape[1], k.shape[2]
        qc, kc, vc = q.contiguous(), k.contiguous(), v.contiguous()
        o = torch.empty_like(qc)
        lse = torch.empty(B, H, Sq, dtype=torch.float32, device=q.device)
        L.call("pa_flash_attn_fwd", L.ptr(qc), L.ptr(kc), L.ptr(vc), L.ptr(o), L.ptr(lse), B, Sq, Sk, H, Hk, D,
               float(scale), int(causal), L.stream_ptr())
        ctx.save_for_backward(qc, kc, vc, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        qc, kc, vc, o, lse = ctx.saved_tensors
        B, Sq, H, D = qc.shape
        Sk, Hk = kc.shape[1], kc.shape[2]
        doc = do.contiguous().to(qc.dtype)
        dq_acc = torch.zeros(B, Sq, H, D, dtype=torch.float32, device=qc.device)
        dk = torch.empty(B, Sk, H, D, dtype=qc.dtype, device=qc.device) if Hk != H else torch.empty_like(kc)
        dv = torch.empty(B, Sk, H, D, dtype=qc.dtype, device=qc.device) if Hk != H else torch.empty_like(vc)
        delta = torch.empty(B, H, Sq, dtype=torch.float32, device=qc.device)
        dq = torch.empty_like(qc)
        L.call("pa_flash_attn_bwd", L.ptr(qc), L.ptr(kc), L.ptr(vc), L.ptr(o), L.ptr(doc), L.ptr(lse),
               L.ptr(dq), L.ptr(dk), L.ptr(dv), L.ptr(dq_acc), L.ptr(delta), B, Sq, Sk, H, Hk, D,
               float(ctx.scale), int(ctx.causal), L.stream_ptr())
        if Hk != H:
            g = H // Hk
            dk = dk.view(B, Sk, Hk, g, D).sum(3)
            dv = dv.view(B, Sk, Hk, g, D).sum(3)
        return dq, dk, dv, None, None


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


def flash_attention(q, k, v, causal=False, scale=None, mask=None, dropout=0.0, training=True):
    """Attention over [B,S,H,D] tensors; returns [B,Sq,H,D]."""
    D = q.shape[-1]
    scale = 1.0 / math.sqrt(D) if scale is None else float(scale)
    if _hip_ok(q, k, v, mask, dropout, training):
        return _FlashAttnHIP.apply(q, k, v, bool(causal), scale)
    return _sdpa(q, k, v, causal, scale, mask, dropout, training)
