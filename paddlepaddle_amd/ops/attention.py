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


def paged_decode_reference(q, key_cache, value_cache, block_tables, lens, scale=None):
    """fp32 reference: q [N,H,D]; caches [num_blocks,Hkv,bs,D]; block_tables [N,max_blocks]; lens [N]
    (cached tokens per sequence, the current one included). Returns [N,H,D] in q's dtype."""
    N, H, D = q.shape
    _, Hkv, bs, _ = key_cache.shape
    scale = 1.0 / math.sqrt(D) if scale is None else float(scale)
    nblk = block_tables.shape[1]
    tab = block_tables.long()
    K = key_cache[tab].permute(0, 2, 1, 3, 4).reshape(N, Hkv, nblk * bs, D).float()
    V = value_cache[tab].permute(0, 2, 1, 3, 4).reshape(N, Hkv, nblk * bs, D).float()
    G = H // Hkv
    qf = q.float().view(N, Hkv, G, D)
    s = torch.einsum("nkgd,nkld->nkgl", qf, K) * scale
    valid = torch.arange(nblk * bs, device=q.device)[None] < lens.long()[:, None]
    s = s.masked_fill(~valid[:, None, None], float("-inf"))
    o = torch.einsum("nkgl,nkld->nkgd", torch.softmax(s, -1), V)
    return o.reshape(N, H, D).to(q.dtype)


def _decode_splits(N, Hkv, max_len, bs):
    """Flash-decoding split count: enough workgroups to fill 256 CUs (≈4 per CU), but every split
    keeps ≥ 4 cache blocks so each of the workgroup's 4 waves has a block to stream."""
    nblk = max(1, (max_len + bs - 1) // bs)
    want = max(1, -(-1024 // max(1, N * Hkv)))
    return int(max(1, min(want, nblk // 4, 64)))


def _decode_hip_ok(q, key_cache, value_cache, Hkv):
    N, H, D = q.shape
    return (L.hip_enabled_for(q) and L.has("pa_paged_decode_attn") and q.dtype == torch.bfloat16
            and key_cache.dtype == torch.bfloat16 and value_cache.dtype == torch.bfloat16 and D == 128
            and H % Hkv == 0 and H // Hkv in (1, 2, 4, 8) and key_cache.is_contiguous()
            and value_cache.is_contiguous())


def _decode_launch(q, kc, vc, tables, lens, Hkv, bs, blk_stride, head_stride, scale, max_len):
    N, H, D = q.shape
    q = q.contiguous()
    tables = tables.to(torch.int32).contiguous()
    lens32 = lens.to(torch.int32).contiguous()
    max_blocks = tables.shape[1]
    splits = _decode_splits(N, Hkv, max_len, bs)
    part_o = torch.empty(N * H * splits * D, dtype=torch.float32, device=q.device)
    part_ml = torch.empty(N * H * splits * 2, dtype=torch.float32, device=q.device)
    out = torch.empty_like(q)
    L.call("pa_paged_decode_attn", L.ptr(q), L.ptr(kc), L.ptr(vc), L.ptr(tables), L.ptr(lens32), L.ptr(part_o),
           L.ptr(part_ml), L.ptr(out), N, H, Hkv, D, bs, max_blocks, splits, int(blk_stride), int(head_stride),
           float(scale), L.stream_ptr())
    return out


@static_op
def paged_decode_attention(q, key_cache, value_cache, block_tables, lens, scale=None, max_len=None):
    """One-token-per-sequence attention over a paged KV cache (block_multihead_attention decode).
    q [N,H,D]; caches [num_blocks,Hkv,block_size,D]; block_tables [N,max_blocks]; lens [N] cached
    tokens incl. the current one. HIP flash-decoding kernel (csrc/kernels/decode_attn.hip) for bf16,
    head_dim 128; otherwise the fp32 reference. ``max_len`` bounds lens (host hint for the split count;
    defaults to the block-table capacity, so no device sync)."""
    N, H, D = q.shape
    _, Hkv, bs, _ = key_cache.shape
    scale = 1.0 / math.sqrt(D) if scale is None else float(scale)
    if not _decode_hip_ok(q, key_cache, value_cache, Hkv):
        return paged_decode_reference(q, key_cache, value_cache, block_tables, lens, scale)
    ml = block_tables.shape[1] * bs if max_len is None else int(max_len)
    return _decode_launch(q, key_cache, value_cache, block_tables, lens, Hkv, bs, Hkv * bs * D, bs * D, scale, ml)


_VBLK = 64  # virtual block size when a dense cache is streamed by the paged kernel


_DENSE_TABLES = {}


@static_op
def dense_decode_attention(q, key_cache, value_cache, lens, scale=None, max_len=None):
    """Decode attention over a dense per-sequence cache [B,Hkv,max_len,D] (masked_multihead_attention
    layout). The same HIP kernel streams it as virtual 64-token blocks: block j of sequence b starts at
    b*Hkv*max_len*D + j*64*D and heads are max_len*D apart, so the block table is just b*Hkv*nb + j."""
    N, H, D = q.shape
    B, Hkv, Lc, _ = key_cache.shape
    scale = 1.0 / math.sqrt(D) if scale is None else float(scale)
    if not _decode_hip_ok(q, key_cache, value_cache, Hkv) or Lc % _VBLK != 0:
        valid = torch.arange(Lc, device=q.device)[None] < lens.long()[:, None]
        G = H // Hkv
        s = torch.einsum("nkgd,nkld->nkgl", q.float().view(N, Hkv, G, D), key_cache.float()) * scale
        s = s.masked_fill(~valid[:, None, None], float("-inf"))
        o = torch.einsum("nkgl,nkld->nkgd", torch.softmax(s, -1), value_cache.float())
        return o.reshape(N, H, D).to(q.dtype)
    nb = Lc // _VBLK
    key = (N, Hkv, nb, q.device)
    tables = _DENSE_TABLES.get(key)
    if tables is None:  # identical for every layer / step: built once (also outside any captured graph)
        tables = (torch.arange(N, device=q.device, dtype=torch.int32)[:, None] * (Hkv * nb)
                  + torch.arange(nb, device=q.device, dtype=torch.int32)[None])
        if len(_DENSE_TABLES) > 64:
            _DENSE_TABLES.clear()
        _DENSE_TABLES[key] = tables
    ml = Lc if max_len is None else int(max_len)
    return _decode_launch(q, key_cache, value_cache, tables, lens, Hkv, _VBLK, _VBLK * D, Lc * D, scale, ml)
