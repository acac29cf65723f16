"""Flash attention API. Reference: python/paddle/nn/functional/flash_attention.py
(flash_attention :364, flash_attn_qkvpacked :609, flash_attn_unpadded :762, flash_attn_varlen_qkvpacked :961,
scaled_dot_product_attention :1145, flashmask_attention :1306).
Layout: [batch, seq_len, num_heads, head_dim]; varlen: packed [total_tokens, num_heads, head_dim] with
cu_seqlens. Every variant (masks, flashmask row bounds, dropout, varlen, GQA, head dims up to 256) runs on the
HIP kernel (csrc/kernels/flash_attn_kernels.h) through ops.attention.attention."""
from __future__ import annotations

import math

import torch

from ...amp.state import maybe_cast
from ...framework.tensor import _wrap
from ...tensor._helpers import T
from ...ops import attention as _A


def _seed_of(fixed_seed_offset):
    if fixed_seed_offset is None:
        return None
    v = T(fixed_seed_offset).reshape(-1).tolist()
    return (int(v[0]) & ((1 << 32) - 1)) | ((int(v[1]) & ((1 << 30) - 1)) << 32) if len(v) > 1 else int(v[0])


def _softmax_of(q, k, causal, scale, mask=None):
    """The attention probabilities [B, H, Sq, Sk] (return_softmax: a debugging output, computed densely)."""
    lse = _A._lse_reference(q, k, causal, scale, mask)
    H, Hk = q.shape[2], k.shape[2]
    qf, kf = q.float().transpose(1, 2), k.float().transpose(1, 2)
    if Hk != H:
        kf = kf.repeat_interleave(H // Hk, 1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    Sq, Sk = q.shape[1], k.shape[1]
    if causal:
        s = s.masked_fill(~torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).tril(Sk - Sq), float("-inf"))
    if mask is not None:
        s = s.masked_fill(~mask, float("-inf")) if mask.dtype == torch.bool else s + mask.float()
    return torch.exp(s - lse.unsqueeze(-1)).to(q.dtype)


def flash_attention(query, key, value, dropout=0.0, causal=False, return_softmax=False, *, fixed_seed_offset=None,
                    rng_name="", training=True, name=None, softmax_scale=None):
    q, k, v = maybe_cast("flash_attention", T(query), T(key), T(value))
    scale = 1.0 / math.sqrt(q.shape[-1]) if softmax_scale is None else float(softmax_scale)
    o = _A.attention(q, k, v, causal=causal, scale=scale, dropout=dropout, training=training,
                     seed=_seed_of(fixed_seed_offset))
    return _wrap(o), (_wrap(_softmax_of(q, k, causal, scale)) if return_softmax else None)


def scaled_dot_product_attention(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False,
                                 training=True, name=None, scale=None):
    """``attn_mask``: bool (True = attend) or additive (added to scale * QK^T), broadcastable to
    [batch, heads, seq_q, seq_k]; evaluated inside the HIP kernel (no dense score matrix)."""
    q, k, v = maybe_cast("scaled_dot_product_attention", T(query), T(key), T(value))
    o = _A.attention(q, k, v, causal=is_causal, scale=scale, mask=T(attn_mask), dropout=dropout_p, training=training)
    return _wrap(o)


def flash_attn_unpadded(query, key, value, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, scale,
                        dropout=0.0, causal=False, return_softmax=False, fixed_seed_offset=None, rng_name="",
                        training=True, name=None):
    """Variable-length attention over packed [total_tokens, heads, dim]: one launch; each workgroup reads its
    sequence's bounds from the device-side cu_seqlens (no host sync, graph-capturable)."""
    q, k, v = maybe_cast("flash_attn_unpadded", T(query), T(key), T(value))
    o = _A.attention(q, k, v, causal=causal, scale=scale, dropout=dropout, training=training,
                     seed=_seed_of(fixed_seed_offset), cu_seqlens_q=T(cu_seqlens_q), cu_seqlens_k=T(cu_seqlens_k),
                     max_seqlen_q=int(max_seqlen_q), max_seqlen_k=int(max_seqlen_k))
    return _wrap(o), None


def _split_packed(t):
    """qkv [..., G + 2, Hk, D] -> q [..., Hk * G, D] (query head h = kv_head * G + g, the grouping the GQA kernel
    maps back with h // G), k, v [..., Hk, D]."""
    g = t.shape[-3] - 2
    lead = t.shape[:-3]
    q = t[..., :g, :, :].transpose(-3, -2).reshape(*lead, g * t.shape[-2], t.shape[-1])
    return q, t[..., g, :, :], t[..., g + 1, :, :]


def flash_attn_qkvpacked(qkv, dropout=0.0, causal=False, return_softmax=False, *, fixed_seed_offset=None,
                         rng_name="", training=True, name=None):
    """qkv [B, S, H/Hk + 2, Hk, D] -> out [B, S, H, D]."""
    t = T(qkv)
    q, k, v = _split_packed(t)
    o = _A.attention(q, k, v, causal=causal, dropout=dropout, training=training, seed=_seed_of(fixed_seed_offset))
    return _wrap(o), None


def flash_attn_varlen_qkvpacked(qkv, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, scale, dropout=0.0,
                                causal=False, return_softmax=False, fixed_seed_offset=None, rng_name="",
                                varlen_padded=True, training=True, name=None):
    """Packed varlen attention: qkv [total, H/Hk + 2, Hk, D]."""
    q, k, v = _split_packed(T(qkv))
    o = _A.attention(q, k, v, causal=causal, scale=scale, dropout=dropout, training=training,
                     seed=_seed_of(fixed_seed_offset), cu_seqlens_q=T(cu_seqlens_q), cu_seqlens_k=T(cu_seqlens_k),
                     max_seqlen_q=int(max_seqlen_q), max_seqlen_k=int(max_seqlen_k))
    return _wrap(o), None


def flashmask_attention(query, key, value, startend_row_indices=None, *, dropout=0.0, causal=False,
                        window_size=None, return_softmax_lse=False, return_seed_offset=False,
                        fixed_seed_offset=None, rng_name="", training=True, name=None):
    """FlashMask: for every key column, the row intervals in ``startend_row_indices`` [B, H|1, Sk, 1|2|4] are
    masked (LTS | LTS, LTE (causal) or LTS, UTE | LTS, LTE, UTS, UTE); evaluated in the kernel from the O(Sk)
    bounds. ``window_size`` (left, right) is turned into bounds the same way."""
    q, k, v = maybe_cast("flashmask_attention", T(query), T(key), T(value))
    Sq, Sk = q.shape[1], k.shape[1]
    se = T(startend_row_indices)
    if window_size is not None:
        wl, wr = (window_size, window_size) if isinstance(window_size, int) else window_size
        j = torch.arange(Sk, device=q.device, dtype=torch.int32)
        shift = Sk - Sq
        lts = (j - shift + wl + 1).clamp(0, Sq).view(1, 1, Sk, 1)          # rows > key + wl (below the band)
        if causal:
            se = lts
        else:
            ute = (j - shift - wr).clamp(0, Sq).view(1, 1, Sk, 1)         # rows < key - wr (above the band)
            se = torch.cat([lts, ute], -1)
        if startend_row_indices is not None:
            raise ValueError("window_size and startend_row_indices are exclusive")
    if se is None:
        o, lse = _A.attention(q, k, v, causal=causal, dropout=dropout, training=training, return_lse=True,
                              seed=_seed_of(fixed_seed_offset))
    else:
        o, lse = _A.attention(q, k, v, causal=causal, startend_row_indices=se, dropout=dropout, training=training,
                              return_lse=True, seed=_seed_of(fixed_seed_offset))
    out = [_wrap(o)]
    if return_softmax_lse:
        out.append(_wrap(lse))
    if return_seed_offset:
        out.append(_wrap(torch.zeros(2, dtype=torch.int64)))
    return out[0] if len(out) == 1 else tuple(out)


def flash_attention_with_sparse_mask(query, key, value, attn_mask_start_row_indices, attn_mask_start_row=0,
                                     dropout_p=0.0, is_causal=False, return_softmax=False, return_softmax_lse=False,
                                     return_seed_offset=False, training=True, name=None):
    """Start-row mask [B, H, Sk]: key j is visible to rows < start[j] (the LTS column of flashmask)."""
    q, k, v = maybe_cast("flash_attention_with_sparse_mask", T(query), T(key), T(value))
    idx = T(attn_mask_start_row_indices).to(torch.int32)
    se = idx.unsqueeze(-1)
    o = _A.attention(q, k, v, causal=is_causal, startend_row_indices=se, dropout=dropout_p, training=training)
    return _wrap(o)


def calc_reduced_attention_scores(query, key, softmax_lse, name=None):
    """sum over the query rows of softmax(Q K^T / sqrt(d)) -> [B, H, 1, Sk] fp32 (inference: no gradient), with the
    softmax normaliser taken from the forward's ``softmax_lse`` [B, H, >= Sq] (Reference:
    python/paddle/nn/functional/flash_attention.py:2040). The probabilities are rebuilt block by block — 512 query
    rows at a time through one batched bf16 GEMM with fp32 output — and summed in place, so no [Sq, Sk] matrix is
    ever resident."""
    q, k, lse = T(query), T(key), T(softmax_lse)
    if getattr(query, "stop_gradient", True) is False or getattr(key, "stop_gradient", True) is False:
        raise ValueError("calc_reduced_attention_scores() is for inference only (stop_gradient inputs)")
    B, Sq, H, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    scale = 1.0 / math.sqrt(D)
    kt = k.transpose(1, 2)                                   # [B, Hk, Sk, D]
    if Hk != H:
        kt = kt.repeat_interleave(H // Hk, 1)
    out = torch.zeros(B, H, 1, Sk, dtype=torch.float32, device=q.device)
    lse = lse.float()
    with torch.no_grad():
        for r0 in range(0, Sq, 512):
            r1 = min(Sq, r0 + 512)
            qb = q[:, r0:r1].transpose(1, 2)                 # [B, H, rb, D]
            s = torch.matmul(qb, kt.transpose(-1, -2)).float() * scale
            s.sub_(lse[:, :, r0:r1].unsqueeze(-1)).exp_()
            out.add_(s.sum(2, keepdim=True))
    return _wrap(out)
