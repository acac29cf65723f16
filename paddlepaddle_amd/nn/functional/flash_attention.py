"""Flash attention API. Reference: python/paddle/nn/functional/flash_attention.py
(flash_attention :364, flash_attn_unpadded :762, scaled_dot_product_attention :1145).
Layout: [batch, seq_len, num_heads, head_dim]. HIP kernel: csrc/kernels/flash_attn.hip."""
from __future__ import annotations

import torch

from ...amp.state import maybe_cast
from ...framework.tensor import _wrap
from ...tensor._helpers import T
from ... import ops as _ops


def flash_attention(query, key, value, dropout=0.0, causal=False, return_softmax=False, *, fixed_seed_offset=None,
                    rng_name="", training=True, name=None, softmax_scale=None):
    q, k, v = maybe_cast("flash_attention", T(query), T(key), T(value))
    o = _ops.flash_attention(q, k, v, causal=causal, scale=softmax_scale, dropout=dropout, training=training)
    return _wrap(o), None


def scaled_dot_product_attention(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False,
                                 training=True, name=None, scale=None):
    q, k, v = maybe_cast("scaled_dot_product_attention", T(query), T(key), T(value))
    m = T(attn_mask)
    if m is not None and m.dtype != torch.bool:
        m = m.to(q.dtype)
    o = _ops.flash_attention(q, k, v, causal=is_causal, scale=scale, mask=m, dropout=dropout_p, training=training)
    return _wrap(o)


def flash_attn_unpadded(query, key, value, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, scale,
                        dropout=0.0, causal=False, return_softmax=False, fixed_seed_offset=None, rng_name="",
                        training=True, name=None):
    """Variable-length attention over packed [total_tokens, heads, dim]: runs each sequence
    through the flash kernel (batched per sequence)."""
    q, k, v = T(query), T(key), T(value)
    cq = T(cu_seqlens_q).tolist()
    ck = T(cu_seqlens_k).tolist()
    outs = []
    for i in range(len(cq) - 1):
        qi = q[cq[i]:cq[i + 1]].unsqueeze(0)
        ki = k[ck[i]:ck[i + 1]].unsqueeze(0)
        vi = v[ck[i]:ck[i + 1]].unsqueeze(0)
        outs.append(_ops.flash_attention(qi, ki, vi, causal=causal, scale=scale, dropout=dropout,
                                         training=training)[0])
    return _wrap(torch.cat(outs, 0)), None


def flash_attn_qkvpacked(qkv, dropout=0.0, causal=False, return_softmax=False, *, fixed_seed_offset=None,
                         rng_name="", training=True, name=None):
    t = T(qkv)  # [B, S, 3, H, D] (paddle packs as [b, s, num_group+2, h, d]); support the 3-way case
    q, k, v = t[:, :, 0], t[:, :, 1], t[:, :, 2]
    return _wrap(_ops.flash_attention(q, k, v, causal=causal, dropout=dropout, training=training)), None


def flash_attention_with_sparse_mask(query, key, value, attn_mask_start_row_indices, attn_mask_start_row=0,
                                     dropout_p=0.0, is_causal=False, return_softmax=False, return_softmax_lse=False,
                                     return_seed_offset=False, training=True, name=None):
    q, k, v = T(query), T(key), T(value)
    S = q.shape[1]
    idx = T(attn_mask_start_row_indices)  # [B, H, Sk]
    rows = torch.arange(S, device=q.device).view(1, 1, S, 1)
    mask = rows < idx.unsqueeze(2)
    if is_causal:
        mask = mask & torch.ones(S, S, dtype=torch.bool, device=q.device).tril()
    o = _ops.flash_attention(q, k, v, causal=False, mask=mask, dropout=dropout_p, training=training)
    return _wrap(o)
