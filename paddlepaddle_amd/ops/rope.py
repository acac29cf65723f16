"""Fused rotary position embedding (HIP).

Reference: paddle/phi/kernels/fusion/gpu/fused_rope_kernel.cu,
python/paddle/incubate/nn/functional/fused_rotary_position_embedding.py.
Layout [batch, seq, heads, head_dim] (paddle flash-attention layout). cos/sin tables are
precomputed on the host side once per (seq, dim) and kept resident (fp32 [seq, head_dim]).
Backward = rotation by -theta (same kernel, inverse flag).
"""
from __future__ import annotations

import torch

from . import _loader as L
from ..framework.trace_hook import static_op


def _rotate_ref(x, cos, sin, neox, inverse):
    # x [B,S,H,D]; cos/sin [S,D] fp32
    c = cos[None, :, None, :]
    s = sin[None, :, None, :]
    if inverse:
        s = -s
    xf = x.float()
    if neox:
        h = x.shape[-1] // 2
        rot = torch.cat([-xf[..., h:], xf[..., :h]], -1)
    else:
        x1 = xf[..., 0::2]
        x2 = xf[..., 1::2]
        rot = torch.stack([-x2, x1], -1).flatten(-2)
    return (xf * c + rot * s).to(x.dtype)


def _rope_hip(x, cos, sin, neox, inverse):
    B, S, H, D = x.shape
    xc = x.contiguous()
    out = torch.empty_like(xc)
    L.call("pa_rope_fwd", L.ptr(xc), L.ptr(cos), L.ptr(sin), L.ptr(out), B, S, H, D,
           int(neox) | (int(inverse) << 1), L.dcode(xc), L.stream_ptr())
    return out


class _RopeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cos, sin, neox):
        ctx.save_for_backward(cos, sin)
        ctx.neox = neox
        return _rope_hip(x, cos, sin, neox, False)

    @staticmethod
    def backward(ctx, dy):
        cos, sin = ctx.saved_tensors
        return _rope_hip(dy.to(dy.dtype), cos, sin, ctx.neox, True), None, None, None


@static_op
def apply_rotary(x, cos, sin, neox=True):
    """Rotate x [B,S,H,D] by tables cos/sin [S,D] (fp32, already expanded to head_dim)."""
    cos = cos.float().contiguous()
    sin = sin.float().contiguous()
    if L.hip_enabled_for(x) and x.dtype in L._DT and x.shape[-1] % (16 if neox else 8) == 0 and cos.shape[0] >= x.shape[1]:
        return _RopeFn.apply(x, cos, sin, neox)
    return _rotate_ref(x, cos[: x.shape[1]], sin[: x.shape[1]], neox, False)


def rope_tables(seq_len, dim, base=10000.0, device=None, neox=True):
    inv = 1.0 / (base ** (torch.arange(0, dim, 2, dtype=torch.float32, device=device) / dim))
    t = torch.arange(seq_len, dtype=torch.float32, device=device)
    f = torch.outer(t, inv)  # [S, D/2]
    if neox:
        emb = torch.cat([f, f], -1)
    else:
        emb = torch.repeat_interleave(f, 2, -1)
    return emb.cos(), emb.sin()


def decode_rope_cache(qkv, H, Hkv, D, cos_row, sin_row, pos_t, k_cache, v_cache):
    """Decode step, one token per sequence: qkv [B, (H + 2*Hkv)*D] (the fused projection output) ->
    rotated q [B, H, D]; rotated k and v are written into the dense caches [Bc, Hkv, Lc, D] at the
    device-side position ``pos_t`` ([1] int64). cos_row / sin_row: fp32 [1, D] rows at that position."""
    B = qkv.shape[0]
    if (L.hip_enabled_for(qkv) and qkv.dtype in L._DT and D % 16 == 0 and qkv.stride(-1) == 1
            and k_cache.is_contiguous() and v_cache.is_contiguous() and L.has("pa_decode_rope_cache")):
        q = torch.empty(B, H, D, dtype=qkv.dtype, device=qkv.device)
        cs = cos_row.float().contiguous()
        sn = sin_row.float().contiguous()
        L.call("pa_decode_rope_cache", L.ptr(qkv), qkv.stride(0), L.ptr(cs), L.ptr(sn), L.ptr(pos_t), L.ptr(q),
               L.ptr(k_cache), L.ptr(v_cache), B, H, Hkv, D, k_cache.shape[2], L.dcode(qkv), L.stream_ptr())
        return q
    q, k, v = qkv.split([H * D, Hkv * D, Hkv * D], -1)
    q = apply_rotary(q.reshape(B, 1, H, D), cos_row, sin_row)
    k = apply_rotary(k.reshape(B, 1, Hkv, D), cos_row, sin_row)
    k_cache[:B].index_copy_(2, pos_t, k.transpose(1, 2))
    v_cache[:B].index_copy_(2, pos_t, v.reshape(B, 1, Hkv, D).transpose(1, 2))
    return q.reshape(B, H, D)
