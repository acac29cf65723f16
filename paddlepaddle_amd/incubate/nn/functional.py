"""paddle.incubate.nn.functional — fused transformer ops on the MI355X hot-op set.

Reference: python/paddle/incubate/nn/functional/ (fused_rms_norm.py, fused_layer_norm.py,
fused_rotary_position_embedding.py, fused_bias_act.py, fused_dropout_add.py, fused_matmul_bias.py,
fused_transformer.py, masked_multihead_attention.py, block_multihead_attention.py,
variable_length_memory_efficient_attention.py, blha_get_max_len.py, swiglu.py, fused_moe.py).

Every entry point lands on a hand-written HIP kernel where one exists (RMSNorm / LayerNorm,
residual+dropout, bias+GELU / SwiGLU epilogues, RoPE, flash attention) and composes them otherwise.
Decode attention (masked / block MHA) reads the paged KV cache through the block table in one batched
gather and runs the attention for all sequences of the step together.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as TF

from ... import ops as _ops
from ...framework.tensor import Tensor, _wrap


def _t(x):
    return None if x is None else (x._t if isinstance(x, Tensor) else torch.as_tensor(x))


# --------------------------------------------------------------------------------------- norms
def fused_rms_norm(x, norm_weight, norm_bias, epsilon, begin_norm_axis, bias=None, residual=None, quant_scale=-1,
                   quant_round_type=0, quant_max_bound=0, quant_min_bound=0):
    """out = rms_norm(x + bias + residual); returns (out, residual_out) when residual is given. Residual without
    bias: the add and the norm are one HIP pass (ops.add_rms_norm) when no gradient is needed."""
    if residual is not None and bias is None and norm_weight is not None:
        xt, rt = _t(x), _t(residual)
        shape = xt.shape
        cols = int(math.prod(shape[begin_norm_axis:]))
        s, y = _ops.add_rms_norm(xt.reshape(-1, cols).contiguous(), rt.reshape(-1, cols).contiguous(),
                                 _t(norm_weight).reshape(-1), epsilon)
        y = y.reshape(shape)
        if norm_bias is not None:
            y = y + _t(norm_bias)
        return _wrap(y), _wrap(s.reshape(shape))
    xt = _t(x)
    if bias is not None:
        xt = xt + _t(bias)
    if residual is not None:
        xt = xt + _t(residual)
    res_out = xt
    shape = xt.shape
    cols = int(math.prod(shape[begin_norm_axis:]))
    y = _ops.rms_norm(xt.reshape(-1, cols), _t(norm_weight).reshape(-1), epsilon).reshape(shape)
    if norm_bias is not None:
        y = y + _t(norm_bias)
    if residual is not None:
        return _wrap(y), _wrap(res_out)
    return _wrap(y)


def fused_layer_norm(x, norm_weight, norm_bias, epsilon, residual_alpha=1.0, begin_norm_axis=1, bias=None,
                     residual=None, quant_scale=-1, quant_round_type=0, quant_max_bound=0, quant_min_bound=0):
    xt = _t(x)
    if bias is not None:
        xt = xt + _t(bias)
    if residual is not None:
        xt = xt + residual_alpha * _t(residual)
    res_out = xt
    shape = xt.shape
    cols = int(math.prod(shape[begin_norm_axis:]))
    w = _t(norm_weight)
    b = _t(norm_bias)
    if w is None:
        w = torch.ones(cols, dtype=xt.dtype, device=xt.device)
    if b is None:
        b = torch.zeros(cols, dtype=xt.dtype, device=xt.device)
    y = _ops.layer_norm(xt.reshape(-1, cols), w.reshape(-1), b.reshape(-1), epsilon).reshape(shape)
    if residual is not None:
        return _wrap(y), _wrap(res_out)
    return _wrap(y)


# --------------------------------------------------------------------------------------- RoPE
def fused_rotary_position_embedding(q, k=None, v=None, sin=None, cos=None, position_ids=None,
                                    use_neox_rotary_style=True, time_major=False, rotary_emb_base=10000.0):
    """q/k/v [B, S, H, D] (or [S, B, H, D] when time_major); sin/cos [1, S, 1, D] or None."""
    def prep(t):
        if t is None:
            return None
        t = _t(t)
        return t.transpose(0, 1) if time_major else t
    qt, kt, vt = prep(q), prep(k), prep(v)
    S, D = qt.shape[1], qt.shape[-1]
    if cos is None or sin is None:
        c, s = _ops.rope.rope_tables(S, D, rotary_emb_base, device=qt.device, neox=use_neox_rotary_style)
    else:
        c, s = _t(cos).reshape(-1, D).float(), _t(sin).reshape(-1, D).float()
    if position_ids is not None:
        pid = _t(position_ids).long()
        if pid.dim() == 2 and not bool((pid == pid[:1]).all()):
            # per-batch positions: rotate each batch row with its own tables
            outs = []
            for t in (qt, kt):
                if t is None:
                    outs.append(None)
                    continue
                rows = [_ops.apply_rotary(t[b:b + 1], c[pid[b]], s[pid[b]], use_neox_rotary_style)
                        for b in range(t.shape[0])]
                outs.append(torch.cat(rows, 0))
            qo, ko = outs
            res = [qo, ko, vt]
            return tuple(None if r is None else _wrap(r.transpose(0, 1) if time_major else r) for r in res)
        c, s = c[pid.reshape(-1)[:S]], s[pid.reshape(-1)[:S]]
    qo = _ops.apply_rotary(qt, c, s, use_neox_rotary_style)
    ko = _ops.apply_rotary(kt, c, s, use_neox_rotary_style) if kt is not None else None
    res = [qo, ko, vt]
    return tuple(None if r is None else _wrap(r.transpose(0, 1) if time_major else r) for r in res)


# --------------------------------------------------------------------------------------- activations
def swiglu(x, y=None, name=None):
    xt = _t(x)
    if y is None:
        a, b = xt.chunk(2, -1)
    else:
        a, b = xt, _t(y)
    return _wrap(_ops.swiglu(a, b))


def fused_bias_act(x, bias=None, dequant_scales=None, shift=None, smooth=None, act_method="gelu",
                   compute_dtype="default", quant_scale=-1, quant_round_type=0, quant_max_bound=0, quant_min_bound=0):
    xt = _t(x)
    if dequant_scales is not None:
        xt = xt.float() * _t(dequant_scales)
    b = _t(bias)
    if act_method in ("gelu", "geglu_tanh", "gelu_tanh"):
        y = _ops.bias_gelu(xt, b) if b is not None else _ops.gelu(xt, approximate=True)
    elif act_method in ("swiglu", "silu_glu"):
        h = xt + b if b is not None else xt
        a, g = h.chunk(2, -1)
        y = _ops.swiglu(a, g)
    elif act_method in ("relu",):
        y = TF.relu(xt + b if b is not None else xt)
    elif act_method in ("silu", "swish"):
        y = TF.silu(xt + b if b is not None else xt)
    elif act_method == "geglu":
        h = xt + b if b is not None else xt
        a, g = h.chunk(2, -1)
        y = TF.gelu(a) * g
    else:
        raise ValueError(f"unsupported act_method {act_method}")
    if shift is not None:
        y = y + _t(shift)
    if smooth is not None:
        y = y * _t(smooth)
    return _wrap(y)


def fused_dropout_add(x, y, p=0.5, training=True, mode="upscale_in_train", name=None):
    xt, yt = _t(x), _t(y)
    if mode == "downscale_in_infer":
        if training:
            keep = (torch.rand_like(xt, dtype=torch.float32) >= p).to(xt.dtype)
            return _wrap(xt * keep + yt)
        return _wrap(xt * (1.0 - p) + yt)
    return _wrap(_ops.dropout_add(xt, yt, p if training else 0.0, training))


def fused_matmul_bias(x, y, bias=None, transpose_x=False, transpose_y=False, name=None):
    xt, w = _t(x), _t(y)
    if transpose_x:
        xt = xt.transpose(-1, -2)
    if transpose_y:
        w = w.t()
    return _wrap(_ops.fused_linear(xt, w, _t(bias)))


def fused_linear(x, weight, bias=None, transpose_weight=False, name=None):
    return fused_matmul_bias(x, weight, bias, False, transpose_weight)


def fused_linear_activation(x, y, bias, trans_x=False, trans_y=False, activation=None):
    act = {None: None, "none": None, "gelu": "gelu", "relu": "relu"}[activation]
    xt, w = _t(x), _t(y)
    if trans_x:
        xt = xt.transpose(-1, -2)
    if trans_y:
        w = w.t()
    return _wrap(_ops.fused_linear(xt, w, _t(bias), act=act))


def fused_bias_dropout_residual_layer_norm(x, residual, bias=None, ln_scale=None, ln_bias=None, dropout_rate=0.5,
                                           ln_epsilon=1e-5, training=True, mode="upscale_in_train", name=None):
    xt = _t(x)
    if bias is not None:
        xt = xt + _t(bias)
    h = _ops.dropout_add(xt, _t(residual), dropout_rate if training else 0.0, training)
    cols = h.shape[-1]
    w = _t(ln_scale) if ln_scale is not None else torch.ones(cols, dtype=h.dtype, device=h.device)
    b = _t(ln_bias) if ln_bias is not None else torch.zeros(cols, dtype=h.dtype, device=h.device)
    return _wrap(_ops.layer_norm(h, w, b, ln_epsilon))


# --------------------------------------------------------------------------------------- transformer
def fused_feedforward(x, linear1_weight, linear2_weight, linear1_bias=None, linear2_bias=None, ln1_scale=None,
                      ln1_bias=None, ln2_scale=None, ln2_bias=None, dropout1_rate=0.5, dropout2_rate=0.5,
                      activation="relu", ln1_epsilon=1e-5, ln2_epsilon=1e-5, pre_layer_norm=False, training=True,
                      mode="upscale_in_train", ring_id=-1, add_residual=True, name=None):
    xt = _t(x)
    d = xt.shape[-1]

    def ln(t, s, b, eps):
        w = _t(s) if s is not None else torch.ones(d, dtype=t.dtype, device=t.device)
        bb = _t(b) if b is not None else torch.zeros(d, dtype=t.dtype, device=t.device)
        return _ops.layer_norm(t, w, bb, eps)
    h = ln(xt, ln1_scale, ln1_bias, ln1_epsilon) if pre_layer_norm else xt
    act = "gelu" if activation == "gelu" else ("relu" if activation == "relu" else None)
    h = _ops.fused_linear(h, _t(linear1_weight), _t(linear1_bias), act=act)
    if dropout1_rate and training:
        h = TF.dropout(h, dropout1_rate, True)
    h = _ops.fused_linear(h, _t(linear2_weight), _t(linear2_bias))
    out = _ops.dropout_add(h, xt if add_residual else None, dropout2_rate if training else 0.0, training)
    if not pre_layer_norm:
        out = ln(out, ln2_scale, ln2_bias, ln2_epsilon)
    return _wrap(out)


def fused_multi_head_attention(x, qkv_weight, linear_weight, pre_layer_norm=False, pre_ln_scale=None,
                               pre_ln_bias=None, ln_scale=None, ln_bias=None, pre_ln_epsilon=1e-5, qkv_bias=None,
                               linear_bias=None, cache_kv=None, attn_mask=None, dropout_rate=0.5,
                               attn_dropout_rate=0.5, ln_epsilon=1e-5, training=True, mode="upscale_in_train",
                               ring_id=-1, add_residual=True, num_heads=-1, transpose_qkv_wb=False, name=None):
    """qkv_weight [3, H, D, E] (or [E, 3E] when transpose_qkv_wb); linear_weight [E, E]."""
    xt = _t(x)
    B, S, E = xt.shape
    d = E

    def ln(t, s, b, eps):
        w = _t(s) if s is not None else torch.ones(d, dtype=t.dtype, device=t.device)
        bb = _t(b) if b is not None else torch.zeros(d, dtype=t.dtype, device=t.device)
        return _ops.layer_norm(t, w, bb, eps)
    h = ln(xt, pre_ln_scale, pre_ln_bias, pre_ln_epsilon) if pre_layer_norm else xt
    w = _t(qkv_weight)
    if transpose_qkv_wb:
        H = num_heads
        Dh = E // H
        qkv = _ops.fused_linear(h, w, _t(qkv_bias).reshape(-1) if qkv_bias is not None else None)
    else:
        _, H, Dh, _ = w.shape
        qkv = torch.matmul(h, w.reshape(3 * H * Dh, E).t())
        if qkv_bias is not None:
            qkv = qkv + _t(qkv_bias).reshape(-1)
    qkv = qkv.view(B, S, 3, H, Dh)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    mask = _t(attn_mask)
    o = _ops.flash_attention(q, k, v, causal=False, mask=mask,
                             dropout=attn_dropout_rate if training else 0.0, training=training)
    out = _ops.fused_linear(o.reshape(B, S, H * Dh), _t(linear_weight), _t(linear_bias))
    out = _ops.dropout_add(out, xt if add_residual else None, dropout_rate if training else 0.0, training)
    if not pre_layer_norm:
        out = ln(out, ln_scale, ln_bias, ln_epsilon)
    return _wrap(out)


def fused_multi_transformer(x, ln_scales, ln_biases, qkv_weights, qkv_biases, linear_weights, linear_biases,
                            ffn_ln_scales, ffn_ln_biases, ffn1_weights, ffn1_biases, ffn2_weights, ffn2_biases,
                            pre_layer_norm=True, epsilon=1e-05, cache_kvs=None, time_step=None, attn_mask=None,
                            dropout_rate=0.0, activation="gelu", training=False, mode="upscale_in_train",
                            trans_qkvw=True, ring_id=-1, name=None, **kw):
    """Stack of pre-LN decoder layers (inference)."""
    h = x
    for i in range(len(qkv_weights)):
        h = fused_multi_head_attention(h, qkv_weights[i], linear_weights[i], pre_layer_norm=pre_layer_norm,
                                       pre_ln_scale=ln_scales[i], pre_ln_bias=ln_biases[i],
                                       pre_ln_epsilon=epsilon, qkv_bias=qkv_biases[i], linear_bias=linear_biases[i],
                                       attn_mask=attn_mask, dropout_rate=dropout_rate, attn_dropout_rate=0.0,
                                       training=training, transpose_qkv_wb=not trans_qkvw and False)
        h = fused_feedforward(h, ffn1_weights[i], ffn2_weights[i], ffn1_biases[i], ffn2_biases[i],
                              ln1_scale=ffn_ln_scales[i], ln1_bias=ffn_ln_biases[i], dropout1_rate=0.0,
                              dropout2_rate=dropout_rate, activation=activation, ln1_epsilon=epsilon,
                              pre_layer_norm=pre_layer_norm, training=training)
    return h


# --------------------------------------------------------------------------------------- attention
def variable_length_memory_efficient_attention(query, key, value, seq_lens, kv_seq_lens, mask=None, scale=None,
                                               causal=False, pre_cache_length=0):
    """query [B, H, Sq, D], key/value [B, Hk, Sk, D]; per-batch valid lengths."""
    q, k, v = _t(query), _t(key), _t(value)
    B, H, Sq, D = q.shape
    sl = _t(seq_lens).reshape(-1).tolist()
    kl = _t(kv_seq_lens).reshape(-1).tolist()
    out = torch.zeros_like(q)
    m = _t(mask)
    for b in range(B):
        n, nk = int(sl[b]), int(kl[b]) + pre_cache_length
        if n == 0:
            continue
        qb = q[b:b + 1, :, :n].transpose(1, 2)
        kb = k[b:b + 1, :, :nk].transpose(1, 2)
        vb = v[b:b + 1, :, :nk].transpose(1, 2)
        mb = m[b:b + 1, :, :n, :nk] if m is not None else None
        o = _ops.flash_attention(qb, kb, vb, causal=causal, scale=scale, mask=mb, training=False)
        out[b, :, :n] = o[0].transpose(0, 1)
    return _wrap(out)


def masked_multihead_attention(x, cache_kv=None, bias=None, src_mask=None, cum_offsets=None, sequence_lengths=None,
                               rotary_tensor=None, beam_cache_offset=None, qkv_out_scale=None, out_shift=None,
                               out_smooth=None, seq_len=1, rotary_emb_dims=0, use_neox_rotary_style=False,
                               compute_dtype="default", out_scale=-1, quant_round_type=1, quant_max_bound=127.0,
                               quant_min_bound=-127.0):
    """One decode step. x [B, 3*H*D]; cache_kv [2, B, H, max_len, D] updated in place at the step.
    The step index is sequence_lengths[b] (per batch) or src_mask's width - 1."""
    xt = _t(x)
    cache = _t(cache_kv)
    _, B, H, L, D = cache.shape
    if bias is not None:
        xt = xt + _t(bias)
    qkv = xt.view(B, 3, H, D)
    q, k, v = qkv[:, 0], qkv[:, 1], qkv[:, 2]
    if sequence_lengths is not None:
        steps = _t(sequence_lengths).reshape(-1).long()
    else:
        t = (_t(src_mask).shape[-1] - 1) if src_mask is not None else 0
        steps = torch.full((B,), t, dtype=torch.long, device=xt.device)
    if rotary_tensor is not None and rotary_emb_dims > 0:
        rot = _t(rotary_tensor)  # [2, B, 1, max_len, D] (cos, sin) per position
        cos = rot[0][torch.arange(B), 0, steps]
        sin = rot[1][torch.arange(B), 0, steps]
        q = _rotate_rows(q, cos, sin, use_neox_rotary_style)
        k = _rotate_rows(k, cos, sin, use_neox_rotary_style)
    bi = torch.arange(B, device=xt.device)
    cache[0][bi, :, steps] = k.to(cache.dtype)
    cache[1][bi, :, steps] = v.to(cache.dtype)
    if src_mask is None:  # HIP flash-decoding over the dense cache (ops.dense_decode_attention)
        o = _ops.dense_decode_attention(q, cache[0], cache[1], steps + 1).to(xt.dtype)
    else:
        pos = torch.arange(L, device=xt.device)
        valid = pos[None, :] <= steps[:, None]  # [B, L]
        s = torch.einsum("bhd,bhld->bhl", q.float(), cache[0].float()) / math.sqrt(D)
        sm = _t(src_mask).float().reshape(B, 1, -1)
        s[..., :sm.shape[-1]] = s[..., :sm.shape[-1]] + sm
        s = s.masked_fill(~valid[:, None], float("-inf"))
        p = torch.softmax(s, -1)
        o = torch.einsum("bhl,bhld->bhd", p, cache[1].float()).to(xt.dtype)
    out = o.reshape(B, H * D)
    if out_shift is not None:
        out = out + _t(out_shift)
    if out_smooth is not None:
        out = out * _t(out_smooth)
    return _wrap(out), _wrap(cache)


def _rotate_rows(x, cos, sin, neox):
    # x [B, H, D], cos/sin [B, D]
    xf = x.float()
    c, s = cos.float()[:, None], sin.float()[:, None]
    if neox:
        h = x.shape[-1] // 2
        rot = torch.cat([-xf[..., h:], xf[..., :h]], -1)
    else:
        rot = torch.stack([-xf[..., 1::2], xf[..., 0::2]], -1).flatten(-2)
    return (xf * c + rot * s).to(x.dtype)


def blha_get_max_len(seq_lens_encoder, seq_lens_decoder, batch_size):
    e = _t(seq_lens_encoder).max().reshape(1)
    d = _t(seq_lens_decoder).max().reshape(1)
    return _wrap(e.to(torch.int32)), _wrap(d.to(torch.int32))


def block_multihead_attention(qkv, key_cache, value_cache, seq_lens_encoder, seq_lens_decoder, seq_lens_this_time,
                              padding_offsets, cum_offsets, cu_seqlens_q, cu_seqlens_k, block_tables,
                              pre_key_cache=None, pre_value_cache=None, cache_k_quant_scales=None,
                              cache_v_quant_scales=None, cache_k_dequant_scales=None, cache_v_dequant_scales=None,
                              qkv_out_scale=None, qkv_bias=None, out_shift=None, out_smooth=None,
                              max_enc_len_this_time=None, max_dec_len_this_time=None, rope_emb=None, mask=None,
                              tgt_mask=None, max_seq_len=-1, block_size=64, use_neox_style=False,
                              use_dynamic_cachekv_quant=False, quant_round_type=1, quant_max_bound=127.0,
                              quant_min_bound=-127.0, out_scale=-1, compute_dtype="default", rope_theta=10000.0):
    """Paged-KV attention for a mixed prefill/decode batch.
    qkv [tokens, 3*H*D] (unpadded, sequences back to back per cu_seqlens_q); key/value_cache
    [num_blocks, H, block_size, D]; block_tables [B, max_blocks]. Prefill sequences (encoder len > 0)
    write their K/V into their blocks and run causal flash attention; decode sequences append one
    position at seq_lens_decoder[b] and attend over the cached prefix (one batched gather)."""
    q_all = _t(qkv)
    kc, vc = _t(key_cache), _t(value_cache)
    nb, H, bs, D = kc.shape
    if qkv_bias is not None:
        q_all = q_all + _t(qkv_bias)
    x = q_all.view(-1, 3, H, D)
    enc = _t(seq_lens_encoder).reshape(-1).tolist()
    dec = _t(seq_lens_decoder).reshape(-1).tolist()
    this = _t(seq_lens_this_time).reshape(-1).tolist()
    bt = _t(block_tables).long()
    cu = _t(cu_seqlens_q).reshape(-1).tolist()
    out = torch.zeros(x.shape[0], H, D, dtype=x.dtype, device=x.device)
    rope = _t(rope_emb)

    def rot(t, pos):  # t [n, H, D]; positions [n]
        if rope is None:
            return t
        cos = rope[0].reshape(rope.shape[1], -1, rope.shape[-1])[0][pos] if rope.dim() >= 3 else None
        sin = rope[1].reshape(rope.shape[1], -1, rope.shape[-1])[0][pos]
        cos = torch.cat([cos, cos], -1) if cos.shape[-1] * 2 == D else cos
        sin = torch.cat([sin, sin], -1) if sin.shape[-1] * 2 == D else sin
        return _rotate_rows(t, cos, sin, True if use_neox_style else False)

    dec_b = []
    for b in range(len(this)):
        n = int(this[b])
        if n == 0:
            continue
        s0 = int(cu[b])
        if enc[b] > 0:  # prefill
            pos = torch.arange(n, device=x.device)
            q = rot(x[s0:s0 + n, 0], pos)
            k = rot(x[s0:s0 + n, 1], pos)
            v = x[s0:s0 + n, 2]
            blk = bt[b, pos // bs]
            kc[blk, :, pos % bs] = k.to(kc.dtype)
            vc[blk, :, pos % bs] = v.to(vc.dtype)
            o = _ops.flash_attention(q[None], k[None], v[None], causal=True, training=False)
            out[s0:s0 + n] = o[0]
        else:
            dec_b.append((b, s0))
    if dec_b:  # all decode sequences of the step together
        bidx = torch.as_tensor([b for b, _ in dec_b], device=x.device)
        toks = torch.as_tensor([s for _, s in dec_b], device=x.device)
        steps = torch.as_tensor([int(dec[b]) for b, _ in dec_b], device=x.device)
        q = rot(x[toks, 0], steps)
        k = rot(x[toks, 1], steps)
        v = x[toks, 2]
        blk = bt[bidx, steps // bs]
        kc[blk, :, steps % bs] = k.to(kc.dtype)
        vc[blk, :, steps % bs] = v.to(vc.dtype)
        L = max(int(dec[b]) for b, _ in dec_b) + 1
        nblk = (L + bs - 1) // bs
        # HIP flash-decoding kernel (ops.paged_decode_attention) streams each sequence's blocks
        o = _ops.paged_decode_attention(q.to(kc.dtype), kc, vc, bt[bidx, :nblk], steps + 1, max_len=L)
        out[toks] = o.to(out.dtype)
    res = out.reshape(x.shape[0], H * D)
    if out_shift is not None:
        res = res + _t(out_shift)
    if out_smooth is not None:
        res = res * _t(out_smooth)
    return _wrap(res), _wrap(q_all), _wrap(kc), _wrap(vc)


def fused_moe(*a, **k):
    from ...parallel.moe import fused_moe as _f
    return _f(*a, **k)


def fused_dot_product_attention(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False, scaling_factor=None,
                                training=True, name=None):
    o = _ops.flash_attention(_t(query), _t(key), _t(value), causal=is_causal, scale=scaling_factor,
                             mask=_t(attn_mask), dropout=dropout_p, training=training)
    return _wrap(o)


def memory_efficient_attention(query, key, value, attn_bias=None, p=0.0, scale=None, training=True):
    return fused_dot_product_attention(query, key, value, attn_bias, p, False, scale, training)
