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
def _quant_out(y, quant_scale, round_type, max_bound, min_bound):
    """int8 output of a quantising norm (reference fused_layernorm_kernel.cu QuantHelperFunc): q =
    clip(round(max_bound * quant_scale * y), min_bound, max_bound); round_type 0 rounds half to even (rint),
    1 half away from zero (round)."""
    v = y.float() * (float(max_bound) * float(quant_scale))
    v = torch.round(v) if int(round_type) == 0 else torch.sign(v) * torch.floor(v.abs() + 0.5)
    return v.clamp(float(min_bound), float(max_bound)).to(torch.int8)


def _with_quant(fn):
    """quant_scale > 0 turns the normalised output into int8 (residual_out stays in the input dtype)."""
    def run(*a, quant_scale=-1, quant_round_type=0, quant_max_bound=0, quant_min_bound=0, **k):
        out = fn(*a, **k)
        if quant_scale is None or float(quant_scale) <= 0:
            return out
        if float(quant_max_bound) <= 0:
            raise ValueError("quant_scale > 0 needs quant_max_bound > 0 (e.g. 127) and quant_min_bound (e.g. -127)")
        y = out[0] if isinstance(out, tuple) else out
        q = _wrap(_quant_out(_t(y), quant_scale, quant_round_type, quant_max_bound, quant_min_bound))
        return (q, out[1]) if isinstance(out, tuple) else q
    return run


def fused_rms_norm(x, norm_weight, norm_bias, epsilon, begin_norm_axis, bias=None, residual=None, quant_scale=-1,
                   quant_round_type=0, quant_max_bound=0, quant_min_bound=0):
    """out = rms_norm(x + bias + residual); returns (out, residual_out) when residual is given. Residual without
    bias: the add and the norm are one HIP pass (ops.add_rms_norm) when no gradient is needed. ``quant_scale`` > 0:
    ``out`` is int8 (reference fused_rms_norm quantised output, see _quant_out)."""
    return _with_quant(_fused_rms_norm)(x, norm_weight, norm_bias, epsilon, begin_norm_axis, bias, residual,
                                        quant_scale=quant_scale, quant_round_type=quant_round_type,
                                        quant_max_bound=quant_max_bound, quant_min_bound=quant_min_bound)


def _fused_rms_norm(x, norm_weight, norm_bias, epsilon, begin_norm_axis, bias=None, residual=None):
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
    """out = layer_norm(x + bias + residual_alpha * residual); (out, residual_out) with a residual; int8 ``out``
    when ``quant_scale`` > 0 (reference fused_layernorm_kernel.cu:996)."""
    return _with_quant(_fused_layer_norm)(x, norm_weight, norm_bias, epsilon, residual_alpha, begin_norm_axis, bias,
                                          residual, quant_scale=quant_scale, quant_round_type=quant_round_type,
                                          quant_max_bound=quant_max_bound, quant_min_bound=quant_min_bound)


def _fused_layer_norm(x, norm_weight, norm_bias, epsilon, residual_alpha=1.0, begin_norm_axis=1, bias=None,
                      residual=None):
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
    return _wrap(_ops.swiglu(_t(x), None if y is None else _t(y)))


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


def _fmt_norm(t, w, b, eps, norm_type):
    if norm_type == "rmsnorm":
        return _ops.rms_norm(t, _t(w), eps)
    d = t.shape[-1]
    ww = _t(w) if w is not None else torch.ones(d, dtype=t.dtype, device=t.device)
    bb = _t(b) if b is not None else torch.zeros(d, dtype=t.dtype, device=t.device)
    return _ops.layer_norm(t, ww, bb, eps)


def _mp_allreduce(t, ring_id):
    """ring_id >= 0: tensor-parallel layers; the row-parallel outputs are summed over the mp group."""
    if ring_id is None or ring_id < 0:
        return t
    from ...parallel import tensor_parallel as _tp
    g = _tp._mp_group()
    if _tp._ws(g) > 1:
        torch.distributed.all_reduce(t, group=g.process_group)
    return t


def fused_multi_transformer(x, ln_scales, ln_biases, qkv_weights, qkv_biases, linear_weights, linear_biases,
                            ffn_ln_scales, ffn_ln_biases, ffn1_weights, ffn1_biases, ffn2_weights, ffn2_biases,
                            pre_layer_norm=True, epsilon=1e-05, residual_alpha=1.0, cache_kvs=None, beam_offset=None,
                            pre_caches=None, seq_lens=None, rotary_embs=None, time_step=None, attn_mask=None,
                            dropout_rate=0.0, rotary_emb_dims=0, activation="gelu", training=False,
                            mode="upscale_in_train", trans_qkvw=True, ring_id=-1, norm_type="layernorm",
                            use_neox_rotary_style=False, gqa_group_size=-1, name=None):
    """Stack of decoder layers for generation (reference incubate/nn/functional/fused_transformer.py:1015).

    Three modes, by (cache_kvs, time_step):
    - no cache: every layer is attention over the S tokens (+ attn_mask), LN/FFN, residuals.
    - cache_kvs, time_step None (context / prefill): K/V of the S tokens (after pre_caches, if any)
      are written into cache_kvs[i][:, :, :, P:P+S] (cache layout [2, B, kv_heads, max_len, D]).
    - cache_kvs and time_step (decode, S == 1): K/V are written at position time_step (or seq_lens[b]
      per sequence) and the token attends over positions [0, step] of the cache with the HIP
      flash-decoding kernel (ops.dense_decode_attention), or the math path when attn_mask is given.
    Returns out, or (out, cache_kvs) when cache_kvs is given (the caches are updated in place).
    beam_offset [batch, beam, max_len] (decode): beam-search cache indirection, as masked_multihead_attention's
    beam_cache_offset (math path over the re-gathered cache).
    qkv_weights: [3, H, D, E] (trans_qkvw) or [E, 3, H, D]; with gqa_group_size = kv heads,
    [H + 2*kv_heads, D, E] / [E, H + 2*kv_heads, D]."""
    if mode not in ("upscale_in_train", "downscale_in_infer"):
        raise ValueError(f"fused_multi_transformer: mode must be upscale_in_train or downscale_in_infer, got {mode!r}")

    def drop_add(t, res):  # residual + dropout(t) in the requested mode
        if mode == "downscale_in_infer" and dropout_rate > 0:
            # training: keep mask without rescale (= the upscaling kernel applied to t * (1 - p)); inference: t * (1 - p)
            return _ops.dropout_add(t * (1.0 - dropout_rate), res, dropout_rate if training else 0.0, training)
        return _ops.dropout_add(t, res, dropout_rate if training else 0.0, training)
    xt = _t(x)
    B, S, E = xt.shape
    decode = cache_kvs is not None and time_step is not None
    if decode and S != 1:
        raise ValueError("fused_multi_transformer decode (time_step given) takes one token per sequence")
    if decode:
        if seq_lens is not None:
            steps = _t(seq_lens).reshape(-1).to(device=xt.device, dtype=torch.long)
        else:  # time_step lives on the host (CPUPlace in the reference): no device sync
            ts = _t(time_step)
            steps = torch.full((B,), int(ts.reshape(-1)[0]), dtype=torch.long, device=xt.device)
    rot = None
    if rotary_embs is not None and rotary_emb_dims > 0:
        r = _t(rotary_embs)  # [2, B|1, 1, L, D]
        rot = (r[0, :, 0], r[1, :, 0])  # [B|1, L, D]
    mask = _t(attn_mask)
    act = "gelu" if activation == "gelu" else ("relu" if activation == "relu" else None)
    if act is None:
        raise ValueError(f"fused_multi_transformer: unsupported activation {activation}")
    h = xt
    for i in range(len(qkv_weights)):
        w = _t(qkv_weights[i])
        if trans_qkvw:
            Dh = w.shape[-2]
            w2 = w.reshape(-1, E)  # [(3|H+2Hk) * Dh, E]
            nh = w2.shape[0] // Dh
        else:
            Dh = w.shape[-1]
            w2 = w.reshape(E, -1).t()
            nh = w2.shape[0] // Dh
        Hk = gqa_group_size if gqa_group_size and gqa_group_size > 0 else nh // 3
        H = nh - 2 * Hk
        residual = h
        t = _fmt_norm(h, ln_scales[i], ln_biases[i], epsilon, norm_type) if pre_layer_norm else h
        qkv = torch.matmul(t, w2.t())
        if qkv_biases is not None and qkv_biases[i] is not None:
            qkv = qkv + _t(qkv_biases[i]).reshape(-1)
        qkv = qkv.view(B, S, nh, Dh)
        q, k, v = qkv[:, :, :H], qkv[:, :, H:H + Hk], qkv[:, :, H + Hk:]
        cache = _t(cache_kvs[i]) if cache_kvs is not None else None
        if decode:
            q, k, v = q[:, 0], k[:, 0], v[:, 0]  # [B, heads, Dh]
            if rot is not None:
                bi = torch.arange(B, device=xt.device) % rot[0].shape[0]
                cs, sn = rot[0][bi, steps], rot[1][bi, steps]
                q = _rotate_rows(q, cs, sn, use_neox_rotary_style)
                k = _rotate_rows(k, cs, sn, use_neox_rotary_style)
            bi = torch.arange(B, device=xt.device)
            cache[0][bi, :, steps] = k.to(cache.dtype)
            cache[1][bi, :, steps] = v.to(cache.dtype)
            if mask is None and beam_offset is None:
                o = _ops.dense_decode_attention(q.to(cache.dtype), cache[0], cache[1], steps + 1).to(q.dtype)
            else:  # additive [B, 1, 1, step + 1] mask / beam indirection: math path over the cache prefix
                Lc = cache.shape[3]
                G = H // Hk
                kc, vc = _beam_kv(cache, beam_offset, steps) if beam_offset is not None else (cache[0], cache[1])
                s = torch.einsum("bkgd,bkld->bkgl", q.float().view(B, Hk, G, Dh), kc.float()) / math.sqrt(Dh)
                if mask is not None:
                    m = mask.float().reshape(B, 1, 1, -1)
                    s[..., :m.shape[-1]] += m
                valid = torch.arange(Lc, device=xt.device)[None] <= steps[:, None]
                s = s.masked_fill(~valid[:, None, None], float("-inf"))
                o = torch.einsum("bkgl,bkld->bkgd", torch.softmax(s, -1), vc.float()).reshape(B, H, Dh)
            o = o.to(h.dtype).reshape(B, 1, H * Dh)
        else:
            if rot is not None:
                pos = torch.arange(S, device=xt.device)
                cs = rot[0][:, pos].expand(B, S, -1).reshape(B * S, -1)
                sn = rot[1][:, pos].expand(B, S, -1).reshape(B * S, -1)
                q = _rotate_rows(q.reshape(B * S, H, Dh), cs, sn, use_neox_rotary_style).view(B, S, H, Dh)
                k = _rotate_rows(k.reshape(B * S, Hk, Dh), cs, sn, use_neox_rotary_style).view(B, S, Hk, Dh)
            kk, vv = k, v
            P = 0
            if pre_caches is not None and pre_caches[i] is not None:
                pc = _t(pre_caches[i])  # [2, B, Hk, P, Dh]
                P = pc.shape[3]
                kk = torch.cat([pc[0].transpose(1, 2).to(k.dtype), k], 1)
                vv = torch.cat([pc[1].transpose(1, 2).to(v.dtype), v], 1)
            if cache is not None:
                cache[0][:, :, :P + S] = kk.transpose(1, 2).to(cache.dtype)
                cache[1][:, :, :P + S] = vv.transpose(1, 2).to(cache.dtype)
            o = _ops.flash_attention(q, kk, vv, causal=False, mask=mask,
                                     dropout=0.0, training=False).reshape(B, S, H * Dh)
        out = torch.matmul(o, _t(linear_weights[i]))
        out = _mp_allreduce(out, ring_id)
        if linear_biases is not None and linear_biases[i] is not None:
            out = out + _t(linear_biases[i])
        out = drop_add(out, residual * residual_alpha if residual_alpha != 1.0 else residual)
        if not pre_layer_norm:
            out = _fmt_norm(out, ln_scales[i], ln_biases[i], epsilon, norm_type)
        residual = out
        t = _fmt_norm(out, ffn_ln_scales[i], ffn_ln_biases[i], epsilon, norm_type) if pre_layer_norm else out
        f = _ops.fused_linear(t, _t(ffn1_weights[i]), _t(ffn1_biases[i]) if ffn1_biases is not None else None,
                              act=act)
        f = torch.matmul(f, _t(ffn2_weights[i]))
        f = _mp_allreduce(f, ring_id)
        if ffn2_biases is not None and ffn2_biases[i] is not None:
            f = f + _t(ffn2_biases[i])
        h = drop_add(f, residual * residual_alpha if residual_alpha != 1.0 else residual)
        if not pre_layer_norm:
            h = _fmt_norm(h, ffn_ln_scales[i], ffn_ln_biases[i], epsilon, norm_type)
    return (_wrap(h), cache_kvs) if cache_kvs is not None else _wrap(h)


# --------------------------------------------------------------------------------------- attention
def variable_length_memory_efficient_attention(query, key, value, seq_lens, kv_seq_lens, mask=None, scale=None,
                                               causal=False, pre_cache_length=0):
    """query [B, H, Sq, D], key/value [B, Hk, Sk, D] padded; row i of batch b is valid for i < seq_lens[b] and
    attends to keys j < kv_seq_lens[b] + pre_cache_length (and, when causal, j <= i + pre_cache_length).
    One flash-attention launch with the lengths folded into a dense keep-mask built on the device (no host
    sync; capturable); rows past seq_lens[b] come out zero. Reference:
    incubate/nn/functional/variable_length_memory_efficient_attention.py:33."""
    q, k, v = _t(query), _t(key), _t(value)
    B, H, Sq, D = q.shape
    Sk = k.shape[2]
    dev = q.device
    sl = _t(seq_lens).reshape(-1).to(dev)
    kl = _t(kv_seq_lens).reshape(-1).to(dev) + int(pre_cache_length)
    rows = torch.arange(Sq, device=dev)
    cols = torch.arange(Sk, device=dev)
    keep = cols.view(1, 1, 1, Sk) < kl.view(B, 1, 1, 1)
    if causal:
        keep = keep & (cols.view(1, 1, 1, Sk) <= rows.view(1, 1, Sq, 1) + int(pre_cache_length))
    row_ok = rows.view(1, Sq) < sl.view(B, 1)
    keep = keep | ~row_ok.view(B, 1, Sq, 1)  # padded rows see every key (finite softmax), zeroed below
    m = _t(mask)
    if m is not None:
        full = m.float().expand(B, 1, Sq, Sk) if m.dim() == 4 else m.float()
        attn_mask = full.masked_fill(~keep, float("-inf"))
    else:
        attn_mask = keep
    o = _ops.flash_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), causal=False, scale=scale,
                             mask=attn_mask, training=False)  # [B, Sq, H, D]
    o = o.transpose(1, 2)
    return _wrap(torch.where(row_ok.view(B, 1, Sq, 1), o, torch.zeros((), dtype=o.dtype, device=dev)))


def masked_multihead_attention(x, cache_kv=None, bias=None, src_mask=None, cum_offsets=None, sequence_lengths=None,
                               rotary_tensor=None, beam_cache_offset=None, qkv_out_scale=None, out_shift=None,
                               out_smooth=None, seq_len=1, rotary_emb_dims=0, use_neox_rotary_style=False,
                               compute_dtype="default", out_scale=-1, quant_round_type=1, quant_max_bound=127.0,
                               quant_min_bound=-127.0):
    """One decode step. x [B, 3*H*D]; cache_kv [2, B, H, max_len, D] updated in place at the step.
    The step index is sequence_lengths[b] (per batch) or src_mask's width - 1. ``qkv_out_scale``: x is the int32
    output of an int8 QKV GEMM, dequantised by these per-column scales; ``out_scale`` > 0: int8 output
    (reference QuantHelperFunc rounding / bounds). ``beam_cache_offset`` [batch, beam, max_len]: beam-search KV
    indirection — key / value of step t of row b are read from beam ``beam_cache_offset[b, t]`` of b's batch
    entry (an entry of 0 reads b's own cache, as the reference kernel does, masked_multihead_attention_kernel.cu
    :423); the result is then (out, cache_kv, beam_cache_offset). ``cum_offsets`` raises, as in the reference
    kernel (masked_multihead_attention_kernel.cu:1061 "does not support cum_offsets")."""
    if cum_offsets is not None:
        raise NotImplementedError("masked_multihead_attention: cum_offsets is not supported (as in the reference "
                                  "kernel)")
    if compute_dtype not in ("default", "bf16", "fp16", "fp32"):
        raise ValueError(f"compute_dtype must be default / bf16 / fp16 / fp32, got {compute_dtype!r}")
    xt = _t(x)
    cache = _t(cache_kv)
    _, B, H, L, D = cache.shape
    if qkv_out_scale is not None:
        xt = (xt.float() * _t(qkv_out_scale).float().reshape(-1)).to(cache.dtype)
    elif not xt.is_floating_point():
        raise ValueError("masked_multihead_attention: an integer x needs qkv_out_scale")
    if bias is not None:
        xt = xt + _t(bias).to(xt.dtype)
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
    if beam_cache_offset is not None:
        kc, vc = _beam_kv(cache, beam_cache_offset, steps)                          # [B, H, L, D]
        pos = torch.arange(L, device=xt.device)
        valid = pos[None, :] <= steps[:, None]
        s_ = torch.einsum("bhd,bhld->bhl", q.float(), kc.float()) / math.sqrt(D)
        if src_mask is not None:
            sm = _t(src_mask).float().reshape(B, 1, -1)
            s_[..., :sm.shape[-1]] = s_[..., :sm.shape[-1]] + sm
        s_ = s_.masked_fill(~valid[:, None], float("-inf"))
        o = torch.einsum("bhl,bhld->bhd", torch.softmax(s_, -1), vc.float()).to(xt.dtype)
    elif src_mask is None:  # HIP flash-decoding over the dense cache (ops.dense_decode_attention)
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
    if out_scale is not None and float(out_scale) > 0:
        out = _quant_out(out, out_scale, quant_round_type, quant_max_bound, quant_min_bound)
    if beam_cache_offset is not None:
        return _wrap(out), _wrap(cache), beam_cache_offset
    return _wrap(out), _wrap(cache)


def _beam_kv(cache, beam_cache_offset, steps):
    """Key / value caches [B, heads, L, D] as seen through beam-search indirection: position t of row b comes
    from beam ``off[b, t]`` of b's batch entry (0: b's own row); the current step is always the row's own
    (reference masked_multihead_attention_kernel.cu beam_offsets)."""
    _, B, Hk, L, D = cache.shape
    dev = cache.device
    off = _t(beam_cache_offset)
    W = off.shape[1] if off.dim() == 3 else 1
    off = off.reshape(B, -1)[:, :L].long()
    off = off.masked_fill(torch.arange(L, device=dev)[None, :] >= steps[:, None], 0)
    bi = torch.arange(B, device=dev)
    src = (bi // W).view(B, 1) * W + torch.where(off != 0, off, (bi % W).view(B, 1))  # [B, L] source row
    hh = torch.arange(Hk, device=dev).view(1, Hk, 1)
    tt = torch.arange(L, device=dev).view(1, 1, L)
    return cache[0][src.view(B, 1, L), hh, tt], cache[1][src.view(B, 1, L), hh, tt]


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
    """Paged-KV attention for a mixed prefill/decode batch, entirely on the device (no host reads of the
    length tensors, so a decode step can be captured in a hipGraph and replayed with new lengths).
    Reference: incubate/nn/functional/block_multihead_attention.py:33.

    qkv [tokens, (H + 2*Hk) * D]: the step's tokens back to back per cu_seqlens_q; key/value_cache
    [num_blocks, Hk, block_size, D]; block_tables [B, max_blocks]. Token t of sequence b sits at cache
    position pos = t - cu_seqlens_q[b] + seq_lens_decoder[b]; its rotated K/V are scattered to
    block_tables[b, pos // bs] row pos % bs. Prefill tokens (seq_lens_encoder[b] > 0) attend causally
    within their sequence through the varlen flash-attention kernel; decode tokens attend over cache
    positions [0, pos] through the paged flash-decoding kernel. max_enc_len_this_time /
    max_dec_len_this_time (host tensors from blha_get_max_len) skip a phase that has no tokens; without
    them both run and the per-token result is selected on the device.
    Static int8 cache quantisation (cache_k/v_quant_scales, cache_k/v_dequant_scales [kv_heads], uint8 caches): the
    step's K / V are stored as clip(round(scale * x), min_bound, max_bound) + 128 and read back as
    (u - 128) * dequant_scale, the current token's own K / V unquantised (reference block_attn.h CacheKernel /
    mul_pointer_v2); ``use_dynamic_cachekv_quant``: the scales are computed from the step (127 / max|x| per kv head
    over its tokens) into the [batch, kv_heads] rows of the prefilling sequences, decode reads row 0
    (quant_write_cache_int8_kernel). out_scale > 0 gives an int8 output (QuantHelperFunc rounding / bounds).
    pre_key_cache / pre_value_cache [B, kv_heads, P, D] (prefix caches): a prefilling sequence's cache positions
    0 .. P-1 receive them and its tokens start at P; its attention covers the prefix plus its tokens, causal
    (bottom-right) or through the additive ``mask`` [B, 1, S, P + S] when given; decode tokens with ``tgt_mask``
    [B, 1, 1, L] add it over their cache positions. The masked / prefixed phases run a math path (per-sequence
    lengths read on the host), the others the HIP kernels."""
    if (pre_key_cache is None) != (pre_value_cache is None):
        raise ValueError("block_multihead_attention: pre_key_cache and pre_value_cache go together")
    quant_cache = cache_k_quant_scales is not None
    if use_dynamic_cachekv_quant and not quant_cache:
        raise ValueError("block_multihead_attention: dynamic cache-KV quantisation needs the scale tensors")
    if quant_cache and any(t is None for t in (cache_v_quant_scales, cache_k_dequant_scales,
                                               cache_v_dequant_scales)):
        raise ValueError("block_multihead_attention: int8 caches need cache_k/v_quant_scales and "
                         "cache_k/v_dequant_scales")
    q_all = _t(qkv)
    kc, vc = _t(key_cache), _t(value_cache)
    nb, Hk, bs, D = kc.shape
    if quant_cache and kc.dtype != torch.uint8:
        raise ValueError("block_multihead_attention: quantised caches are uint8 (int8 value + 128)")
    if qkv_out_scale is not None:  # int32 GEMM output -> real values
        cdt = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(
            compute_dtype, kc.dtype if kc.is_floating_point() else torch.bfloat16)
        q_all = (q_all.float() * _t(qkv_out_scale).float().reshape(-1)).to(cdt)
    if qkv_bias is not None:
        q_all = q_all + _t(qkv_bias).reshape(-1)
    T = q_all.shape[0]
    H = q_all.shape[1] // D - 2 * Hk
    x = q_all.view(T, H + 2 * Hk, D)
    q, k, v = x[:, :H], x[:, H:H + Hk], x[:, H + Hk:]
    dev = x.device
    cu = _t(cu_seqlens_q).reshape(-1).to(device=dev, dtype=torch.long)
    B = cu.numel() - 1
    tok = torch.arange(T, device=dev)
    bid = torch.searchsorted(cu[1:].contiguous(), tok, right=True).clamp_(max=B - 1)
    dec = _t(seq_lens_decoder).reshape(-1).to(device=dev, dtype=torch.long)
    enc = _t(seq_lens_encoder).reshape(-1).to(device=dev, dtype=torch.long)
    pk, pv = _t(pre_key_cache), _t(pre_value_cache)
    P = pk.shape[2] if pk is not None else 0
    pos = tok - cu[bid] + dec[bid] + P
    rope = _t(rope_emb)
    if rope is not None:  # [2, B|1, max_len, 1, D//2 | D] (cos, sin)
        cos = rope[0].reshape(rope.shape[1], rope.shape[2], -1)
        sin = rope[1].reshape(rope.shape[1], rope.shape[2], -1)
        rb = bid % cos.shape[0]
        cs, sn = cos[rb, pos], sin[rb, pos]
        if cs.shape[-1] * 2 == D:
            cs, sn = torch.cat([cs, cs], -1), torch.cat([sn, sn], -1)
        q = _rotate_rows(q, cs, sn, bool(use_neox_style))
        k = _rotate_rows(k, cs, sn, bool(use_neox_style))
    bt = _t(block_tables).to(device=dev, dtype=torch.long)
    blk = bt[bid, pos // bs]
    if P:  # prefix caches into positions 0 .. P-1 of the prefilling sequences
        pb = torch.nonzero(enc > 0).reshape(-1)
        pp = torch.arange(P, device=dev)
        pblk = bt[pb.view(-1, 1), (pp // bs).view(1, -1)]                      # [nb_pre, P]
        for cache, src in ((kc, pk), (vc, pv)):
            vals = src[pb].permute(0, 2, 1, 3).to(dev)                             # [nb_pre, P, Hk, D]
            if not quant_cache:
                cache[pblk, :, (pp % bs).view(1, -1)] = vals.to(cache.dtype)
    adt = kc.dtype if not quant_cache else (q_all.dtype if q_all.is_floating_point() else torch.bfloat16)
    if quant_cache:
        def qz(t, sc):  # [T, Hk, D] -> uint8 with per-token per-kv-head scales sc [T, Hk]
            z = t.float() * sc.unsqueeze(-1)
            z = torch.round(z) if int(quant_round_type) == 0 else torch.sign(z) * torch.floor(z.abs() + 0.5)
            return (z.clamp(float(quant_min_bound), float(quant_max_bound)) + 128.0).to(torch.uint8)
        sk, sv = _t(cache_k_quant_scales), _t(cache_v_quant_scales)
        if use_dynamic_cachekv_quant:
            # reference block_attn.h quant_write_cache_int8_kernel: per kv head, scale = 127 / max|x| over the
            # step's tokens, stored (with 1 / scale) in the [batch, kv_heads] rows of the prefilling sequences;
            # prefill tokens use their sequence's row, decode tokens (and the decode reads) row 0
            dk, dv = _t(cache_k_dequant_scales), _t(cache_v_dequant_scales)
            pre = enc > 0
            for t, s_, d_ in ((k, sk, dk), (v, sv, dv)):
                amax = t.float().abs().amax(dim=(0, 2)).clamp_min(1e-20)        # [Hk]
                rows = s_.view(-1, Hk)
                upd = pre.view(-1, 1)[:rows.shape[0]]
                rows.copy_(torch.where(upd, (127.0 / amax).to(rows.dtype).view(1, -1), rows))
                dr = d_.view(-1, Hk)
                dr.copy_(torch.where(upd, (amax / 127.0).to(dr.dtype).view(1, -1), dr))
            tok_pre = pre[bid].view(T, 1)
            ksc_t = torch.where(tok_pre, sk.view(-1, Hk).float()[bid], sk.view(-1, Hk).float()[0].view(1, -1))
            vsc_t = torch.where(tok_pre, sv.view(-1, Hk).float()[bid], sv.view(-1, Hk).float()[0].view(1, -1))
        else:
            ksc_t = sk.float().reshape(1, -1).to(dev).expand(T, Hk)
            vsc_t = sv.float().reshape(1, -1).to(dev).expand(T, Hk)
        kc[blk, :, pos % bs] = qz(k, ksc_t)
        vc[blk, :, pos % bs] = qz(v, vsc_t)
        if P:
            for cache, src, sc in ((kc, pk, sk), (vc, pv, sv)):
                rows = sc.float().reshape(-1, Hk).to(dev)
                srow = rows[pb] if rows.shape[0] > 1 else rows.expand(pb.numel(), Hk)  # [nb_pre, Hk]
                vals = src[pb].permute(0, 2, 1, 3).to(dev)                                 # [nb_pre, P, Hk, D]
                cache[pblk, :, (pp % bs).view(1, -1)] = qz(vals.reshape(-1, Hk, D),
                                                           srow.repeat_interleave(P, 0)).view(vals.shape)
    else:
        kc[blk, :, pos % bs] = k.to(kc.dtype)
        vc[blk, :, pos % bs] = v.to(vc.dtype)
    def host(t):  # the hints are host tensors (blha_get_max_len on CPU): reading them never syncs the device
        if t is None:
            return None
        tt = _t(t)
        if tt.is_cuda and torch.cuda.is_current_stream_capturing():
            return None  # a device-resident hint cannot be read inside a captured graph: run both phases
        return int(tt.reshape(-1)[0])
    max_enc, max_dec = host(max_enc_len_this_time), host(max_dec_len_this_time)
    run_prefill = max_enc is None or max_enc > 0
    run_decode = max_dec is None or max_dec > 0
    prefill_tok = enc[bid] > 0
    o = None
    if run_prefill and (P or mask is not None):
        o = _blha_prefill_math(q.to(adt), k.to(adt), v.to(adt), cu, enc, pk, pv, _t(mask))
    elif run_prefill:
        mq = max_enc if max_enc else T
        o_p = _ops.attention.attention(q.to(adt), k.to(adt), v.to(adt), causal=True, cu_seqlens_q=cu,
                                       cu_seqlens_k=cu, max_seqlen_q=mq, max_seqlen_k=mq, training=False)
        o = o_p
    if run_decode:
        # prefill tokens ride along reading one position; their rows are replaced by o_p below
        lens = torch.where(prefill_tok, torch.ones_like(pos), pos + 1) if run_prefill else pos + 1
        ml = None
        if max_dec is not None:
            ml = max_dec + 1 + P
        kd, vd = kc, vc
        if quant_cache:  # dequantised view of the cache; the step's own rows stay exact
            kdq = _t(cache_k_dequant_scales).float().reshape(-1, Hk)[0].to(dev)  # dynamic: row 0, as the reference
            vdq = _t(cache_v_dequant_scales).float().reshape(-1, Hk)[0].to(dev)
            kd = ((kc.float() - 128.0) * kdq.view(1, -1, 1, 1)).to(adt)
            vd = ((vc.float() - 128.0) * vdq.view(1, -1, 1, 1)).to(adt)
            kd[blk, :, pos % bs] = k.to(adt)
            vd[blk, :, pos % bs] = v.to(adt)
        if tgt_mask is not None:
            o_d = _blha_decode_math(q.to(adt), kd, vd, bt[bid], lens, _t(tgt_mask)[bid])
        else:
            o_d = _ops.paged_decode_attention(q.to(adt), kd, vd, bt[bid], lens, max_len=ml)
        o = o_d if o is None else torch.where(prefill_tok.view(T, 1, 1), o, o_d)
    res = o.to(q_all.dtype).reshape(T, H * D)
    if out_shift is not None:
        res = res + _t(out_shift)
    if out_smooth is not None:
        res = res * _t(out_smooth)
    if out_scale is not None and float(out_scale) > 0:
        res = _quant_out(res, out_scale, quant_round_type, quant_max_bound, quant_min_bound)
    return _wrap(res), _wrap(q_all), _wrap(kc), _wrap(vc)


def _blha_prefill_math(q, k, v, cu, enc, pk, pv, mask):
    """Prefill attention of the prefilling sequences with prefix caches and / or an additive mask (math path;
    per-sequence lengths on the host). q [T, H, D], k / v [T, Hk, D]; rows of other sequences stay zero."""
    T, H, D = q.shape
    Hk = k.shape[1]
    o = torch.zeros_like(q)
    cuh, ench = cu.tolist(), enc.tolist()
    for b in range(len(cuh) - 1):
        if ench[b] <= 0:
            continue
        s0, s1 = cuh[b], cuh[b + 1]
        n = s1 - s0
        kk, vv = k[s0:s1].transpose(0, 1).float(), v[s0:s1].transpose(0, 1).float()    # [Hk, n, D]
        if pk is not None:
            kk = torch.cat([pk[b].to(kk.device).float(), kk], 1)
            vv = torch.cat([pv[b].to(vv.device).float(), vv], 1)
        L_ = kk.shape[1]
        P = L_ - n
        qq = q[s0:s1].transpose(0, 1).float().view(Hk, H // Hk, n, D)
        sc = torch.einsum("kgnd,kld->kgnl", qq, kk) / math.sqrt(D)
        if mask is not None:
            sc = sc + mask[b, 0, :n, :L_].float().to(sc.device)
        else:
            keep = torch.arange(L_, device=sc.device)[None] <= (torch.arange(n, device=sc.device)[:, None] + P)
            sc = sc.masked_fill(~keep, float("-inf"))
        ob = torch.einsum("kgnl,kld->kgnd", torch.softmax(sc, -1), vv).reshape(H, n, D)
        o[s0:s1] = ob.transpose(0, 1).to(o.dtype)
    return o


def _blha_decode_math(q, kc, vc, tables, lens, tmask):
    """Decode attention over the paged cache with an additive [T, 1, 1, L] mask (math path). q [T, H, D]."""
    T, H, D = q.shape
    nb, Hk, bs, _ = kc.shape
    Lmax = tables.shape[1] * bs
    posi = torch.arange(Lmax, device=q.device)
    blk = tables[:, posi // bs]                                         # [T, Lmax]
    kk = kc[blk, :, (posi % bs).view(1, -1)].float()                    # [T, Lmax, Hk, D]
    vv = vc[blk, :, (posi % bs).view(1, -1)].float()
    qq = q.float().view(T, Hk, H // Hk, D)
    sc = torch.einsum("tkgd,tlkd->tkgl", qq, kk) / math.sqrt(D)
    m = tmask.float().reshape(T, 1, 1, -1)
    w = min(m.shape[-1], Lmax)
    sc[..., :w] = sc[..., :w] + m[..., :w]
    sc = sc.masked_fill(~(posi.view(1, 1, 1, -1) < lens.view(-1, 1, 1, 1)), float("-inf"))
    return torch.einsum("tkgl,tlkd->tkgd", torch.softmax(sc, -1), vv).reshape(T, H, D).to(q.dtype)


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


def fused_gate_attention(query, key=None, query_weight=None, key_weight=None, value_weight=None, qkv_weight=None,
                         gate_linear_weight=None, gate_linear_bias=None, out_linear_weight=None, out_linear_bias=None,
                         nonbatched_bias=None, attn_mask=None, has_gating=True, merge_qkv=True, use_flash_attn=False):
    """AlphaFold-style gated self / cross attention over MSA rows (reference
    incubate/nn/functional/fused_gate_attention.py:26). query [B, M, R, q_dim]; merge_qkv: qkv_weight
    [3, H, c, q_dim], else key [B, M, K, kv_dim] with query / key / value weights [dim, H, c]. The attention
    runs as one flash-attention launch over the B*M rows with attn_mask [B, M, 1, 1, K] and nonbatched_bias
    [B, 1, H, R, K] folded into one additive mask; gating = sigmoid(query . gate_w + gate_b) multiplies the
    heads' outputs, then out = avg . out_w [H, c, q_dim] + out_b."""
    q_in = _t(query)
    B, M, R, Dq = q_in.shape
    if merge_qkv:
        w = _t(qkv_weight)  # [3, H, c, q_dim]
        H, c = w.shape[1], w.shape[2]
        qkv = torch.matmul(q_in, w.reshape(3 * H * c, Dq).t()).view(B, M, R, 3, H, c)
        q, k, v = qkv[..., 0, :, :], qkv[..., 1, :, :], qkv[..., 2, :, :]
    else:
        kin = _t(key)
        wq, wk, wv = _t(query_weight), _t(key_weight), _t(value_weight)
        H, c = wq.shape[1], wq.shape[2]
        q = torch.matmul(q_in, wq.reshape(Dq, H * c)).view(B, M, R, H, c)
        k = torch.matmul(kin, wk.reshape(kin.shape[-1], H * c)).view(B, M, kin.shape[2], H, c)
        v = torch.matmul(kin, wv.reshape(kin.shape[-1], H * c)).view(B, M, kin.shape[2], H, c)
    K = k.shape[2]
    bias = None
    if attn_mask is not None:
        bias = _t(attn_mask).to(q.dtype).reshape(B, M, 1, 1, K)
    if nonbatched_bias is not None:
        nb = _t(nonbatched_bias).to(q.dtype).reshape(B, 1, H, R, K)
        bias = nb if bias is None else bias + nb
    if bias is not None:
        bias = bias.expand(B, M, H, R, K).reshape(B * M, H, R, K)
    o = _ops.flash_attention(q.reshape(B * M, R, H, c), k.reshape(B * M, K, H, c), v.reshape(B * M, K, H, c),
                             causal=False, scale=c ** -0.5, mask=bias, training=False)
    o = o.reshape(B, M, R, H, c)
    if has_gating:
        gw = _t(gate_linear_weight)  # [q_dim, H, c]
        g = torch.matmul(q_in, gw.reshape(Dq, H * c)).view(B, M, R, H, c)
        if gate_linear_bias is not None:
            g = g + _t(gate_linear_bias)
        o = o * torch.sigmoid(g)
    ow = _t(out_linear_weight)  # [H, c, q_dim]
    out = torch.matmul(o.reshape(B, M, R, H * c), ow.reshape(H * c, ow.shape[-1]))
    if out_linear_bias is not None:
        out = out + _t(out_linear_bias)
    return _wrap(out)
