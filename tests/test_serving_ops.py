"""Serving ops against plain fp32 math: fused_multi_transformer (no cache / prefill into cache_kvs /
decode at time_step, GQA, rotary, rmsnorm), variable_length_memory_efficient_attention (device-side
length masking) and block_multihead_attention (mixed prefill + decode batch over a paged cache, with and
without the host max-length hints). GPU tests run the bf16 HIP paths (varlen flash attention, paged /
dense flash-decoding) and replay a captured decode step with new lengths.

Reference semantics: python/paddle/incubate/nn/functional/fused_transformer.py:1015 (fused_multi_transformer),
block_multihead_attention.py:33, variable_length_memory_efficient_attention.py:33."""
import math

import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle
import paddlepaddle_amd.incubate.nn.functional as IF


def _T(a, dev="cpu", dt=torch.float32):
    return paddle.to_tensor(torch.as_tensor(a).to(dev, dt))


# ------------------------------------------------------------------------------------ references
def _rot(x, cos, sin):
    """x [..., D] interleaved-pair rotation (use_neox_rotary_style=False)."""
    x1, x2 = x[..., 0::2], x[..., 1::2]
    r = torch.stack([-x2, x1], -1).flatten(-2)
    return x * cos + r * sin


def _ref_attention(q, k, v, mask):
    """q [B,S,H,D], k/v [B,L,Hk,D] fp32; mask additive [B,1,S,L] or None."""
    H, Hk = q.shape[2], k.shape[2]
    k = k.repeat_interleave(H // Hk, 2)
    v = v.repeat_interleave(H // Hk, 2)
    s = torch.einsum("bshd,blhd->bhsl", q, k) / math.sqrt(q.shape[-1])
    if mask is not None:
        s = s + mask
    return torch.einsum("bhsl,blhd->bshd", torch.softmax(s, -1), v)


def _ref_stack(x, P, mask, H, Hk, rot=None, norm="layernorm", eps=1e-5):
    """Pre-LN decoder stack over all positions of x [B,S,E] (fp32), relu FFN."""
    B, S, E = x.shape
    Dh = E // H

    def nrm(t, w, b):
        if norm == "rmsnorm":
            return t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True) + eps) * w
        return torch.nn.functional.layer_norm(t, (E,), w, b, eps)
    h = x
    for p in P:
        t = nrm(h, p["ln_s"], p["ln_b"])
        qkv = t @ p["qkv_w"].reshape(-1, E).t() + p["qkv_b"].reshape(-1)
        qkv = qkv.view(B, S, H + 2 * Hk, Dh)
        q, k, v = qkv[:, :, :H], qkv[:, :, H:H + Hk], qkv[:, :, H + Hk:]
        if rot is not None:
            cos, sin = rot[0][:, :S][:, :, None], rot[1][:, :S][:, :, None]
            q, k = _rot(q, cos, sin), _rot(k, cos, sin)
        o = _ref_attention(q, k, v, mask).reshape(B, S, H * Dh)
        h = h + o @ p["lin_w"] + p["lin_b"]
        t = nrm(h, p["ffn_ln_s"], p["ffn_ln_b"])
        h = h + torch.relu(t @ p["ffn1_w"] + p["ffn1_b"]) @ p["ffn2_w"] + p["ffn2_b"]
    return h


def _params(nl, E, H, Hk, F, gen, gqa):
    P = []
    for _ in range(nl):
        heads = (H + 2 * Hk)
        P.append({
            "ln_s": 1 + 0.1 * torch.randn(E, generator=gen), "ln_b": 0.1 * torch.randn(E, generator=gen),
            "qkv_w": torch.randn((heads, E // H, E) if gqa else (3, H, E // H, E), generator=gen) / math.sqrt(E),
            "qkv_b": 0.1 * torch.randn((heads, E // H) if gqa else (3, H, E // H), generator=gen),
            "lin_w": torch.randn(E, E, generator=gen) / math.sqrt(E), "lin_b": 0.1 * torch.randn(E, generator=gen),
            "ffn_ln_s": 1 + 0.1 * torch.randn(E, generator=gen), "ffn_ln_b": 0.1 * torch.randn(E, generator=gen),
            "ffn1_w": torch.randn(E, F, generator=gen) / math.sqrt(E), "ffn1_b": 0.1 * torch.randn(F, generator=gen),
            "ffn2_w": torch.randn(F, E, generator=gen) / math.sqrt(F), "ffn2_b": 0.1 * torch.randn(E, generator=gen),
        })
    return P


def _fmt(x, P, dev, dt, **kw):
    g = lambda k: [_T(p[k], dev, dt) for p in P]  # noqa: E731
    return IF.fused_multi_transformer(
        x, g("ln_s"), g("ln_b"), g("qkv_w"), g("qkv_b"), g("lin_w"), g("lin_b"), g("ffn_ln_s"), g("ffn_ln_b"),
        g("ffn1_w"), g("ffn1_b"), g("ffn2_w"), g("ffn2_b"), activation="relu", **kw)


def _causal(B, S, L, off, dev):
    keep = torch.arange(L, device=dev)[None] <= (torch.arange(S, device=dev)[:, None] + off)
    return torch.zeros(B, 1, S, L, device=dev).masked_fill(~keep, float("-inf"))


def _run_fmt_prefill_decode(dev, dt, E, H, Hk, norm="layernorm", rotary=False, tol=1e-4):
    gen = torch.Generator().manual_seed(0)
    B, S, steps, Lmax, F = 2, 5, 3, 16, 2 * E
    gqa = Hk != H
    P = _params(2, E, H, Hk, F, gen, gqa)
    xs = torch.randn(B, S + steps, E, generator=gen)
    Dh = E // H
    rot = None
    kw = {}
    if rotary:
        pos = torch.arange(Lmax)[:, None].float()
        inv = 1.0 / (10000 ** (torch.arange(0, Dh, 2).float() / Dh))
        ang = (pos * inv).repeat_interleave(2, -1)  # interleaved pairs share an angle
        rot = (ang.cos()[None].expand(B, -1, -1), ang.sin()[None].expand(B, -1, -1))
        kw = dict(rotary_embs=_T(torch.stack([rot[0], rot[1]])[:, :, None], dev, torch.float32), rotary_emb_dims=1)
    if gqa:
        kw["gqa_group_size"] = Hk
    full = _ref_stack(xs, P, _causal(B, S + steps, S + steps, 0, "cpu"), H, Hk, rot, norm)
    caches = [paddle.to_tensor(torch.zeros(2, B, Hk, Lmax, Dh, device=dev, dtype=dt)) for _ in P]
    out, caches = _fmt(_T(xs[:, :S], dev, dt), P, dev, dt, cache_kvs=caches,
                       attn_mask=_T(_causal(B, S, S, 0, "cpu"), dev, dt), norm_type=norm, **kw)
    got = out._t.float().cpu()
    np.testing.assert_allclose(got.numpy(), full[:, :S].numpy(), rtol=tol, atol=tol)
    for t in range(steps):
        step = S + t
        out, caches = _fmt(_T(xs[:, step:step + 1], dev, dt), P, dev, dt, cache_kvs=caches,
                           time_step=paddle.to_tensor(np.array([step], "int32")), norm_type=norm, **kw)
        np.testing.assert_allclose(out._t.float().cpu().numpy(), full[:, step:step + 1].numpy(), rtol=tol,
                                   atol=tol)


def test_fused_multi_transformer_no_cache_matches_math():
    gen = torch.Generator().manual_seed(1)
    B, S, E, H = 2, 6, 32, 4
    P = _params(2, E, H, H, 64, gen, False)
    x = torch.randn(B, S, E, generator=gen)
    mask = torch.randn(B, 1, S, S, generator=gen)
    out = _fmt(_T(x), P, "cpu", torch.float32, attn_mask=_T(mask))
    np.testing.assert_allclose(out.numpy(), _ref_stack(x, P, mask, H, H).numpy(), rtol=1e-4, atol=1e-4)


def test_fused_multi_transformer_prefill_then_decode_cpu():
    _run_fmt_prefill_decode("cpu", torch.float32, 32, 4, 4)


def test_fused_multi_transformer_gqa_rotary_rmsnorm_cpu():
    _run_fmt_prefill_decode("cpu", torch.float32, 32, 4, 2, norm="rmsnorm", rotary=True)


def test_fused_multi_transformer_beam_offset_equals_reordered_cache():
    """beam_offset indirection == physically copying each position from the parent beam's cache row."""
    gen = torch.Generator().manual_seed(3)
    bsz, W, E, H, Lmax, step = 2, 2, 32, 4, 8, 4
    B, Dh = bsz * W, E // H
    P = _params(2, E, H, H, 64, gen, False)
    x = torch.randn(B, 1, E, generator=gen)
    base = [torch.randn(2, B, H, Lmax, Dh, generator=gen) for _ in P]
    off = torch.randint(0, W, (bsz, W, Lmax), generator=gen).int()
    ts = paddle.to_tensor(np.array([step], "int32"))
    out_b, _ = _fmt(_T(x), P, "cpu", torch.float32, cache_kvs=[paddle.to_tensor(c.clone()) for c in base],
                    time_step=ts, beam_offset=paddle.to_tensor(off))
    phys = []
    for c in base:
        r = c.clone()
        for b in range(B):
            for t in range(step):
                o = int(off[b // W, b % W, t])
                if o:
                    r[:, b, :, t] = c[:, (b // W) * W + o, :, t]
        phys.append(paddle.to_tensor(r))
    out_p, _ = _fmt(_T(x), P, "cpu", torch.float32, cache_kvs=phys, time_step=ts)
    np.testing.assert_allclose(out_b.numpy(), out_p.numpy(), rtol=1e-4, atol=1e-4)


def test_fused_multi_transformer_downscale_in_infer_mode():
    """mode='downscale_in_infer': inference scales the dropped branches by (1 - p); training keeps them unscaled
    where kept (reference fused_transformer.py dropout modes)."""
    gen = torch.Generator().manual_seed(2)
    B, S, E, H = 2, 4, 32, 4
    P = _params(1, E, H, H, 64, gen, False)
    x = torch.randn(B, S, E, generator=gen)
    base = _fmt(_T(x), P, "cpu", torch.float32, attn_mask=_T(torch.zeros(B, 1, S, S)))
    scaled = _fmt(_T(x), P, "cpu", torch.float32, attn_mask=_T(torch.zeros(B, 1, S, S)), dropout_rate=0.25,
                  mode="downscale_in_infer", training=False)
    assert not np.allclose(base.numpy(), scaled.numpy())
    P2 = [dict(p, lin_w=p["lin_w"] * 0.75, lin_b=p["lin_b"] * 0.75, ffn2_w=p["ffn2_w"] * 0.75,
               ffn2_b=p["ffn2_b"] * 0.75) for p in P]  # (1 - p) on both dropped branches
    np.testing.assert_allclose(scaled.numpy(), _ref_stack(x, P2, torch.zeros(B, 1, S, S), H, H).numpy(), rtol=1e-4,
                               atol=1e-4)
    out = _fmt(_T(x), P, "cpu", torch.float32, attn_mask=_T(torch.zeros(B, 1, S, S)), dropout_rate=0.25,
               mode="downscale_in_infer", training=True)
    assert np.isfinite(out.numpy()).all()
    with pytest.raises(ValueError):
        _fmt(_T(x), P, "cpu", torch.float32, dropout_rate=0.25, mode="bogus")


def test_fused_multi_transformer_layer_returns_caches():
    m = paddle.incubate.nn.FusedMultiTransformer(32, 4, 64, num_layers=2)
    m.eval()
    x = paddle.randn([2, 3, 32])
    caches = [paddle.zeros([2, 2, 4, 8, 8]) for _ in range(2)]
    out, c2 = m(x, caches=caches)
    assert out.shape == [2, 3, 32] and c2 is caches
    assert float(caches[0]._t[:, :, :, :3].abs().sum()) > 0 and float(caches[0]._t[:, :, :, 3:].abs().sum()) == 0


def _ref_varlen(q, k, v, sl, kl, mask, causal, pre):
    B, H, Sq, D = q.shape
    out = torch.zeros_like(q)
    for b in range(B):
        n, nk = int(sl[b]), int(kl[b]) + pre
        if n == 0:
            continue
        s = torch.einsum("hqd,hkd->hqk", q[b, :, :n], k[b, :, :nk]) / math.sqrt(D)
        if mask is not None:
            s = s + mask[b, :, :n, :nk]
        if causal:
            keep = torch.arange(nk)[None] <= torch.arange(n)[:, None] + pre
            s = s.masked_fill(~keep, float("-inf"))
        out[b, :, :n] = torch.einsum("hqk,hkd->hqd", torch.softmax(s, -1), v[b, :, :nk])
    return out


@pytest.mark.parametrize("causal,with_mask,pre", [(False, False, 0), (True, False, 0), (True, True, 2)])
def test_variable_length_attention_cpu(causal, with_mask, pre):
    gen = torch.Generator().manual_seed(2)
    B, H, S, D = 3, 2, 7, 16
    q, k, v = (torch.randn(B, H, S, D, generator=gen) for _ in range(3))
    sl, kl = torch.tensor([7, 4, 1]), torch.tensor([5, 4, 1])
    mask = torch.randn(B, 1, S, S, generator=gen) if with_mask else None
    out = IF.variable_length_memory_efficient_attention(
        _T(q), _T(k), _T(v), _T(sl, dt=torch.int32), _T(kl, dt=torch.int32),
        mask=None if mask is None else _T(mask), causal=causal, pre_cache_length=pre)
    np.testing.assert_allclose(out.numpy(), _ref_varlen(q, k, v, sl, kl, mask, causal, pre).numpy(),
                               rtol=1e-4, atol=1e-5)


def _blha_case(dev, dt, H, Hk, D, hints):
    """Step 1: sequences 0 and 1 prefill (5 and 3 tokens). Step 2 (mixed): sequence 0 decodes one token,
    sequence 1 decodes one token, sequence 2 prefills 4 tokens. Every output row is checked against
    causal attention over that sequence's whole history."""
    gen = torch.Generator().manual_seed(3)
    bs, nblocks = 4, 12
    kc = torch.zeros(nblocks, Hk, bs, D, device=dev, dtype=dt)
    vc = torch.zeros_like(kc)
    tables = torch.tensor([[0, 1, 2], [3, 4, 5], [6, 7, 8]], dtype=torch.int32)
    W = (H + 2 * Hk) * D
    hist = {0: [], 1: [], 2: []}

    def call(per_seq):  # per_seq: [(enc, dec, tokens [n, W])]
        toks = torch.cat([t for _, _, t in per_seq])
        lens = [t.shape[0] for _, _, t in per_seq]
        cu = torch.tensor(np.concatenate([[0], np.cumsum(lens)]), dtype=torch.int32)
        enc = torch.tensor([e for e, _, _ in per_seq], dtype=torch.int32)
        dec = torch.tensor([d for _, d, _ in per_seq], dtype=torch.int32)
        extra = {}
        if hints:
            extra = dict(max_enc_len_this_time=paddle.to_tensor(np.array([int(enc.max())], "int32"),
                                                                place=paddle.CPUPlace()),
                         max_dec_len_this_time=paddle.to_tensor(np.array([int(dec.max())], "int32"),
                                                                place=paddle.CPUPlace()))
        out, _, _, _ = IF.block_multihead_attention(
            _T(toks, dev, dt), paddle.to_tensor(kc), paddle.to_tensor(vc), _T(enc, dev, torch.int32),
            _T(dec, dev, torch.int32), _T(torch.tensor(lens), dev, torch.int32), None, None,
            _T(cu, dev, torch.int32), _T(cu, dev, torch.int32), _T(tables[:len(per_seq)], dev, torch.int32),
            block_size=bs, **extra)
        return out._t.float().cpu()

    def check(out, per_seq, tol):
        r = 0
        for b, (_, _, t) in enumerate(per_seq):
            hist[b].append(t)
            full = torch.cat(hist[b]).view(-1, H + 2 * Hk, D).float()
            n = t.shape[0]
            q, k, v = full[-n:, :H][None], full[:, H:H + Hk][None], full[:, H + Hk:][None]
            Ltot = full.shape[0]
            ref = _ref_attention(q, k, v, _causal(1, n, Ltot, Ltot - n, "cpu"))[0].reshape(n, H * D)
            np.testing.assert_allclose(out[r:r + n].numpy(), ref.numpy(), rtol=tol, atol=tol)
            r += n

    tol = 1e-4 if dt == torch.float32 else 3e-2
    rnd = lambda n: (torch.randn(n, W, generator=gen) * 0.5).to(dt).float()  # noqa: E731
    s1 = [(5, 0, rnd(5)), (3, 0, rnd(3))]
    check(call(s1), s1, tol)
    s2 = [(0, 5, rnd(1)), (0, 3, rnd(1)), (4, 0, rnd(4))]
    check(call(s2), s2, tol)
    return kc


@pytest.mark.parametrize("hints", [False, True])
def test_block_mha_mixed_prefill_decode_cpu(hints):
    _blha_case("cpu", torch.float32, 4, 2, 16, hints)


def test_block_mha_rejects_unsupported_args():
    z = paddle.zeros([1], dtype="int32")
    with pytest.raises(ValueError):
        IF.block_multihead_attention(paddle.zeros([1, 48]), paddle.zeros([2, 1, 4, 16]), paddle.zeros([2, 1, 4, 16]),
                                     z, z, z + 1, None, None, paddle.to_tensor(np.array([0, 1], "int32")),
                                     paddle.to_tensor(np.array([0, 1], "int32")), paddle.zeros([1, 2], "int32"),
                                     pre_key_cache=paddle.zeros([1, 1, 2, 16]))  # without pre_value_cache
    with pytest.raises(ValueError):
        IF.block_multihead_attention(paddle.zeros([1, 48]), paddle.zeros([2, 1, 4, 16], "uint8"),
                                     paddle.zeros([2, 1, 4, 16], "uint8"), z, z, z + 1, None, None,
                                     paddle.to_tensor(np.array([0, 1], "int32")),
                                     paddle.to_tensor(np.array([0, 1], "int32")), paddle.zeros([1, 2], "int32"),
                                     cache_k_quant_scales=paddle.ones([1]), use_dynamic_cachekv_quant=True)


@pytest.mark.parametrize("use_mask", [False, True])
def test_block_mha_prefix_cache_and_masks(use_mask):
    """pre_key_cache / pre_value_cache: the prefilling sequence's cache positions 0..P-1 hold the prefix and its
    tokens attend to prefix + causal tokens (or through an additive mask that says the same); a decode step then
    attends over prefix + history (+ tgt_mask). Checked against explicit attention."""
    gen = torch.Generator().manual_seed(13)
    H, Hk, D, bs, P, n = 4, 2, 16, 4, 3, 5
    W = (H + 2 * Hk) * D
    kc = torch.zeros(4, Hk, bs, D)
    vc = torch.zeros_like(kc)
    pk, pv = torch.randn(1, Hk, P, D, generator=gen), torch.randn(1, Hk, P, D, generator=gen)
    tables = torch.tensor([[0, 1, 2, 3]], dtype=torch.int32)
    Pt = paddle.to_tensor

    def ref(xs, q_rows):
        full = xs.view(-1, H + 2 * Hk, D)
        kk = torch.cat([pk[0].transpose(0, 1), full[:, H:H + Hk]], 0)          # [P + L, Hk, D]
        vv = torch.cat([pv[0].transpose(0, 1), full[:, H + Hk:]], 0)
        q = full[q_rows, :H]                                                   # [m, H, D]
        Ltot = kk.shape[0]
        out = []
        for i, r in enumerate(q_rows):
            sc = torch.einsum("hd,lhd->hl", q[i], kk.repeat_interleave(H // Hk, 1)) / D ** 0.5
            sc[:, P + r + 1:] = float("-inf")
            out.append(torch.einsum("hl,lhd->hd", torch.softmax(sc, -1), vv.repeat_interleave(H // Hk, 1)))
        return torch.stack(out).reshape(len(q_rows), H * D)

    x1 = torch.randn(n, W, generator=gen) * 0.5
    mask = None
    if use_mask:
        keep = torch.arange(P + n)[None] <= (torch.arange(n)[:, None] + P)
        mask = Pt(torch.zeros(1, 1, n, P + n).masked_fill(~keep, -1e4))
    cu = torch.tensor([0, n], dtype=torch.int32)
    out, _, _, _ = IF.block_multihead_attention(
        Pt(x1), Pt(kc), Pt(vc), Pt(torch.tensor([n], dtype=torch.int32)), Pt(torch.tensor([0], dtype=torch.int32)),
        Pt(torch.tensor([n], dtype=torch.int32)), None, None, Pt(cu), Pt(cu), Pt(tables), pre_key_cache=Pt(pk),
        pre_value_cache=Pt(pv), mask=mask, block_size=bs)
    np.testing.assert_allclose(out.numpy(), ref(x1, list(range(n))).numpy(), rtol=1e-4, atol=1e-4)
    # the prefix sits at cache positions 0..P-1
    np.testing.assert_allclose(kc[0, :, :P].numpy(), pk[0].numpy(), rtol=0, atol=0)
    # decode one token at position P + n (dec = n: tokens so far, the prefix offset is added inside)
    x2 = torch.randn(1, W, generator=gen) * 0.5
    tgt = Pt(torch.zeros(1, 1, 1, 16)) if use_mask else None
    cu1 = torch.tensor([0, 1], dtype=torch.int32)
    hints = dict(max_enc_len_this_time=paddle.to_tensor(np.array([0], "int32"), place=paddle.CPUPlace()),
                 max_dec_len_this_time=paddle.to_tensor(np.array([n], "int32"), place=paddle.CPUPlace()))
    out2, _, _, _ = IF.block_multihead_attention(
        Pt(x2), Pt(kc), Pt(vc), Pt(torch.tensor([0], dtype=torch.int32)), Pt(torch.tensor([n], dtype=torch.int32)),
        Pt(torch.tensor([1], dtype=torch.int32)), None, None, Pt(cu1), Pt(cu1), Pt(tables), pre_key_cache=Pt(pk),
        pre_value_cache=Pt(pv), tgt_mask=tgt, block_size=bs, **hints)
    np.testing.assert_allclose(out2.numpy(), ref(torch.cat([x1, x2]), [n]).numpy(), rtol=1e-4, atol=1e-4)


def test_block_mha_dynamic_int8_cache():
    """use_dynamic_cachekv_quant: the prefill step sets scale = 127 / max|k| per kv head (over the step's tokens)
    in the [batch, kv_heads] scale rows, stores round(scale * k) + 128, and the decode step reads the cache with
    row 0's dequant scales (reference quant_write_cache_int8_kernel / blha)."""
    gen = torch.Generator().manual_seed(5)
    H, Hk, D, bs = 4, 2, 16, 4
    W = (H + 2 * Hk) * D
    kq = torch.zeros(3, Hk, bs, D, dtype=torch.uint8)
    vq = torch.zeros_like(kq)
    sk, sv, dk, dv = (torch.zeros(1, Hk) for _ in range(4))
    P = paddle.to_tensor
    tables = torch.tensor([[0, 1, 2]], dtype=torch.int32)

    def step(x, enc, dec, kc, vc, quant):
        n = x.shape[0]
        cu = torch.tensor([0, n], dtype=torch.int32)
        extra = dict(cache_k_quant_scales=P(sk), cache_v_quant_scales=P(sv), cache_k_dequant_scales=P(dk),
                     cache_v_dequant_scales=P(dv), use_dynamic_cachekv_quant=True) if quant else {}
        out, _, _, _ = IF.block_multihead_attention(
            P(x), P(kc), P(vc), P(torch.tensor([enc], dtype=torch.int32)), P(torch.tensor([dec], dtype=torch.int32)),
            P(torch.tensor([n], dtype=torch.int32)), None, None, P(cu), P(cu), P(tables), block_size=bs, **extra)
        return out._t

    x1 = torch.randn(5, W, generator=gen)
    step(x1, 5, 0, kq, vq, True)
    k1 = x1.view(5, H + 2 * Hk, D)[:, H:H + Hk]
    amax = k1.abs().amax(dim=(0, 2))
    np.testing.assert_allclose(sk[0].numpy(), (127.0 / amax).numpy(), rtol=1e-6)
    np.testing.assert_allclose(dk[0].numpy(), (amax / 127.0).numpy(), rtol=1e-6)
    z = k1 * sk.view(1, -1, 1)
    exp = (torch.sign(z) * torch.floor(z.abs() + 0.5)).clamp(-127, 127)
    got = kq[torch.tensor([0, 0, 0, 0, 1]), :, torch.tensor([0, 1, 2, 3, 0])].float() - 128
    np.testing.assert_array_equal(got.numpy(), exp.numpy())
    kf = (kq.float() - 128) * dk.view(1, -1, 1, 1)
    vf = (vq.float() - 128) * dv.view(1, -1, 1, 1)
    x2 = torch.randn(1, W, generator=gen)
    o_q = step(x2, 0, 5, kq, vq, True)
    o_f = step(x2, 0, 5, kf, vf, False)
    np.testing.assert_allclose(o_q.numpy(), o_f.numpy(), rtol=1e-5, atol=1e-5)


def test_block_mha_static_int8_cache_and_int8_output():
    _blha_int8("cpu", torch.float32, 16, 1e-5)


@pytest.mark.gpu
def test_block_mha_static_int8_cache_gpu_bf16():
    _blha_int8("cuda", torch.bfloat16, 128, 3e-2)


def _blha_int8(dev, dt, D, tol):
    """uint8 caches with per-kv-head static scales: stored = clip(round(scale * x)) + 128, read back as
    (u - 128) * dequant_scale (reference block_attn.h); a prefill step then a decode step, compared with the same
    steps over float caches holding the dequantised history, and an int8 output for out_scale > 0."""
    gen = torch.Generator().manual_seed(9)
    H, Hk, bs = 4, 2, 4
    W = (H + 2 * Hk) * D
    ksc = torch.tensor([40.0, 60.0])
    vsc = torch.tensor([50.0, 30.0])
    kdq, vdq = 1.0 / ksc, 1.0 / vsc
    tables = torch.tensor([[0, 1, 2]], dtype=torch.int32, device=dev)
    kq = torch.zeros(3, Hk, bs, D, dtype=torch.uint8, device=dev)
    vq = torch.zeros_like(kq)
    kf = torch.zeros(3, Hk, bs, D, device=dev, dtype=dt)
    vf = torch.zeros_like(kf)
    ksc, vsc, kdq, vdq = (t.to(dev) for t in (ksc, vsc, kdq, vdq))
    P = paddle.to_tensor

    def step(x, enc, dec, quant, out_scale=-1):
        n = x.shape[0]
        x = x.to(dev, dt)
        cu = torch.tensor([0, n], dtype=torch.int32, device=dev)
        kc, vc = (kq, vq) if quant else (kf, vf)
        extra = dict(cache_k_quant_scales=P(ksc), cache_v_quant_scales=P(vsc), cache_k_dequant_scales=P(kdq),
                     cache_v_dequant_scales=P(vdq)) if quant else {}
        out, _, _, _ = IF.block_multihead_attention(
            P(x), P(kc), P(vc), P(torch.tensor([enc], dtype=torch.int32, device=dev)),
            P(torch.tensor([dec], dtype=torch.int32, device=dev)), P(torch.tensor([n], dtype=torch.int32, device=dev)),
            None, None, P(cu), P(cu), P(tables), block_size=bs, out_scale=out_scale, **extra)
        return out._t.cpu()

    x1 = (torch.randn(5, W, generator=gen) * 0.5).to(dt)
    o_q = step(x1, 5, 0, True)
    o_f = step(x1, 5, 0, False)
    np.testing.assert_allclose(o_q.float().numpy(), o_f.float().numpy(), rtol=tol, atol=tol)  # prefill: no cache read
    k1 = x1.float().view(5, H + 2 * Hk, D)[:, H:H + Hk]
    ks = ksc.cpu().view(1, -1, 1)
    exp = (torch.sign(k1 * ks) * torch.floor((k1 * ks).abs() + 0.5)).clamp(-127, 127)
    got = kq.cpu().view(-1, Hk, bs, D)[torch.tensor([0, 0, 0, 0, 1]), :, torch.tensor([0, 1, 2, 3, 0])].float() - 128
    np.testing.assert_array_equal(got.numpy(), exp.numpy())
    # float caches holding what the quantised ones hold, then one decode step on each
    kf.copy_((kq.float() - 128) * kdq.view(1, -1, 1, 1))
    vf.copy_((vq.float() - 128) * vdq.view(1, -1, 1, 1))
    x2 = (torch.randn(1, W, generator=gen) * 0.5).to(dt)
    o_q = step(x2, 0, 5, True)
    o_f = step(x2, 0, 5, False)
    np.testing.assert_allclose(o_q.float().numpy(), o_f.float().numpy(), rtol=tol, atol=tol)
    # int8 output
    x3 = (torch.randn(1, W, generator=gen) * 0.5).to(dt)
    o_i8 = step(x3, 0, 6, True, out_scale=0.5)
    assert o_i8.dtype == torch.int8


# ------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_fused_multi_transformer_prefill_decode_gpu_bf16():
    _run_fmt_prefill_decode("cuda", torch.bfloat16, 256, 2, 2, tol=6e-2)
    _run_fmt_prefill_decode("cuda", torch.bfloat16, 512, 4, 2, norm="rmsnorm", rotary=True, tol=6e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("hints", [False, True])
def test_block_mha_mixed_prefill_decode_gpu_bf16(hints):
    _blha_case("cuda", torch.bfloat16, 8, 2, 128, hints)


@pytest.mark.gpu
def test_variable_length_attention_gpu_bf16():
    gen = torch.Generator().manual_seed(4)
    B, H, S, D = 3, 4, 96, 128
    q, k, v = ((torch.randn(B, H, S, D, generator=gen) * 0.5).bfloat16().float() for _ in range(3))
    sl, kl = torch.tensor([96, 40, 1]), torch.tensor([80, 40, 3])
    out = IF.variable_length_memory_efficient_attention(
        _T(q, "cuda", torch.bfloat16), _T(k, "cuda", torch.bfloat16), _T(v, "cuda", torch.bfloat16),
        _T(sl, "cuda", torch.int32), _T(kl, "cuda", torch.int32), causal=True)
    ref = _ref_varlen(q, k, v, sl, kl, None, True, 0)
    np.testing.assert_allclose(out._t.float().cpu().numpy(), ref.numpy(), rtol=3e-2, atol=3e-2)


@pytest.mark.gpu
def test_block_mha_decode_step_graph_replay_gpu():
    """One decode step of 4 sequences captured once, replayed at three later steps with new tokens and
    lengths written into the captured input buffers; each replay matches the fp32 reference."""
    H, Hk, D, bs, B = 8, 2, 128, 64, 4
    W = (H + 2 * Hk) * D
    gen = torch.Generator().manual_seed(5)
    dev = "cuda"
    nblk = 4
    kc = torch.zeros(B * nblk, Hk, bs, D, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    tables = torch.arange(B * nblk, dtype=torch.int32, device=dev).view(B, nblk)
    prompt = [37, 64, 5, 100]
    hist = [(torch.randn(n, W, generator=gen) * 0.5).bfloat16().float() for n in prompt]
    for b in range(B):  # prompts straight into the cache
        full = hist[b].view(-1, H + 2 * Hk, D)
        for p in range(prompt[b]):
            kc[tables[b, p // bs], :, p % bs] = full[p, H:H + Hk].to(dev, torch.bfloat16)
            vc[tables[b, p // bs], :, p % bs] = full[p, H + Hk:].to(dev, torch.bfloat16)
    x = torch.zeros(B, W, device=dev, dtype=torch.bfloat16)
    dec = torch.tensor(prompt, dtype=torch.int32, device=dev)
    zeros = torch.zeros(B, dtype=torch.int32, device=dev)
    ones = torch.ones(B, dtype=torch.int32, device=dev)
    cu = torch.arange(B + 1, dtype=torch.int32, device=dev)
    hint_e = paddle.to_tensor(np.array([0], "int32"), place=paddle.CPUPlace())  # host hints, as blha_get_max_len
    hint_d = paddle.to_tensor(np.array([nblk * bs - 1], "int32"), place=paddle.CPUPlace())
    P = lambda t: paddle.to_tensor(t)  # noqa: E731

    def step():
        return IF.block_multihead_attention(P(x), P(kc), P(vc), P(zeros), P(dec), P(ones), None, None, P(cu), P(cu),
                                            P(tables), block_size=bs, max_enc_len_this_time=hint_e,
                                            max_dec_len_this_time=hint_d)[0]._t
    step()  # warm-up (lazy init) writes a throw-away token at the prompt position, overwritten below
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = step()
    for _ in range(3):
        new = (torch.randn(B, W, generator=gen) * 0.5).bfloat16().float()
        x.copy_(new.to(dev, torch.bfloat16))
        g.replay()
        torch.cuda.synchronize()
        got = out.float().cpu()
        for b in range(B):
            hist[b] = torch.cat([hist[b], new[b:b + 1]])
            full = hist[b].view(-1, H + 2 * Hk, D)
            Ltot = full.shape[0]
            ref = _ref_attention(full[-1:, :H][None], full[:, H:H + Hk][None], full[:, H + Hk:][None], None)
            np.testing.assert_allclose(got[b].numpy(), ref[0, 0].reshape(-1).numpy(), rtol=3e-2, atol=3e-2)
            assert Ltot == int(dec[b]) + 1
        dec += 1


def _ref_gate_attention(q_data, m_data, wq, wk, wv, gw, gb, ow, ob, nb, mask):
    c = wq.shape[-1]
    q = torch.einsum("nbqa,ahc->nbqhc", q_data, wq) * c ** -0.5
    k = torch.einsum("nbka,ahc->nbkhc", m_data, wk)
    v = torch.einsum("nbka,ahc->nbkhc", m_data, wv)
    logits = torch.einsum("nbqhc,nbkhc->nbhqk", q, k) + mask
    if nb is not None:
        logits = logits + nb
    avg = torch.einsum("nbhqk,nbkhc->nbqhc", torch.softmax(logits, -1), v)
    avg = avg * torch.sigmoid(torch.einsum("nbqc,chv->nbqhv", q_data, gw) + gb)
    return torch.einsum("nbqhc,hco->nbqo", avg, ow) + ob


@pytest.mark.parametrize("merge", [True, False])
def test_fused_gate_attention_matches_einsum(merge):
    g = torch.Generator().manual_seed(6)
    B, M, R, Dq, H, c = 2, 3, 5, 16, 4, 8
    r = lambda *s: torch.randn(*s, generator=g) * 0.5  # noqa: E731
    q_data = r(B, M, R, Dq)
    wq, wk, wv = r(Dq, H, c), r(Dq, H, c), r(Dq, H, c)
    gw, gb, ow, ob = r(Dq, H, c), r(H, c), r(H, c, Dq), r(Dq)
    nb, mask = r(B, 1, H, R, R), r(B, M, 1, 1, R)
    ref = _ref_gate_attention(q_data, q_data, wq, wk, wv, gw, gb, ow, ob, nb, mask)
    kw = dict(gate_linear_weight=_T(gw), gate_linear_bias=_T(gb), out_linear_weight=_T(ow), out_linear_bias=_T(ob),
              nonbatched_bias=_T(nb), attn_mask=_T(mask))
    if merge:
        qkv = torch.stack([wq.permute(1, 2, 0), wk.permute(1, 2, 0), wv.permute(1, 2, 0)])  # [3, H, c, q_dim]
        out = IF.fused_gate_attention(_T(q_data), qkv_weight=_T(qkv), merge_qkv=True, **kw)
    else:
        out = IF.fused_gate_attention(_T(q_data), _T(q_data), _T(wq), _T(wk), _T(wv), merge_qkv=False, **kw)
    np.testing.assert_allclose(out.numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)
