"""HIP flash attention with its optional terms, each against an fp32 PyTorch reference of the same op:
dense bool / additive masks, flashmask row bounds, in-kernel dropout (keep mask recovered exactly), varlen
batches from device cu_seqlens, GQA with in-kernel dK / dV group sums, head dims 32..256, fp16.
Every test asserts the HIP launchers ran and the ATen SDPA fallback did not."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from paddlepaddle_amd.ops import _loader as L  # noqa: E402
from paddlepaddle_amd.ops.attention import attention, attention_reference, flashmask_keep  # noqa: E402


def _rand(shape, dt, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randn(shape, device="cuda", dtype=torch.float32, generator=g).to(dt)


def _check(B, Sq, Sk, H, Hk, D, causal=False, mask=None, startend=None, dt=torch.bfloat16, seed=0, tol=3e-2):
    q, k, v = _rand((B, Sq, H, D), dt, seed), _rand((B, Sk, Hk, D), dt, seed + 1), _rand((B, Sk, Hk, D), dt, seed + 2)
    for t in (q, k, v):
        t.requires_grad_(True)
    o = attention(q, k, v, causal=causal, mask=mask, startend_row_indices=startend)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref_mask, ref_causal = mask, causal
    if startend is not None:
        ref_mask, ref_causal = flashmask_keep(startend, Sq, Sk, causal, q.device), False
    orf = attention_reference(qr, kr, vr, causal=ref_causal, mask=ref_mask)
    err = (o.float() - orf).abs().max().item()  # fully masked rows: 0 in both
    assert err < tol, f"fwd max err {err}"
    g = _rand(orf.shape, torch.float32, seed + 3)
    o.backward(g.to(dt))
    orf.backward(g)
    for name, a, b in (("dq", q.grad, qr.grad), ("dk", k.grad, kr.grad), ("dv", v.grad, vr.grad)):
        e = (a.float() - b).abs().max().item() / (b.abs().max().item() + 1e-6)
        assert e < 3e-2, f"{name} rel err {e}"
    assert L.calls("pa_flash_attn_fwd_ex") > 0
    assert L.calls("pa_flash_attn_bwd_ex") + L.calls("pa_flash_attn_bwd_ds") > 0  # the dS route takes the plain cases
    assert L.calls("attn_aten_fallback") == 0


@pytest.mark.parametrize("causal", [False, True])
def test_bool_mask_padding(causal):
    B, S, H = 2, 256, 4
    lens = torch.tensor([200, 137], device="cuda")
    keep = torch.arange(S, device="cuda")[None, None, None, :] < lens[:, None, None, None]  # [B,1,1,Sk]
    _check(B, S, S, H, H, 128, causal=causal, mask=keep)


def test_bool_mask_full_and_ragged_keys():
    torch.manual_seed(1)
    B, Sq, Sk, H = 1, 192, 300, 2
    keep = torch.rand(B, H, Sq, Sk, device="cuda") > 0.3
    keep[..., 0] = True
    _check(B, Sq, Sk, H, H, 64, mask=keep)


@pytest.mark.parametrize("mdt", [torch.bfloat16, torch.float32])
def test_additive_mask(mdt):
    torch.manual_seed(2)
    B, S, H = 2, 256, 4
    bias = (torch.randn(1, H, S, S, device="cuda") * 2).to(mdt)   # ALiBi-like per-head bias
    _check(B, S, S, H, H, 128, causal=True, mask=bias)
    _check(B, S, S, H, 2, 128, mask=bias[0, 0])                       # [Sq, Sk], broadcast over B, H; GQA


@pytest.mark.parametrize("D", [32, 80, 96, 256])
def test_head_dims(D):
    _check(2, 192, 192, 4, 2, D, causal=True)


def test_fp16():
    _check(2, 256, 256, 4, 4, 128, causal=True, dt=torch.float16)
    _check(1, 160, 160, 4, 1, 64, mask=torch.ones(160, 160, dtype=torch.bool, device="cuda").tril(), dt=torch.float16)


def test_gqa_group_sum_in_kernel():
    _check(2, 256, 256, 8, 2, 128, causal=True)
    _check(1, 128, 384, 16, 2, 64, causal=True)


def _doc_bounds(B, Sk, docs):
    """causal document mask: key j of a document ending at row e is masked for rows >= e (LTS = doc end)."""
    lts = torch.empty(Sk, dtype=torch.int32)
    s = 0
    for n in docs:
        lts[s:s + n] = s + n
        s += n
    return lts.view(1, 1, Sk, 1).expand(B, 1, Sk, 1).contiguous().cuda()


def test_flashmask_causal_documents():
    _check(2, 384, 384, 4, 4, 128, causal=True, startend=_doc_bounds(2, 384, [100, 200, 84]))


def test_flashmask_two_and_four_columns():
    torch.manual_seed(5)
    B, S, H = 1, 256, 2
    a = torch.randint(0, S, (B, H, S, 1), dtype=torch.int32)
    b = torch.randint(0, S, (B, H, S, 1), dtype=torch.int32)
    lo, hi = torch.minimum(a, b), torch.maximum(a, b)
    _check(B, S, S, H, H, 64, causal=True, startend=torch.cat([lo, hi], -1).cuda())              # LTS, LTE
    ute = torch.randint(0, S // 4, (B, H, S, 1), dtype=torch.int32)
    lts = torch.randint(S // 2, S + 1, (B, H, S, 1), dtype=torch.int32)
    _check(B, S, S, H, H, 64, causal=False, startend=torch.cat([lts, ute], -1).cuda())           # LTS, UTE
    four = torch.cat([lo, hi, torch.zeros_like(lo), ute], -1).cuda()
    _check(B, S, S, H, H, 128, causal=False, startend=four)


def test_dropout_keep_mask_recovered_exactly():
    """V = identity rows makes O = P' (the dropped, rescaled probabilities): the kernel's keep mask is read off
    the output, checked against the reference softmax and reused in the reference backward."""
    B, Sq, Sk, H, D, p = 2, 128, 64, 4, 64, 0.3
    q, k = _rand((B, Sq, H, D), torch.bfloat16, 11), _rand((B, Sk, H, D), torch.bfloat16, 12)
    v = torch.eye(D, device="cuda", dtype=torch.bfloat16)[:Sk].view(1, Sk, 1, D).expand(B, Sk, H, D).contiguous()
    o1 = attention(q, k, v, dropout=p, seed=1234)
    o2 = attention(q, k, v, dropout=p, seed=1234)
    assert torch.equal(o1, o2), "same seed must give the same mask"
    keep = (o1.float() != 0).permute(0, 2, 1, 3)[..., :Sk]          # [B, H, Sq, Sk]
    frac = keep.float().mean().item()
    assert abs(frac - (1 - p)) < 0.02, frac
    pr = torch.softmax(torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) / math.sqrt(D), -1)
    want = (pr * keep / (1 - p)).permute(0, 2, 1, 3)
    torch.testing.assert_close(o1.float()[..., :Sk], want, atol=2e-2, rtol=2e-2)
    # backward against the reference with the same keep mask (random V now)
    v2 = _rand((B, Sk, H, D), torch.bfloat16, 13)
    qq, kk, vv = (t.clone().requires_grad_(True) for t in (q, k, v2))
    o = attention(qq, kk, vv, dropout=p, seed=1234)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v2))
    orf = attention_reference(qr, kr, vr, dropout=p, keep=keep)
    assert (o.float() - orf).abs().max().item() < 4e-2
    g = _rand(orf.shape, torch.float32, 14)
    o.backward(g.bfloat16())
    orf.backward(g)
    for a, b in ((qq.grad, qr.grad), (kk.grad, kr.grad), (vv.grad, vr.grad)):
        assert (a.float() - b).abs().max().item() / (b.abs().max().item() + 1e-6) < 3e-2
    assert L.calls("attn_aten_fallback") == 0


@pytest.mark.parametrize("causal", [False, True])
def test_varlen_matches_per_sequence(causal):
    lens_q = [100, 256, 64, 1]
    lens_k = [100, 256, 64, 1] if causal else [120, 200, 64, 30]
    H, Hk, D = 4, 2, 128
    cq = torch.tensor([0] + list(torch.tensor(lens_q).cumsum(0)), dtype=torch.int32, device="cuda")
    ck = torch.tensor([0] + list(torch.tensor(lens_k).cumsum(0)), dtype=torch.int32, device="cuda")
    q = _rand((int(cq[-1]), H, D), torch.bfloat16, 21).requires_grad_(True)
    k = _rand((int(ck[-1]), Hk, D), torch.bfloat16, 22).requires_grad_(True)
    v = _rand((int(ck[-1]), Hk, D), torch.bfloat16, 23).requires_grad_(True)
    o, lse = attention(q, k, v, causal=causal, cu_seqlens_q=cq, cu_seqlens_k=ck, max_seqlen_q=max(lens_q),
                       max_seqlen_k=max(lens_k), return_lse=True)
    g = _rand(o.shape, torch.float32, 24)
    o.backward(g.bfloat16())
    for i in range(len(lens_q)):
        a, b, c, d = int(cq[i]), int(cq[i + 1]), int(ck[i]), int(ck[i + 1])
        qr, kr, vr = (t.detach()[s:e].float()[None].requires_grad_(True) for t, s, e in ((q, a, b), (k, c, d), (v, c, d)))
        orf = attention_reference(qr, kr, vr, causal=causal)
        assert (o[a:b].float() - orf[0]).abs().max().item() < 3e-2
        orf.backward(g[a:b][None])
        for got, ref in ((q.grad[a:b], qr.grad[0]), (k.grad[c:d], kr.grad[0]), (v.grad[c:d], vr.grad[0])):
            # (a 1-token sequence has dK = 0 exactly; bf16 rounding leaves ~1e-3 there)
            assert (got.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-1) < 3e-2
    assert lse.shape == (H, int(cq[-1]))
    assert L.calls("pa_flash_attn_fwd_ex") > 0 and L.calls("attn_aten_fallback") == 0


def test_varlen_graph_capturable():
    """No host sync in the varlen path: it captures into a hipGraph and replays."""
    H, D = 2, 64
    cu = torch.tensor([0, 50, 178], dtype=torch.int32, device="cuda")
    q = _rand((178, H, D), torch.bfloat16, 31)
    out = attention(q, q, q, cu_seqlens_q=cu, cu_seqlens_k=cu, max_seqlen_q=128, max_seqlen_k=128)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph):
            o_g = attention(q, q, q, cu_seqlens_q=cu, cu_seqlens_k=cu, max_seqlen_q=128, max_seqlen_k=128)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(o_g, out)


def test_paddle_api_routes_to_kernel():
    import paddlepaddle_amd as paddle
    F = paddle.nn.functional
    L.reset_calls()
    x = paddle.Tensor(_rand((2, 128, 4, 64), torch.bfloat16, 41))
    m = paddle.Tensor(torch.ones(2, 1, 128, 128, dtype=torch.bool, device="cuda").tril())
    F.scaled_dot_product_attention(x, x, x, attn_mask=m)
    F.flashmask_attention(x, x, x, paddle.Tensor(_doc_bounds(2, 128, [64, 64])), causal=True)
    cu = paddle.Tensor(torch.tensor([0, 100, 256], dtype=torch.int32, device="cuda"))
    F.flash_attn_unpadded(paddle.Tensor(x._t.reshape(256, 4, 64)), paddle.Tensor(x._t.reshape(256, 4, 64)),
                          paddle.Tensor(x._t.reshape(256, 4, 64)), cu, cu, 156, 156, 0.125)
    assert L.calls("pa_flash_attn_fwd_ex") == 3 and L.calls("attn_aten_fallback") == 0
