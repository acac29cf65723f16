"""HIP flash attention (forward + backward) vs an fp32 PyTorch reference of the same op."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from paddlepaddle_amd import ops  # noqa: E402
from paddlepaddle_amd.ops import _loader as L  # noqa: E402
from paddlepaddle_amd.ops.attention import attention_reference, _FlashAttnHIP  # noqa: E402


def _run(B, Sq, Sk, H, Hk, D, causal, dt=torch.bfloat16, spike=False, seed=0):
    torch.manual_seed(seed)
    q = torch.randn(B, Sq, H, D, device="cuda", dtype=dt)
    k = torch.randn(B, Sk, Hk, D, device="cuda", dtype=dt)
    v = torch.randn(B, Sk, Hk, D, device="cuda", dtype=dt)
    if spike:  # force the running max to jump mid-sequence (online-softmax rescale path)
        k[:, Sk // 2 + 3] *= 8
        q[:, Sq - 1] *= 4
    q.requires_grad_(True), k.requires_grad_(True), v.requires_grad_(True)
    o = ops.flash_attention(q, k, v, causal=causal)
    assert L._LIB is not None and L.has("pa_flash_attn_fwd_ex")
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    orf = attention_reference(qr, kr, vr, causal=causal)
    err = (o.float() - orf).abs().max().item()
    assert err < 3e-2, f"fwd max err {err}"
    g = torch.randn_like(orf)
    o.backward(g.to(dt))
    orf.backward(g)
    for name, a, b in (("dq", q.grad, qr.grad), ("dk", k.grad, kr.grad), ("dv", v.grad, vr.grad)):
        scale = b.abs().max().item() + 1e-6
        e = (a.float() - b).abs().max().item() / scale
        assert e < 2.5e-2, f"{name} rel err {e}"
    assert L.calls("pa_flash_attn_fwd_ex") > 0
    assert L.calls("pa_flash_attn_bwd_ex") + L.calls("pa_flash_attn_bwd_ds") > 0
    assert L.calls("attn_aten_fallback") == 0


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("D", [64, 128])
def test_fa_basic(causal, D):
    _run(2, 256, 256, 4, 4, D, causal)


@pytest.mark.parametrize("causal", [False, True])
def test_fa_ragged_seq(causal):
    _run(1, 300, 300, 2, 2, 128, causal)


def test_fa_gqa():
    _run(2, 192, 192, 8, 2, 128, True)


def test_fa_cross_len_causal_bottom_right():
    _run(1, 128, 320, 2, 2, 128, True)


def test_fa_online_softmax_rescale():
    _run(1, 512, 512, 2, 2, 128, False, spike=True)
    _run(1, 512, 512, 2, 2, 128, True, spike=True, seed=3)


def test_fa_qkvpacked_matches_unpacked():
    torch.manual_seed(7)
    B, S, H, D = 2, 256, 4, 128
    qkv = torch.randn(B, S, H, 3, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    o = ops.flash_attention_qkvpacked(qkv, causal=True)
    q, k, v = (qkv.detach().float()[:, :, :, i].requires_grad_(True) for i in range(3))
    orf = attention_reference(q, k, v, causal=True)
    assert (o.float() - orf).abs().max().item() < 3e-2
    g = torch.randn_like(orf)
    o.backward(g.bfloat16())
    orf.backward(g)
    for i, ref in enumerate((q.grad, k.grad, v.grad)):
        e = (qkv.grad[:, :, :, i].float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
        assert e < 2.5e-2


def test_fa_lse_matches_logsumexp():
    from paddlepaddle_amd.ops.attention import attention
    torch.manual_seed(2)
    B, S, H, D = 1, 200, 2, 128
    q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    o, lse = attention(q, k, v, causal=True, return_lse=True)
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) / math.sqrt(D)
    s = s.masked_fill(~torch.ones(S, S, dtype=torch.bool, device="cuda").tril(), float("-inf"))
    ref = torch.logsumexp(s, -1)
    torch.testing.assert_close(lse, ref, atol=2e-2, rtol=1e-3)


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", [(2, 256, 256, 4, 4), (1, 300, 300, 2, 2), (2, 192, 192, 8, 2), (1, 128, 320, 2, 2)])
@pytest.mark.parametrize("k16", ["1", "0"])
def test_fa_bwd16_kernel(monkeypatch, causal, shape, k16):
    """Both D = 128 backward kernels — the 8-wave 16-keys-per-wave one (default) and the 4-wave one
    (PA_FA_BWD16=0) — against the fp32 reference."""
    monkeypatch.setenv("PA_FA_BWD16", k16)
    B, Sq, Sk, H, Hk = shape
    _run(B, Sq, Sk, H, Hk, 128, causal)


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", [(2, 256, 256, 4, 4), (1, 300, 300, 2, 2), (2, 192, 192, 8, 2), (1, 128, 320, 2, 2),
                                   (1, 320, 128, 2, 1), (1, 200, 456, 4, 2), (1, 1024, 1024, 2, 2)])
@pytest.mark.parametrize("ds", ["1", "0"])
def test_fa_bwd_ds_route(monkeypatch, causal, shape, ds):
    """D = 128 backward through the dS route (dS^T tiles + the dQ kernel, no fp32 atomics; the default) and the
    atomics kernel (PA_FA_BWD_DS=0), against the fp32 reference: ragged lengths, GQA, Sq < Sk and Sq > Sk causal."""
    monkeypatch.setenv("PA_FA_BWD_DS", ds)
    B, Sq, Sk, H, Hk = shape
    L.reset_calls()
    _run(B, Sq, Sk, H, Hk, 128, causal)
    if ds == "1":
        assert L.calls("flash_attn_bwd_ds") > 0 and L.calls("pa_flash_attn_bwd_ex") == 0
    else:
        assert L.calls("flash_attn_bwd_ds") == 0 and L.calls("pa_flash_attn_bwd_ex") > 0
