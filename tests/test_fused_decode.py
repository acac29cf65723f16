"""Fused decode-step kernels (csrc/kernels/decode_fused.hip): residual add + RMSNorm, and RoPE + QKV split +
KV-cache write at a device-side position. GPU tests compare the HIP kernels with plain fp32 PyTorch references;
the CPU test checks the fallback composition."""
import pytest
import torch

from paddlepaddle_amd import ops
from paddlepaddle_amd.ops.rope import rope_tables


def _rms_ref(s, w, eps):
    s = s.float()
    return s * torch.rsqrt(s.pow(2).mean(-1, keepdim=True) + eps) * w.float()


def _rot_ref(x, cos, sin):  # NeoX halves, fp32
    d = x.shape[-1] // 2
    x = x.float()
    rot = torch.cat([-x[..., d:], x[..., :d]], -1)
    return x * cos.float() + rot * sin.float()


def _rope_cache_ref(qkv, H, Hkv, D, cs, sn, pos, kc, vc):
    B = qkv.shape[0]
    q, k, v = qkv.float().split([H * D, Hkv * D, Hkv * D], -1)
    q = _rot_ref(q.view(B, H, D), cs, sn)
    k = _rot_ref(k.view(B, Hkv, D), cs, sn)
    kc, vc = kc.clone(), vc.clone()
    kc[:B, :, pos] = k.to(kc.dtype)
    vc[:B, :, pos] = v.view(B, Hkv, D).to(vc.dtype)
    return q, kc, vc


def test_fused_decode_fallbacks_cpu():
    g = torch.Generator().manual_seed(0)
    x, r = torch.randn(6, 64, generator=g), torch.randn(6, 64, generator=g)
    w = torch.rand(64, generator=g) + 0.5
    s, y = ops.add_rms_norm(x, r, w, 1e-6)
    torch.testing.assert_close(s, x + r)
    torch.testing.assert_close(y, _rms_ref(x + r, w, 1e-6), rtol=1e-5, atol=1e-5)
    B, H, Hkv, D, Lc = 3, 4, 2, 32, 16
    qkv = torch.randn(B, (H + 2 * Hkv) * D, generator=g)
    cos, sin = rope_tables(Lc, D)
    pos = torch.tensor([5])
    kc, vc = torch.zeros(B, Hkv, Lc, D), torch.zeros(B, Hkv, Lc, D)
    q_ref, kc_ref, vc_ref = _rope_cache_ref(qkv, H, Hkv, D, cos[5], sin[5], 5, kc, vc)
    q = ops.decode_rope_cache(qkv, H, Hkv, D, cos.index_select(0, pos), sin.index_select(0, pos), pos, kc, vc)
    torch.testing.assert_close(q, q_ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(kc, kc_ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(vc, vc_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [37, 300])  # workgroup-per-row / wave-per-row kernels
@pytest.mark.parametrize("cols", [256, 4096, 5120, 8192])
def test_add_rms_norm_hip(cols, rows):
    g = torch.Generator().manual_seed(cols)
    x = torch.randn(rows, cols, generator=g).to("cuda", torch.bfloat16)
    r = torch.randn(rows, cols, generator=g).to("cuda", torch.bfloat16)
    w = (torch.rand(cols, generator=g) + 0.5).to("cuda", torch.bfloat16)
    s, y = ops.add_rms_norm(x, r, w, 1e-5)
    assert torch.equal(s, x + r)  # the same rounded sum as the unfused add
    ref = _rms_ref(x + r, w, 1e-5)
    assert (y.float() - ref).abs().max().item() < 3e-2 * ref.abs().max().item()
    x2 = x.clone()
    s2, y2 = ops.add_rms_norm(x2, r, w, 1e-5, inplace=True)
    assert s2.data_ptr() == x2.data_ptr() and torch.equal(s2, s) and torch.equal(y2, y)


@pytest.mark.gpu
@pytest.mark.parametrize("H,Hkv,D", [(32, 32, 128), (8, 2, 128), (4, 4, 64)])
def test_decode_rope_cache_hip(H, Hkv, D):
    g = torch.Generator().manual_seed(H + D)
    B, Bc, Lc, p = 5, 7, 96, 41
    qkv = torch.randn(B, (H + 2 * Hkv) * D, generator=g).to("cuda", torch.bfloat16)
    cos, sin = rope_tables(Lc, D, device="cuda")
    pos = torch.tensor([p], device="cuda")
    kc = torch.randn(Bc, Hkv, Lc, D, generator=g).to("cuda", torch.bfloat16)
    vc = torch.randn(Bc, Hkv, Lc, D, generator=g).to("cuda", torch.bfloat16)
    q_ref, kc_ref, vc_ref = _rope_cache_ref(qkv, H, Hkv, D, cos[p], sin[p], p, kc, vc)
    q = ops.decode_rope_cache(qkv, H, Hkv, D, cos.index_select(0, pos), sin.index_select(0, pos), pos, kc, vc)
    assert (q.float() - q_ref).abs().max().item() < 3e-2
    assert (kc.float() - kc_ref.float()).abs().max().item() < 3e-2
    assert torch.equal(vc, vc_ref)
