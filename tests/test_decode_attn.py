"""Paged-KV decode attention (ops.paged_decode_attention / dense_decode_attention): the HIP
flash-decoding kernel (csrc/kernels/decode_attn.hip) against a plain fp32 PyTorch reference."""
import math

import numpy as np
import pytest
import torch

from paddlepaddle_amd import ops
from paddlepaddle_amd.ops.attention import paged_decode_reference


def _naive(q, kc, vc, tables, lens):
    N, H, D = q.shape
    _, Hkv, bs, _ = kc.shape
    out = torch.zeros(N, H, D)
    for n in range(N):
        ln = int(lens[n])
        blocks = [int(b) for b in tables[n, :(ln + bs - 1) // bs]]
        K = torch.cat([kc[b] for b in blocks], 1)[:, :ln].float()   # [Hkv, ln, D]
        V = torch.cat([vc[b] for b in blocks], 1)[:, :ln].float()
        for h in range(H):
            hk = h // (H // Hkv)
            p = torch.softmax(q[n, h].float() @ K[hk].T / math.sqrt(D), -1)
            out[n, h] = p @ V[hk]
    return out


def _case(N, H, Hkv, D, bs, lens, device="cpu", dtype=torch.float32, seed=0):
    g = torch.Generator().manual_seed(seed)
    max_blocks = max((l + bs - 1) // bs for l in lens) + 1
    nb = N * max_blocks + 3
    kc = torch.randn(nb, Hkv, bs, D, generator=g).to(dtype)
    vc = torch.randn(nb, Hkv, bs, D, generator=g).to(dtype)
    perm = torch.randperm(nb, generator=g)[:N * max_blocks].view(N, max_blocks).int()
    q = torch.randn(N, H, D, generator=g).to(dtype)
    return q.to(device), kc.to(device), vc.to(device), perm.to(device), torch.tensor(lens, dtype=torch.int32).to(device)


def test_paged_reference_matches_naive_cpu():
    q, kc, vc, tab, lens = _case(3, 8, 2, 32, 4, [1, 7, 13])
    np.testing.assert_allclose(paged_decode_reference(q, kc, vc, tab, lens).numpy(),
                               _naive(q, kc, vc, tab, lens).numpy(), rtol=1e-5, atol=1e-5)
    got = ops.paged_decode_attention(q, kc, vc, tab, lens)  # CPU: reference path
    np.testing.assert_allclose(got.numpy(), _naive(q, kc, vc, tab, lens).numpy(), rtol=1e-5, atol=1e-5)


def test_dense_decode_cpu():
    torch.manual_seed(0)
    B, H, L, D = 2, 4, 16, 32
    kc, vc, q = torch.randn(B, H, L, D), torch.randn(B, H, L, D), torch.randn(B, H, D)
    lens = torch.tensor([5, 16])
    got = ops.dense_decode_attention(q, kc, vc, lens)
    for b in range(B):
        p = torch.softmax(torch.einsum("hd,hld->hl", q[b], kc[b, :, :lens[b]]) / math.sqrt(D), -1)
        np.testing.assert_allclose(got[b].numpy(), torch.einsum("hl,hld->hd", p, vc[b, :, :lens[b]]).numpy(),
                                   rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,Hkv,bs,lens", [
    (1, 8, 8, 64, [1]),
    (2, 32, 8, 16, [17, 300]),
    (4, 16, 4, 64, [64, 65, 1000, 4097]),
    (3, 8, 1, 32, [2000, 1, 33]),
    (64, 40, 40, 64, [129] * 64),
])
def test_paged_decode_hip_matches_fp32(N, H, Hkv, bs, lens):
    from paddlepaddle_amd.ops import _loader as L
    q, kc, vc, tab, ln = _case(N, H, Hkv, 128, bs, lens, "cuda", torch.bfloat16)
    assert L.hip_enabled_for(q) and L.has("pa_paged_decode_attn")
    got = ops.paged_decode_attention(q, kc, vc, tab, ln).float()
    ref = paged_decode_reference(q.float(), kc.float(), vc.float(), tab, ln)
    torch.testing.assert_close(got, ref, rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
def test_dense_decode_hip_matches_fp32():
    torch.manual_seed(0)
    B, H, L, D = 5, 16, 512, 128
    kc = torch.randn(B, H, L, D, device="cuda").bfloat16()
    vc = torch.randn(B, H, L, D, device="cuda").bfloat16()
    q = torch.randn(B, H, D, device="cuda").bfloat16()
    lens = torch.tensor([1, 63, 64, 300, 512], device="cuda")
    got = ops.dense_decode_attention(q, kc, vc, lens).float()
    valid = torch.arange(L, device="cuda")[None] < lens[:, None]
    s = torch.einsum("bhd,bhld->bhl", q.float(), kc.float()) / math.sqrt(D)
    s = s.masked_fill(~valid[:, None], float("-inf"))
    ref = torch.einsum("bhl,bhld->bhd", torch.softmax(s, -1), vc.float())
    torch.testing.assert_close(got, ref, rtol=2e-2, atol=2e-2)
