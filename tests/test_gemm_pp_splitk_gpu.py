"""Split-K on the ping-pong 256x256 GEMM (pa_gemm_bf16_pp_splitk: every tile cut into K slices, fp32 partial tiles
summed by the tail-reduction kernel) against the fp32 product, for the operand layouts the 1x1-convolution weight
gradient uses (dY^T: MN-major A; X: MN-major B) and K-major ones, ragged M / N."""
import pytest
import torch

from paddlepaddle_amd.ops import gemm as G
from paddlepaddle_amd.ops import _loader as L

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K,a_t", [(1024, 256, 50176, True), (512, 2048, 12544, True), (300, 520, 4096, False),
                                       (256, 256, 1024, True)])
def test_pp_splitk_matches_fp32(M, N, K, a_t):
    g = torch.Generator(device="cuda").manual_seed(0)
    if a_t:  # A = dY^T: stored [K, M]
        a = torch.randn(K, M, device="cuda", dtype=torch.bfloat16, generator=g).t()
    else:
        a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16, generator=g)
    sp = G.pp_splits(M, N, K)
    assert sp > 1 and G.gemm_pp_splitk_ok(a, b, sp)
    n0 = L.calls("pa_gemm_bf16_pp_splitk")
    out = G.gemm_pp_splitk(a, b, sp, torch.bfloat16)
    assert L.calls("pa_gemm_bf16_pp_splitk") == n0 + 1
    ref = a.float() @ b.float()
    err = (out.float() - ref).abs().max() / ref.abs().max()
    assert err < 1e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_pp_splitk_accumulate_wgrad(dt):
    """C += x^T dY on the split-K ping-pong kernel (the linear weight-gradient candidate for few output tiles over
    many tokens, e.g. GPT-3 1.3B's 2048 x 2048 weights at 32k tokens): accumulated into an existing bf16 / fp32
    gradient, against the fp32 reference; the linear backward picks it by measured time (ops/linear.py)."""
    g = torch.Generator(device="cuda").manual_seed(1)
    M, N, K = 512, 768, 8192
    x = torch.randn(K, M, device="cuda", dtype=torch.bfloat16, generator=g)
    dy = torch.randn(K, N, device="cuda", dtype=torch.bfloat16, generator=g)
    acc = torch.randn(M, N, device="cuda", dtype=dt, generator=g)
    ref = acc.float() + x.t().float() @ dy.float()
    sp = G.pp_splits(M, N, K)
    assert sp > 1 and G.gemm_pp_splitk_ok(x.t(), dy, sp)
    n0 = L.calls("pa_gemm_bf16_pp_splitk")
    out = G.gemm_pp_splitk(x.t(), dy, sp, out=acc, accumulate=True)
    assert out is acc and L.calls("pa_gemm_bf16_pp_splitk") == n0 + 1
    err = (acc.float() - ref).abs().max() / ref.abs().max()
    assert err < 1e-2, err
