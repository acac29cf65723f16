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
