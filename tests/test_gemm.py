"""Numerics of the hand-written MFMA GEMM (csrc/kernels/gemm.hip) against an fp32 PyTorch reference:
all four operand layouts, ragged M/N tails, both tile widths and every fused epilogue."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from paddlepaddle_amd.ops import _loader as L  # noqa: E402
from paddlepaddle_amd.ops import gemm as G  # noqa: E402

DEV = "cuda"


def _operands(M, N, K, a_kmaj, b_kmaj, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    a32 = torch.randn(M, K, device=DEV, generator=g)
    b32 = torch.randn(K, N, device=DEV, generator=g)
    # asymmetric operands: a row/col swap in the kernel cannot pass
    a32[:, 0] += torch.arange(M, device=DEV) * 0.01
    a = a32.to(torch.bfloat16) if a_kmaj else a32.t().contiguous().to(torch.bfloat16).t()
    b = b32.t().contiguous().to(torch.bfloat16).t() if b_kmaj else b32.to(torch.bfloat16)
    return a, b


def _ref(a, b):
    return a.float() @ b.float()


@pytest.mark.parametrize("a_kmaj", [True, False])
@pytest.mark.parametrize("b_kmaj", [True, False])
@pytest.mark.parametrize("bn", [160, 256, 128, 1])
@pytest.mark.parametrize("M,N,K", [(512, 512, 256), (264, 392, 128), (1000, 776, 320)])
def test_gemm_layouts(a_kmaj, b_kmaj, bn, M, N, K):
    a, b = _operands(M, N, K, a_kmaj, b_kmaj)
    assert G.supported(a, b)
    c = G.gemm(a, b, bn=bn)
    assert L._LIB is not None
    torch.testing.assert_close(c.float(), _ref(a, b), atol=0.15, rtol=1e-2)


def test_gemm_bias_gelu_aux():
    M, N, K = 768, 1024, 512
    a, b = _operands(M, N, K, True, False, seed=1)
    bias = torch.randn(N, device=DEV).to(torch.bfloat16)
    aux = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    c = G.gemm(a, b, bias=bias, gelu=True, aux=aux)
    pre = _ref(a, b) + bias.float()
    torch.testing.assert_close(aux.float(), pre, atol=0.2, rtol=1e-2)
    torch.testing.assert_close(c.float(), torch.nn.functional.gelu(pre, approximate="tanh"), atol=0.2, rtol=1e-2)


@pytest.mark.parametrize("out_dt", [torch.float32, torch.bfloat16])
def test_gemm_accumulate(out_dt):
    M, N, K = 520, 640, 1024
    a, b = _operands(M, N, K, False, False, seed=2)  # wgrad layout: x^T . dy
    base = torch.randn(M, N, device=DEV).to(out_dt)
    out = base.clone()
    G.gemm(a, b, out=out, accumulate=True, alpha=0.5)
    ref = base.float() + 0.5 * _ref(a, b)
    torch.testing.assert_close(out.float(), ref, atol=0.3 if out_dt == torch.bfloat16 else 0.05, rtol=1e-2)


def test_gemm_large_gpt_shape():
    # one GPT-3 13B projection (fc1 of a 2x2048 micro-batch), reduced K to keep the test fast
    M, N, K = 4096, 20480, 512
    a, b = _operands(M, N, K, True, False, seed=3)
    c = G.gemm(a, b)
    ref = _ref(a, b)
    err = (c.float() - ref).abs().max().item()
    assert err < 0.25 + 1e-2 * ref.abs().max().item()
