"""Numerics of the hand-written MFMA GEMM (csrc/kernels/gemm.hip) against an fp32 PyTorch reference:
all four operand layouts, ragged M/N tails, both tile widths and every fused epilogue."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from paddlepaddle_amd.ops import _loader as L  # noqa: E402
from paddlepaddle_amd.ops import gemm as G  # noqa: E402

DEV = "cuda"

# launchers each test must have dispatched (ops._loader.CALLS, reset per test by conftest)
_EXPECT = {
    "test_gemm_skinny": ["pa_gemm_skinny"],
    "test_gemm_small_m": ["pa_gemm_small_m"],
    "test_conv_implicit_gemm_fwd": ["pa_conv2d_nhwc_fwd"],
    "test_conv_implicit_gemm_dgrad": ["pa_conv2d_nhwc_fwd"],
    "test_conv_implicit_gemm_wgrad": ["pa_conv2d_nhwc_fwd", "pa_conv2d_nhwc_wgrad"],
    "test_gemm_pp": ["pa_gemm_bf16_pp"],
    "test_": ["pa_gemm_bf16|pa_gemm_bf16_pp"],  # any of
}


@pytest.fixture(autouse=True)
def _assert_dispatch(request):
    from paddlepaddle_amd.framework.flags import get_flags, set_flags
    name = request.node.originalname
    old = get_flags(["FLAGS_gemm_backend"])["FLAGS_gemm_backend"]
    set_flags({"FLAGS_gemm_backend": "hip"})  # numerics of the hand-written kernels, not the autotuner's pick
    try:
        yield
    finally:
        set_flags({"FLAGS_gemm_backend": old})
    for prefix, launchers in _EXPECT.items():
        if name.startswith(prefix):
            for n in launchers:
                assert any(L.calls(x) > 0 for x in n.split("|")), f"{n} did not run in {name}: {dict(L.CALLS)}"
            break


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
@pytest.mark.parametrize("bn", [160, 256, 128, 1, 4])
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


@pytest.mark.parametrize("bn", [256, 128])
def test_gemm_splitk_wgrad_layout(bn):
    # conv-style weight gradient: few output tiles, long K split over workgroups
    P, Cout, Cin = 4096, 64, 256
    g = torch.Generator(device=DEV).manual_seed(5)
    dy = torch.randn(P, Cout, device=DEV, generator=g).to(torch.bfloat16)
    x = torch.randn(P, Cin, device=DEV, generator=g).to(torch.bfloat16)
    out = G.gemm_splitk(dy.t(), x, 8, out_dtype=torch.float32, bn=bn)
    ref = dy.float().t() @ x.float()
    torch.testing.assert_close(out, ref, atol=0.05, rtol=1e-3)


@pytest.mark.parametrize("stride", [1, 2])
def test_conv1x1_nhwc_gemm_path(stride):
    from paddlepaddle_amd.ops import conv as C
    torch.manual_seed(0)
    x = torch.randn(4, 16, 16, 128, device=DEV).to(torch.bfloat16).requires_grad_(True)
    w = (torch.randn(192, 128, 1, 1, device=DEV) * 0.05).to(torch.bfloat16).requires_grad_(True)
    assert C.eligible(x, w, 1, True)
    y = C._Conv1x1.apply(x, w, None, stride)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, None, stride).permute(0, 2, 3, 1)
    torch.testing.assert_close(y.float(), yr, atol=0.05, rtol=2e-2)
    gy = torch.randn_like(yr)
    y.backward(gy.to(torch.bfloat16))
    yr.backward(gy)
    torch.testing.assert_close(x.grad.float(), xr.grad.permute(0, 2, 3, 1), atol=0.05, rtol=2e-2)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=0.5, rtol=2e-2)


@pytest.mark.parametrize("k,stride,pad", [(3, 1, 1), (3, 2, 1), (1, 1, 0), (5, 1, 2)])
def test_conv_implicit_gemm_fwd(k, stride, pad):
    from paddlepaddle_amd.ops import conv as C
    torch.manual_seed(1)
    x = torch.randn(3, 13, 11, 64, device=DEV).to(torch.bfloat16)
    w = (torch.randn(72, 64, k, k, device=DEV) * 0.05).to(torch.bfloat16)
    b = torch.randn(72, device=DEV).to(torch.bfloat16)
    assert C.eligible_implicit(x, w, 1)
    y = C._ConvImplicit.apply(x, w, b, stride, pad, 1)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float(), b.float(), stride, pad)
    torch.testing.assert_close(y.float(), ref.permute(0, 2, 3, 1), atol=0.06, rtol=2e-2)


@pytest.mark.parametrize("k,pad", [(3, 1), (5, 2), (3, 0)])
def test_conv_implicit_gemm_dgrad(k, pad):
    from paddlepaddle_amd.ops import conv as C
    torch.manual_seed(2)
    x = torch.randn(2, 9, 10, 64, device=DEV).to(torch.bfloat16).requires_grad_(True)
    w = (torch.randn(128, 64, k, k, device=DEV) * 0.05).to(torch.bfloat16).requires_grad_(True)
    y = C._ConvImplicit.apply(x, w, None, 1, pad, 1)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, None, 1, pad)
    g = torch.randn_like(yr)
    y.backward(g.permute(0, 2, 3, 1).to(torch.bfloat16))
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad.permute(0, 2, 3, 1), atol=0.08, rtol=2e-2)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=0.5, rtol=3e-2)


@pytest.mark.parametrize("shape,C,Cout,k,stride,pad,dil", [((4, 8, 8), 64, 64, 3, 1, 1, 1),
                                                          ((4, 16, 16), 64, 72, 3, 2, 1, 1),
                                                          ((2, 12, 16), 128, 64, 3, 1, 1, 1),
                                                          ((2, 8, 16), 64, 64, 5, 1, 2, 1),
                                                          ((2, 8, 16), 64, 64, 3, 1, 2, 2)])
def test_conv_implicit_gemm_wgrad(shape, C, Cout, k, stride, pad, dil):
    """Weight gradient by the split-K implicit GEMM (im2col rows gathered per pixel and tap)."""
    from paddlepaddle_amd.ops import conv as Cv
    torch.manual_seed(3)
    N, H, W = shape
    x = torch.randn(N, H, W, C, device=DEV).to(torch.bfloat16)
    w = (torch.randn(Cout, C, k, k, device=DEV) * 0.05).to(torch.bfloat16).requires_grad_(True)
    y = Cv._ConvImplicit.apply(x, w, None, stride, pad, dil)
    P = y.shape[0] * y.shape[1] * y.shape[2]
    assert P % 64 == 0  # the HIP weight-gradient path, not MIOpen
    wr = w.detach().float().requires_grad_(True)
    yr = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wr, None, stride, pad, dil)
    g = torch.randn_like(yr)
    y.backward(g.permute(0, 2, 3, 1).to(torch.bfloat16))
    yr.backward(g)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=0.5, rtol=3e-2)


@pytest.mark.parametrize("stages", [4, 3])
@pytest.mark.parametrize("M,K,N,splits", [(32, 4096, 1280, None), (1, 512, 264, 2), (64, 1024, 4096, 4), (17, 256, 8, 1),
                                          (32, 11008, 512, 43)])
def test_gemm_small_m_decode_shapes(M, K, N, splits, stages):
    g = torch.Generator(device=DEV).manual_seed(9)
    a = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    b = (torch.randn(K, N, device=DEV, generator=g) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device=DEV, generator=g).to(torch.bfloat16)
    assert G.small_m_supported(a, b)
    c = G.gemm_small_m(a, b, bias, splits=splits, stages=stages)
    ref = a.float() @ b.float() + bias.float()
    torch.testing.assert_close(c.float(), ref, atol=0.05, rtol=2e-2)


@pytest.mark.parametrize("a_kmaj,b_kmaj", [(True, False), (True, True), (False, False), (False, True)])
@pytest.mark.parametrize("M,N", [(4096, 5120), (4000, 5000)])
def test_gemm_pp_balanced_tail(a_kmaj, b_kmaj, M, N):
    """320 output tiles on 256 CUs: 256 whole tiles + 64 tiles cut 4-ways along K (fp32 partials summed by
    the tail reduction); ragged M / N edges in the tail tiles."""
    K = 1024
    a, b = _operands(M, N, K, a_kmaj, b_kmaj, seed=11)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    if cus == 256:
        assert L.lib().pa_gemm_pp_ws_bytes(M, N, K) == 64 * 4 * 65536 * 4
    c = G.gemm(a, b, bn=1)
    torch.testing.assert_close(c.float(), _ref(a, b), atol=0.3, rtol=1e-2)


def test_gemm_pp_tail_epilogues():
    M, N, K = 4096, 5120, 1024
    a, b = _operands(M, N, K, True, False, seed=12)
    bias = torch.randn(N, device=DEV).to(torch.bfloat16)
    aux = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    c = G.gemm(a, b, bias=bias, gelu=True, aux=aux, bn=1)
    pre = _ref(a, b) + bias.float()
    torch.testing.assert_close(aux.float(), pre, atol=0.3, rtol=1e-2)
    torch.testing.assert_close(c.float(), torch.nn.functional.gelu(pre, approximate="tanh"), atol=0.3, rtol=1e-2)
    base = torch.randn(M, N, device=DEV)
    out = base.clone()
    G.gemm(a, b, out=out, accumulate=True, alpha=0.5, bn=1)
    torch.testing.assert_close(out, base + 0.5 * _ref(a, b), atol=0.1, rtol=1e-2)


@pytest.mark.parametrize("N,K", [(64, 64), (256, 64), (64, 256), (128, 128), (32, 32), (256, 256)])
@pytest.mark.parametrize("b_kmaj", [True, False])
@pytest.mark.parametrize("epi", ["none", "bias_relu", "accum"])
def test_gemm_skinny(N, K, b_kmaj, epi):
    """Memory-bound tall-M kernel (csrc/kernels/gemm_skinny.hip) incl. a ragged last 16-row block."""
    M = 4104
    a, b = _operands(M, N, K, True, b_kmaj, seed=N + K)
    assert G.skinny_supported(a, b)
    ref = _ref(a, b)
    bias = None
    out = None
    if epi == "bias_relu":
        bias = torch.randn(N, device=DEV).bfloat16()
        ref = torch.relu(ref + bias.float())
    if epi == "accum":
        out = torch.randn(M, N, device=DEV).bfloat16()
        ref = ref + out.float()
    got = G.gemm_skinny(a, b, bias=bias, out=out, accumulate=epi == "accum", relu=epi == "bias_relu")
    torch.testing.assert_close(got.float(), ref, rtol=2e-2, atol=2e-2 * (K ** 0.5))
