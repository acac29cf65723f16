"""fp8_fp8_half_gemm_fused / ops.fp8.gemm_fp8 against the fp32 dequantised reference. GPU: the hand-written
block-scaled-MFMA kernel (csrc/kernels/gemm_fp8.hip) must be the path that runs (dispatch counter), exact on
small-integer data (checks the fragment / output mapping) and within output rounding on random data, for
e4m3 / e5m2 operand mixes, fp16 / bf16 outputs, bias and identity / relu / gelu epilogues, ragged M / N."""
import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle
from paddlepaddle_amd.ops import _loader as L
from paddlepaddle_amd.ops.fp8 import gemm_fp8


def _ref(a, b_nk, bias, alpha, act, odt):
    y = alpha * (a.float() @ b_nk.float().t())
    if bias is not None:
        y = y + bias.float()
    y = torch.nn.functional.gelu(y) if act == "gelu" else (torch.relu(y) if act == "relu" else y)
    return y.to(odt)


def test_fp8_api_semantics_cpu():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, 5, 256, generator=g).to(torch.float8_e4m3fn)
    w = torch.randn(256, 40, generator=g).to(torch.float8_e5m2)
    bias = torch.randn(40, generator=g).half()
    out = paddle.linalg.fp8_fp8_half_gemm_fused(paddle.to_tensor(x), paddle.to_tensor(w), bias=paddle.to_tensor(bias),
                                                scale=0.25, output_dtype="float16", act="relu")
    ref = _ref(x.reshape(-1, 256), w.t(), bias, 0.25, "relu", torch.float16).view(3, 5, 40)
    np.testing.assert_allclose(out.numpy().astype("float32"), ref.float().numpy(), rtol=1e-3, atol=1e-3)
    with pytest.raises(ValueError):
        paddle.linalg.fp8_fp8_half_gemm_fused(paddle.to_tensor(x), paddle.to_tensor(w), output_dtype="float32")


@pytest.mark.gpu
def test_fp8_gemm_exact_on_small_integers_gpu():
    g = torch.Generator().manual_seed(1)
    M, N, K = 300, 260, 384
    a = torch.randint(-2, 3, (M, K), generator=g).float()
    b = torch.randint(-2, 3, (N, K), generator=g).float()
    a8, b8 = a.to(torch.float8_e4m3fn).cuda(), b.to(torch.float8_e4m3fn).cuda()
    n0 = L.calls("pa_gemm_fp8") + L.calls("pa_gemm_fp8_ws")
    out = gemm_fp8(a8, b8, None, 1.0, "identity", torch.float16)
    assert L.calls("pa_gemm_fp8") + L.calls("pa_gemm_fp8_ws") == n0 + 1
    torch.testing.assert_close(out.float().cpu(), a @ b.t(), rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("fa,fb,odt,act,bias,shape", [
    (torch.float8_e4m3fn, torch.float8_e4m3fn, torch.float16, "identity", False, (512, 768, 1024)),
    (torch.float8_e4m3fn, torch.float8_e5m2, torch.bfloat16, "relu", True, (333, 516, 640)),
    (torch.float8_e5m2, torch.float8_e4m3fn, torch.float16, "gelu", True, (1024, 1280, 2048)),
    (torch.float8_e5m2, torch.float8_e5m2, torch.bfloat16, "identity", True, (64, 4096, 512)),
])
def test_fp8_gemm_matches_dequantised_reference_gpu(fa, fb, odt, act, bias, shape):
    M, N, K = shape
    g = torch.Generator().manual_seed(2)
    a = (torch.randn(M, K, generator=g)).to(fa).cuda()
    b = (torch.randn(N, K, generator=g)).to(fb).cuda()
    bv = torch.randn(N, generator=g).to(odt).cuda() if bias else None
    alpha = 1.0 / 16
    out = gemm_fp8(a, b, bv, alpha, act, odt)
    ref = _ref(a.cpu(), b.cpu(), None if bv is None else bv.cpu(), alpha, act, torch.float32)
    tol = 1e-2 if odt == torch.float16 else 2e-2
    torch.testing.assert_close(out.float().cpu(), ref, rtol=tol, atol=tol * 2)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(300, 264, 384), (1000, 2048, 1280), (256, 256, 128), (77, 520, 256),
                                   (513, 776, 896), (4096, 5120, 2048)])
@pytest.mark.parametrize("kernel", ["auto", "generic"])
def test_fp8_gemm_kernels_exact_on_small_integers_gpu(shape, kernel):
    """Both fp8 kernels — the ping-pong 256x256 schedule (auto, N % 8 == 0) and the generic one — exact on
    small-integer data: ragged M / N tiles, a single K-tile (K = 128) and two (K = 256); 4096 x 5120 (320 tiles)
    runs the ping-pong kernel's balanced tail (64 tiles cut into 4 K slices + the reduction kernel)."""
    from paddlepaddle_amd.ops import fp8 as F8
    M, N, K = shape
    g = torch.Generator().manual_seed(5)
    a = torch.randint(-3, 4, (M, K), generator=g).float()
    b = torch.randint(-2, 3, (N, K), generator=g).float()
    bias = torch.randint(-4, 5, (N,), generator=g).float()
    a8, b8 = a.to(torch.float8_e4m3fn).cuda(), b.to(torch.float8_e4m3fn).cuda()
    old = F8.set_kernel(kernel)
    try:
        out = gemm_fp8(a8, b8, bias.to(torch.bfloat16).cuda(), 0.5, "relu", torch.bfloat16)
    finally:
        F8.set_kernel(old)
    ref = torch.relu(0.5 * (a @ b.t()) + bias)
    torch.testing.assert_close(out.float().cpu(), ref.to(torch.bfloat16).float(), rtol=0, atol=0)


@pytest.mark.gpu
def test_fp8_fused_api_weight_layouts_gpu():
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 96, 512, generator=g).to(torch.float8_e4m3fn).cuda()
    w_kn = torch.randn(512, 384, generator=g).to(torch.float8_e4m3fn).cuda()
    ref = _ref(x.reshape(-1, 512).cpu(), w_kn.t().cpu(), None, 0.5, "identity", torch.float32).view(2, 96, 384)
    for wt, ty in ((w_kn, False), (w_kn.t().contiguous(), True)):
        out = paddle.linalg.fp8_fp8_half_gemm_fused(paddle.to_tensor(x), paddle.to_tensor(wt), transpose_y=ty,
                                                    scale=0.5, output_dtype="bfloat16")
        torch.testing.assert_close(out._t.float().cpu(), ref, rtol=2e-2, atol=4e-2)
