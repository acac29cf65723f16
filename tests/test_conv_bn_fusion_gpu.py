"""Conv -> BN fusion (ops/_conv_bn.py): the convolution's GEMM epilogue writes the batch-norm partial sums of its
bf16 output (csrc/kernels/gemm.hip kEpiStats) and the BN forward starts from them (bn.hip pa_bn_fwd_nhwc_pre)
instead of re-reading the activation. Reference: paddle/phi/kernels/fusion/gpu/fused_scale_bias_relu_conv_bn_kernel.cu.
Each check compares against plain PyTorch fp64/fp32 math of the same op, or against the unfused path."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from paddlepaddle_amd.ops import _loader as L  # noqa: E402
from paddlepaddle_amd.ops import gemm as G  # noqa: E402
from paddlepaddle_amd.ops import conv as C  # noqa: E402
from paddlepaddle_amd.ops import _conv_bn as CB  # noqa: E402


def _fold(stats, chunks, n):
    s = stats.view(2, chunks, n).double().sum(1)
    return s[0], s[1]


@pytest.mark.parametrize("M,N,K", [(1000, 64, 64), (4096, 192, 256), (25088, 128, 576), (300, 512, 128)])
def test_gemm_epilogue_bn_partials(M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M + N)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    y, stats, chunks = G.gemm_bn_stats(a, w.t())
    torch.cuda.synchronize()
    ref = a.float() @ w.float().t()
    assert (y.float() - ref).abs().max().item() < 3e-2 * ref.abs().max().item()
    s1, s2 = _fold(stats, chunks, N)
    yd = y.double()
    torch.testing.assert_close(s1, yd.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(s2, (yd * yd).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("n,hw,cin,cout,k,stride", [(4, 28, 64, 64, 3, 1), (8, 28, 128, 128, 3, 2),
                                                    (2, 14, 64, 256, 1, 1), (32, 28, 128, 128, 3, 1)])
def test_conv_epilogue_bn_partials(n, hw, cin, cout, k, stride):
    g = torch.Generator(device="cuda").manual_seed(n * hw + cin)
    x = torch.randn(n, hw, hw, cin, device="cuda", generator=g).bfloat16()
    w = (torch.randn(cout, cin, k, k, device="cuda", generator=g) / (cin * k * k) ** 0.5).bfloat16()
    L.reset_calls()
    y, (stats, chunks) = C._own_fwd_stats(x, w, None, stride, k // 2, 1)
    torch.cuda.synchronize()
    assert L.calls("pa_conv2d_nhwc_fwd_stats") + L.calls("pa_gemm_bf16_stats") == 1
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float(), None, stride, k // 2)
    ref = ref.permute(0, 2, 3, 1)
    assert (y.float() - ref).abs().max().item() < 3e-2 * ref.abs().max().item()
    s1, s2 = _fold(stats, chunks, cout)
    yd = y.double().reshape(-1, cout)
    torch.testing.assert_close(s1, yd.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(s2, (yd * yd).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("M,N,K", [(5000, 64, 256), (20000, 128, 64), (3136, 64, 64)])
def test_skinny_gemm_epilogue_bn_partials(M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M + K)
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    r = G.gemm_skinny_bn_stats(a, w.t())
    assert r is not None
    y, stats, chunks = r
    torch.cuda.synchronize()
    ref = a.float() @ w.float().t()
    assert (y.float() - ref).abs().max().item() < 3e-2 * ref.abs().max().item()
    s1, s2 = _fold(stats, chunks, N)
    yd = y.double()
    torch.testing.assert_close(s1, yd.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(s2, (yd * yd).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("n,hw", [(2, 56), (8, 20)])
def test_skinny_halo_conv_epilogue_bn_partials(n, hw):
    g = torch.Generator(device="cuda").manual_seed(n + hw)
    x = torch.randn(n, hw, hw, 64, device="cuda", generator=g).bfloat16()
    w = (torch.randn(64, 64, 3, 3, device="cuda", generator=g) / 24.0).bfloat16()
    L.reset_calls()
    y, (stats, chunks) = C._own_fwd_stats(x, w, None, 1, 1, 1, skinny=True)
    torch.cuda.synchronize()
    assert L.calls("pa_conv_skinny_stats") == 1
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float(), None, 1, 1).permute(0, 2, 3, 1)
    assert (y.float() - ref).abs().max().item() < 3e-2 * ref.abs().max().item()
    s1, s2 = _fold(stats, chunks, 64)
    yd = y.double().reshape(-1, 64)
    torch.testing.assert_close(s1, yd.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(s2, (yd * yd).sum(0), rtol=1e-4, atol=1e-2)


def _block(fused, x0, params, steps=2):
    """conv(3x3) -> BN+relu -> conv(1x1) -> BN (+ residual) + relu on the paddle NHWC layers."""
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.framework import flags
    flags.set_flags({"FLAGS_conv_bn_fusion": fused})
    CB._FEEDS_BN.clear()
    paddle.seed(0)
    nn = paddle.nn
    conv1 = nn.Conv2D(64, 64, 3, padding=1, bias_attr=False, data_format="NHWC")
    bn1 = nn.BatchNorm2D(64, data_format="NHWC")
    conv2 = nn.Conv2D(64, 64, 1, bias_attr=False, data_format="NHWC")
    bn2 = nn.BatchNorm2D(64, data_format="NHWC")
    conv1.weight._t.data = params[0].bfloat16()
    conv2.weight._t.data = params[1].bfloat16()
    outs = []
    for _ in range(steps):
        x = paddle.Tensor(x0.clone().requires_grad_(True))
        x.stop_gradient = False
        h = bn1.fused_forward(conv1(x), "relu", None)
        y = bn2.fused_forward(conv2(h), "relu", x)
        gy = torch.randn(y.shape, device="cuda", generator=torch.Generator(device="cuda").manual_seed(9))
        y.astype("float32").backward(paddle.Tensor(gy))
        outs.append((y._t.float().clone(), x.grad._t.float().clone(), conv1.weight.grad._t.float().clone()))
        conv1.weight.clear_gradient()
        conv2.weight.clear_gradient()
    torch.cuda.synchronize()
    return outs, bn1._mean._t.clone(), bn2._variance._t.clone()


def test_fused_block_matches_unfused():
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.framework import flags
    paddle.set_device("gpu:0")
    g = torch.Generator(device="cuda").manual_seed(5)
    x0 = torch.randn(16, 28, 28, 64, device="cuda", generator=g).bfloat16()
    params = [torch.randn(64, 64, 3, 3, device="cuda", generator=g) * 0.05,
              torch.randn(64, 64, 1, 1, device="cuda", generator=g) * 0.1]
    try:
        ref, rm_ref, rv_ref = _block(False, x0, params)
        L.reset_calls()
        got, rm, rv = _block(True, x0, params)
        # step 1 learns the conv -> BN pairs, step 2 runs fused
        assert L.calls("pa_bn_fwd_nhwc_pre") >= 1, dict(L.CALLS)
    finally:
        flags.set_flags({"FLAGS_conv_bn_fusion": True})
    for (y, dx, dw), (yr, dxr, dwr) in zip(got, ref):
        assert (y - yr).abs().max().item() <= 0.02 * yr.abs().max().item() + 1e-3
        assert (dx - dxr).abs().max().item() <= 0.02 * dxr.abs().max().item() + 1e-3
        assert (dw - dwr).abs().max().item() <= 0.02 * dwr.abs().max().item() + 1e-3
    torch.testing.assert_close(rm, rm_ref, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(rv, rv_ref, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("k,cin,cout,hw", [(1, 64, 128, 28), (3, 64, 64, 20), (1, 256, 64, 14)])
def test_dgrad_epilogue_bn_backward_partials(k, cin, cout, hw):
    g = torch.Generator(device="cuda").manual_seed(k + cin + hw)
    n = 4
    bx = torch.randn(n, hw, hw, cin, device="cuda", generator=g).bfloat16()      # BN input (= conv input shape)
    mean = torch.randn(cin, device="cuda", generator=g) * 0.1
    ss = torch.stack([torch.rand(cin, device="cuda", generator=g) + 0.5,
                      torch.randn(cin, device="cuda", generator=g) * 0.2]).contiguous()
    w = (torch.randn(cout, cin, k, k, device="cuda", generator=g) / (cin * k * k) ** 0.5).bfloat16()
    x = torch.empty(n, hw, hw, cin, device="cuda", dtype=torch.bfloat16)     # only its shape is used
    dy = torch.randn(n, hw, hw, cout, device="cuda", generator=g).bfloat16()
    L.reset_calls()
    dx, (stats, chunks) = C._own_dgrad_bnbwd(x, w, dy, k // 2, (bx.view(-1, cin), mean, ss))
    torch.cuda.synchronize()
    assert L.calls("pa_gemm_bf16_bnbwd") + L.calls("pa_conv2d_nhwc_fwd_bnbwd") == 1
    ref = torch.nn.grad.conv2d_input((n, cin, hw, hw), w.float(), dy.float().permute(0, 3, 1, 2), 1, k // 2)
    ref = ref.permute(0, 2, 3, 1)
    assert (dx.float() - ref).abs().max().item() < 3e-2 * ref.abs().max().item()
    xf = bx.float().reshape(-1, cin)
    g2 = dx.float().reshape(-1, cin)
    dyp = torch.where(xf * ss[0] + ss[1] > 0, g2, torch.zeros_like(g2)).double()
    s1, s2 = _fold(stats, chunks, cin)
    torch.testing.assert_close(s1, dyp.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(s2, (dyp * (xf.double() - mean.double())).sum(0), rtol=1e-4, atol=1e-2)


def test_fused_block_forward_and_backward_paths_forced_hip(monkeypatch):
    """With the hand-written kernels forced, both halves of the fusion run: conv epilogue -> BN forward
    statistics, and dgrad epilogue -> BN backward reduction (bn1 feeds the second convolution)."""
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.framework import flags
    paddle.set_device("gpu:0")
    g = torch.Generator(device="cuda").manual_seed(6)
    x0 = torch.randn(8, 28, 28, 64, device="cuda", generator=g).bfloat16()
    params = [torch.randn(64, 64, 3, 3, device="cuda", generator=g) * 0.05,
              torch.randn(64, 64, 1, 1, device="cuda", generator=g) * 0.1]
    flags.set_flags({"FLAGS_gemm_backend": "hip"})
    try:
        ref, rm_ref, rv_ref = _block(False, x0, params)
        L.reset_calls()
        got, rm, rv = _block(True, x0, params)
        assert L.calls("pa_bn_fwd_nhwc_pre") >= 2, dict(L.CALLS)
        assert L.calls("pa_bn_bwd_nhwc_pre") >= 1, dict(L.CALLS)
    finally:
        flags.set_flags({"FLAGS_gemm_backend": "auto", "FLAGS_conv_bn_fusion": True})
    for (y, dx, dw), (yr, dxr, dwr) in zip(got, ref):
        assert (y - yr).abs().max().item() <= 0.02 * yr.abs().max().item() + 1e-3
        assert (dx - dxr).abs().max().item() <= 0.03 * dxr.abs().max().item() + 1e-3
        assert (dw - dwr).abs().max().item() <= 0.03 * dwr.abs().max().item() + 1e-3
    torch.testing.assert_close(rm, rm_ref, rtol=1e-3, atol=1e-4)


def test_fused_resnet_stage_is_deterministic():
    """Two fused passes of the same ResNet-50 stage 1 (statistics from the conv epilogues, one writer per chunk,
    fixed-order folds) produce bit-identical outputs."""
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.vision.models import resnet50
    paddle.set_device("gpu:0")
    g = torch.Generator(device="cuda").manual_seed(2)
    x = torch.randn(8, 56, 56, 64, device="cuda", generator=g).bfloat16()
    CB._FEEDS_BN.clear()
    outs = []
    for _ in range(3):  # pass 1 learns the conv -> BN pairs, passes 2 and 3 are fused
        paddle.seed(5)
        stage = resnet50(num_classes=10, data_format="NHWC").layer1
        for p in stage.parameters():
            p._t.data = p._t.data.bfloat16() if p._t.dim() == 4 else p._t.data
        L.reset_calls()
        xb = paddle.Tensor(x.clone().requires_grad_(True))
        xb.stop_gradient = False
        y = stage(xb)
        y.astype("float32").sum().backward()
        torch.cuda.synchronize()
        outs.append((y._t.float().clone(), dict(L.CALLS)))
    assert outs[1][1].get("pa_bn_fwd_nhwc_pre", 0) > 0
    d = (outs[1][0] - outs[2][0]).abs().max().item()
    assert d == 0.0, f"fused passes differ by {d}"
