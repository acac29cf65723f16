"""Depthwise NHWC convolution HIP kernels (csrc/kernels/dwconv.hip) against the fp32 torch reference
conv2d(groups=C): forward, data / weight / bias gradients, strides, padding, dilation, 3x3 .. 7x7 filters."""
import pytest
import torch
import torch.nn.functional as F

import paddlepaddle_amd as paddle
from paddlepaddle_amd.ops import _loader as L

CASES = [  # N, H, W, C, K, stride, pad, dil, bias
    (2, 17, 19, 32, 3, 1, 1, 1, True),
    (3, 28, 28, 96, 3, 2, 1, 1, False),
    (2, 14, 14, 144, 5, 1, 2, 1, True),
    (1, 23, 20, 64, 7, 2, 3, 1, True),
    (2, 16, 16, 40, 3, 1, 2, 2, False),
]


def _run(dev, dt, case, through_paddle):
    N, H, W, C, K, s, p, d, bias = case
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, H, W, C, generator=g)
    w = torch.randn(C, 1, K, K, generator=g) * 0.3
    b = torch.randn(C, generator=g) if bias else None
    dy_seed = torch.randn(1, generator=g)
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True) if bias else None
    yr = F.conv2d(xr.permute(0, 3, 1, 2), wr, br, s, p, d, C).permute(0, 2, 3, 1)
    gy = torch.cos(yr.detach() + dy_seed)
    yr.backward(gy)
    xt = paddle.to_tensor(x.to(dev, dt), stop_gradient=False)
    wt = paddle.to_tensor(w.to(dev, dt), stop_gradient=False)
    bt = paddle.to_tensor(b.to(dev, dt), stop_gradient=False) if bias else None
    y = paddle.nn.functional.conv2d(xt, wt, bt, s, p, d, C, data_format="NHWC")
    y.backward(paddle.to_tensor(gy.to(dev, dt)))
    tol = 2e-2 if dt == torch.bfloat16 else 1e-4
    for got, ref in ((y._t, yr), (xt.grad._t, xr.grad), (wt.grad._t, wr.grad)) + \
            (((bt.grad._t, br.grad),) if bias else ()):
        err = (got.float().cpu() - ref).abs().max().item()
        assert err <= tol * max(1.0, ref.abs().max().item()), (case, err)


@pytest.mark.parametrize("case", CASES[:2])
def test_depthwise_nhwc_matches_reference_cpu(case):
    _run("cpu", torch.float32, case, True)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("case", CASES)
def test_depthwise_nhwc_hip_kernels(case, dt):
    paddle.set_flags({"FLAGS_gemm_backend": "hip"})
    try:
        L.CALLS.clear()
        _run("cuda", dt, case, True)
        for n in ("pa_dwconv_fwd", "pa_dwconv_dgrad", "pa_dwconv_wgrad"):
            assert L.calls(n) > 0, (n, dict(L.CALLS))
    finally:
        paddle.set_flags({"FLAGS_gemm_backend": "auto"})


@pytest.mark.gpu
@pytest.mark.parametrize("K,pad", [(3, 1), (1, 0), (3, 0)])
def test_conv2d_transpose_stride1_nhwc_on_conv_kernels(K, pad):
    """NHWC stride-1 conv2d_transpose runs as a convolution with the flipped / swapped filter (hand-written
    implicit GEMM or 1x1 GEMM path); values and gradients against torch conv_transpose2d in fp32."""
    paddle.set_flags({"FLAGS_gemm_backend": "hip"})
    try:
        g = torch.Generator().manual_seed(1)
        x = torch.randn(2, 12, 12, 64, generator=g)
        w = torch.randn(64, 128, K, K, generator=g) * 0.05  # [Cin, Cout, K, K]
        xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
        yr = F.conv_transpose2d(xr.permute(0, 3, 1, 2), wr, None, 1, pad).permute(0, 2, 3, 1)
        gy = torch.cos(yr.detach())
        yr.backward(gy)
        xt = paddle.to_tensor(x.cuda().bfloat16(), stop_gradient=False)
        wt = paddle.to_tensor(w.cuda().bfloat16(), stop_gradient=False)
        L.CALLS.clear()
        y = paddle.nn.functional.conv2d_transpose(xt, wt, None, 1, pad, data_format="NHWC")
        y.backward(paddle.to_tensor(gy.cuda().bfloat16()))
        assert sum(L.CALLS.values()) > 0, "no hand-written kernel ran"
        for got, ref in ((y._t, yr), (xt.grad._t, xr.grad), (wt.grad._t, wr.grad)):
            err = (got.float().cpu() - ref).abs().max().item()
            assert err <= 3e-2 * max(1.0, ref.abs().max().item()), err
    finally:
        paddle.set_flags({"FLAGS_gemm_backend": "auto"})


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("case", [CASES[0], CASES[1], CASES[4]])
def test_relu_depthwise_fused_hip_kernels(case, dt):
    """ops.fused_conv.relu_depthwise_conv2d (the fuse_relu_depthwise_conv node): the ReLU on the kernels' loads and
    as the data-gradient mask, against relu + conv2d in fp32 — values and x / w / b gradients."""
    from paddlepaddle_amd.ops.fused_conv import relu_depthwise_conv2d
    N, H, W, C, K, s, p, d, bias = case
    g = torch.Generator().manual_seed(2)
    x = torch.randn(N, H, W, C, generator=g)
    w = torch.randn(C, 1, K, K, generator=g) * 0.3
    b = torch.randn(C, generator=g) if bias else None
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True) if bias else None
    yr = F.conv2d(torch.relu(xr.permute(0, 3, 1, 2)), wr, br, s, p, d, C)
    gy = torch.cos(yr.detach())
    yr.backward(gy)
    paddle.set_flags({"FLAGS_gemm_backend": "hip"})
    try:
        L.CALLS.clear()
        xc, wc = x.cuda().to(dt).requires_grad_(True), w.cuda().to(dt).requires_grad_(True)
        bc = b.cuda().to(dt).requires_grad_(True) if bias else None
        y = relu_depthwise_conv2d(xc, wc, bc, s, p, d, C, True)
        y.backward(gy.cuda().to(dt))
        for n in ("pa_dwconv_fwd", "pa_dwconv_dgrad", "pa_dwconv_wgrad"):
            assert L.calls(n) > 0, (n, dict(L.CALLS))
    finally:
        paddle.set_flags({"FLAGS_gemm_backend": "auto"})
    tol = 2e-2 if dt == torch.bfloat16 else 1e-4
    for got, ref in ((y, yr), (xc.grad.permute(0, 3, 1, 2), xr.grad.permute(0, 3, 1, 2)), (wc.grad, wr.grad)) + \
            (((bc.grad, br.grad),) if bias else ()):
        err = (got.float().cpu() - ref).abs().max().item()
        assert err <= tol * max(1.0, ref.abs().max().item()), (case, err)
