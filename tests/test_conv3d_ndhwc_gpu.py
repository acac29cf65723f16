"""3-D convolutions in NDHWC layout reach the hand-written implicit GEMM ("3-D convs never reach our
kernels"): the kernel's forward against PyTorch fp32 conv3d (every (kd, kh, kw) tap is one 64-channel K tile,
depth / height / width padding through the zero page), and the functional path end to end (forward + MIOpen
gradients)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

import paddlepaddle_amd as paddle  # noqa: E402
from paddlepaddle_amd.ops import _loader as L  # noqa: E402
from paddlepaddle_amd.ops import conv as C  # noqa: E402


def _rel(a, b):
    return (a.float() - b).abs().max().item() / (b.abs().max().item() + 1e-6)


@pytest.mark.parametrize("n,d,hw,cin,cout,k,stride,pad", [(2, 8, 16, 64, 64, 3, 1, 1), (1, 6, 12, 128, 96, 3, 2, 1),
                                                          (2, 4, 10, 64, 128, 1, 1, 0), (1, 9, 9, 64, 64, 3, 1, 0)])
def test_conv3d_implicit_gemm_forward_matches_fp32(n, d, hw, cin, cout, k, stride, pad):
    g = torch.Generator(device="cuda").manual_seed(d * hw + cin)
    x = torch.randn(n, d, hw, hw, cin, device="cuda", generator=g).bfloat16()
    w = (torch.randn(cout, cin, k, k, k, device="cuda", generator=g) / (cin * k ** 3) ** 0.5).bfloat16()
    L.reset_calls()
    y = C._conv3d_own(x, w, None, stride, (pad, pad, pad), 1)
    torch.cuda.synchronize()
    assert L.calls("pa_conv3d_ndhwc_fwd") == 1
    ref = torch.nn.functional.conv3d(x.float().permute(0, 4, 1, 2, 3), w.float(), None, stride, pad)
    ref = ref.permute(0, 2, 3, 4, 1)
    assert tuple(y.shape) == tuple(ref.shape)
    assert _rel(y, ref) < 2e-2


def test_conv3d_functional_ndhwc_forward_and_backward():
    paddle.set_device("gpu:0")
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(2, 6, 12, 12, 64, device="cuda", generator=g).bfloat16()
    w = (torch.randn(64, 64, 3, 3, 3, device="cuda", generator=g) * 0.02).bfloat16()
    xt = paddle.Tensor(x.clone().requires_grad_(True))
    xt.stop_gradient = False
    wt = paddle.Tensor(w.clone().requires_grad_(True))
    wt.stop_gradient = False
    y = paddle.nn.functional.conv3d(xt, wt, None, stride=1, padding=1, data_format="NDHWC")
    y.astype("float32").sum().backward()
    torch.cuda.synchronize()
    xr = x.float().permute(0, 4, 1, 2, 3).requires_grad_(True)
    wr = w.float().requires_grad_(True)
    yr = torch.nn.functional.conv3d(xr, wr, None, 1, 1)
    yr.sum().backward()
    assert _rel(y._t, yr.permute(0, 2, 3, 4, 1).detach()) < 2e-2
    assert _rel(xt.grad._t, xr.grad.permute(0, 2, 3, 4, 1)) < 3e-2
    assert _rel(wt.grad._t, wr.grad) < 3e-2


@pytest.mark.parametrize("cin,cout,k,pad", [(64, 64, 3, 1), (96, 128, 3, 1), (64, 64, 1, 0), (32, 64, 3, 0)])
def test_conv3d_data_gradient_on_implicit_gemm(cin, cout, k, pad):
    """Stride-1 data gradient on the hand-written kernel: dY convolved with the flipped, in/out-swapped filter
    (padding K - 1 - p) against PyTorch fp32 conv3d's input gradient."""
    g = torch.Generator(device="cuda").manual_seed(cin + cout + k)
    x = torch.randn(2, 6, 10, 10, cin, device="cuda", generator=g).bfloat16()
    w = (torch.randn(cout, cin, k, k, k, device="cuda", generator=g) / (cin * k ** 3) ** 0.5).bfloat16()
    Do = 6 + 2 * pad - (k - 1)
    Ho = 10 + 2 * pad - (k - 1)
    dy = torch.randn(2, Do, Ho, Ho, cout, device="cuda", generator=g).bfloat16()
    assert C._dgrad3d_own_ok(x, w, 1, (pad,) * 3, 1)
    L.reset_calls()
    gi = C._dgrad3d_own(dy, w, (pad,) * 3, 1)
    assert L.calls("pa_conv3d_ndhwc_fwd") == 1
    xr = x.float().permute(0, 4, 1, 2, 3).requires_grad_(True)
    torch.nn.functional.conv3d(xr, w.float(), None, 1, pad).backward(dy.float().permute(0, 4, 1, 2, 3))
    ref = xr.grad.permute(0, 2, 3, 4, 1)
    assert tuple(gi.shape) == tuple(ref.shape)
    assert _rel(gi, ref) < 2e-2
