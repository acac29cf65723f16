"""1-D convolutions in NLC layout on the NHWC hand-written kernels ("1-D convs never reach our
kernels"): a 1 x L image with a 1 x K filter and padding (0, p); forward and weight gradient on the implicit GEMM,
the data gradient of the 1 x K filter on MIOpen. Compared with PyTorch fp32 conv1d."""
import pytest
import torch

pytestmark = pytest.mark.gpu

import paddlepaddle_amd as paddle  # noqa: E402
from paddlepaddle_amd.ops import _loader as L  # noqa: E402


@pytest.mark.parametrize("n,l,cin,cout,k,pad,stride", [(4, 200, 64, 128, 3, 1, 1), (2, 512, 128, 64, 5, 2, 1),
                                                       (3, 97, 64, 64, 1, 0, 1), (2, 160, 64, 96, 3, 1, 2)])
def test_conv1d_nlc_hip_matches_fp32(n, l, cin, cout, k, pad, stride):
    paddle.set_device("gpu:0")
    g = torch.Generator(device="cuda").manual_seed(l + k)
    x = torch.randn(n, l, cin, device="cuda", generator=g).bfloat16()
    w = (torch.randn(cout, cin, k, device="cuda", generator=g) / (cin * k) ** 0.5).bfloat16()
    xt = paddle.Tensor(x.clone().requires_grad_(True))
    xt.stop_gradient = False
    wt = paddle.Tensor(w.clone().requires_grad_(True))
    wt.stop_gradient = False
    L.reset_calls()
    y = paddle.nn.functional.conv1d(xt, wt, None, stride=stride, padding=pad, data_format="NLC")
    gy = torch.randn(tuple(y.shape), device="cuda", generator=g)
    y.astype("float32").backward(paddle.Tensor(gy))
    torch.cuda.synchronize()
    assert sum(L.CALLS.values()) > 0, "no hand-written kernel ran"
    xr = x.float().permute(0, 2, 1).requires_grad_(True)
    wr = w.float().requires_grad_(True)
    yr = torch.nn.functional.conv1d(xr, wr, None, stride, pad)
    yr.backward(gy.permute(0, 2, 1))

    def rel(a, b):
        return (a.float() - b).abs().max().item() / (b.abs().max().item() + 1e-6)
    assert tuple(y.shape) == tuple(yr.permute(0, 2, 1).shape)
    assert rel(y._t, yr.permute(0, 2, 1).detach()) < 2e-2
    assert rel(xt.grad._t, xr.grad.permute(0, 2, 1)) < 2e-2
    assert rel(wt.grad._t, wr.grad) < 2e-2
