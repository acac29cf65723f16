"""Gradient-accumulation fusion for biases and norm parameters: the HIP finalize kernels (pa_colsum,
pa_bias_gelu_bwd, pa_reduce_parts with the accumulate bit) add the parameter gradient straight into a registered
buffer, like the weight-gradient GEMM does for weights (ops/linear.py register_main_grad). Checked against an
fp32 PyTorch reference of the same ops."""
import pytest
import torch

from paddlepaddle_amd.ops import linear as LIN
from paddlepaddle_amd.ops import norm as NORM
from paddlepaddle_amd.ops import _loader as L

pytestmark = pytest.mark.gpu


def _reg(p):
    buf = torch.full_like(p, 0.5)
    seen = []
    LIN.register_main_grad(p, buf, lambda t: seen.append(t))
    return buf, seen


@pytest.mark.parametrize("act", [None, "gelu"])
def test_linear_bias_accumulates_in_place(act):
    torch.manual_seed(0)
    dev = "cuda"
    x = torch.randn(256, 128, device=dev, dtype=torch.bfloat16, requires_grad=True)
    w = torch.randn(128, 192, device=dev, dtype=torch.bfloat16).mul_(0.05).requires_grad_()
    b = torch.randn(192, device=dev, dtype=torch.bfloat16).mul_(0.1).requires_grad_()
    wbuf, wseen = _reg(w)
    bbuf, bseen = _reg(b)
    try:
        y = LIN.fused_linear(x, w, b, act=act)
        dy = torch.randn_like(y)
        y.backward(dy)
        torch.cuda.synchronize()
        assert L._LIB is not None
        xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
        yr = xr @ wr + br
        if act == "gelu":
            yr = torch.nn.functional.gelu(yr, approximate="tanh")
        yr.backward(dy.float())
        assert b.grad is None and w.grad is None  # nothing went through autograd accumulation
        assert bseen == [b] and wseen == [w]
        torch.testing.assert_close(bbuf.float(), 0.5 + br.grad, rtol=2e-2, atol=2e-1)
        torch.testing.assert_close(wbuf.float(), 0.5 + wr.grad, rtol=2e-2, atol=2e-1)
    finally:
        LIN.unregister_main_grad(w)
        LIN.unregister_main_grad(b)


def test_layer_norm_params_accumulate_in_place():
    torch.manual_seed(1)
    x = torch.randn(512, 256, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(256, device="cuda")).to(torch.bfloat16).requires_grad_()
    b = (0.1 * torch.randn(256, device="cuda")).to(torch.bfloat16).requires_grad_()
    wbuf, wseen = _reg(w)
    bbuf, bseen = _reg(b)
    try:
        y = NORM.layer_norm(x, w, b, 1e-5)
        dy = torch.randn_like(y)
        y.backward(dy)
        torch.cuda.synchronize()
        xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
        torch.nn.functional.layer_norm(xr, (256,), wr, br, 1e-5).backward(dy.float())
        assert w.grad is None and b.grad is None and wseen == [w] and bseen == [b]
        torch.testing.assert_close(wbuf.float(), 0.5 + wr.grad, rtol=2e-2, atol=2e-1)
        torch.testing.assert_close(bbuf.float(), 0.5 + br.grad, rtol=2e-2, atol=2e-1)
        torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=5e-2)
    finally:
        LIN.unregister_main_grad(w)
        LIN.unregister_main_grad(b)


def test_rms_norm_weight_accumulates_in_place():
    torch.manual_seed(2)
    x = torch.randn(384, 256, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(256, device="cuda")).to(torch.bfloat16).requires_grad_()
    wbuf, wseen = _reg(w)
    try:
        y = NORM.rms_norm(x, w, 1e-6)
        dy = torch.randn_like(y)
        y.backward(dy)
        torch.cuda.synchronize()
        xr, wr = (t.detach().float().requires_grad_() for t in (x, w))
        (xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6) * wr).backward(dy.float())
        assert w.grad is None and wseen == [w]
        torch.testing.assert_close(wbuf.float(), 0.5 + wr.grad, rtol=2e-2, atol=2e-1)
    finally:
        LIN.unregister_main_grad(w)
