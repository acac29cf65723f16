"""Per-direction NHWC convolution (ops/conv.py _ConvNHWC): every combination of hand-written / MIOpen forward,
data gradient and weight gradient against an fp32 PyTorch reference of the same convolution, and the residual
gradient hand-off (ResidualGradSink) on either data-gradient backend."""
import itertools

import pytest
import torch

pytestmark = pytest.mark.gpu

from paddlepaddle_amd.ops import _loader as L  # noqa: E402
from paddlepaddle_amd.ops import conv as C  # noqa: E402


def _ref(x, w, b, stride, pad, dy):
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.float().requires_grad_(True)
    y = torch.nn.functional.conv2d(xr, wr, None if b is None else b.float(), stride, pad)
    y.backward(dy.float().permute(0, 3, 1, 2))
    return y.permute(0, 2, 3, 1), xr.grad.permute(0, 2, 3, 1), wr.grad


def _close(got, exp, what):
    scale = exp.abs().max().item() + 1e-6
    err = (got.float() - exp).abs().max().item() / scale
    assert err < 2e-2, f"{what}: max rel err {err:.3g}"


@pytest.mark.parametrize("k,stride,cin,cout,hw", [(1, 1, 64, 128, 14), (1, 2, 128, 64, 14), (3, 1, 64, 64, 12),
                                                 (3, 2, 64, 128, 12)])
@pytest.mark.parametrize("combo", list(itertools.product(["hip", "blas"], repeat=3)))
def test_conv_nhwc_per_direction(monkeypatch, k, stride, cin, cout, hw, combo):
    forced = dict(zip(("convf", "convd", "convw"), combo))
    monkeypatch.setattr(C, "_pick", lambda key, own, mi, skinny=None, mm=None: forced[key[0]])
    g = torch.Generator(device="cuda").manual_seed(k * 10 + stride)
    x = torch.randn(4, hw, hw, cin, device="cuda", generator=g).bfloat16()
    w = (torch.randn(cout, cin, k, k, device="cuda", generator=g) * 0.1).bfloat16()
    pad = k // 2
    assert C.eligible_nhwc(x, w, 1)
    xx = x.clone().requires_grad_(True)
    ww = w.clone().requires_grad_(True)
    L.CALLS.clear()
    y = C.conv2d_nhwc(xx, ww, None, stride, pad, 1)
    dy = torch.randn(y.shape, device="cuda", generator=g).bfloat16()
    y.backward(dy)
    yr, dxr, dwr = _ref(x, w, None, stride, pad, dy)
    _close(y, yr, "y")
    _close(xx.grad, dxr, "dx")
    _close(ww.grad, dwr, "dw")
    assert ww.grad.shape == w.shape and xx.grad.shape == x.shape
    own = [combo[0] == "hip", combo[1] == "hip" and C._own_dgrad_ok(x, w, stride, pad, 1),
           combo[2] == "hip" and C._own_wgrad_ok(x, w, dy)]
    if any(own):
        assert sum(L.CALLS.values()) > 0, "no hand-written launch although a direction was forced to it"


@pytest.mark.parametrize("dgrad", ["hip", "blas"])
def test_conv_nhwc_residual_sink(monkeypatch, dgrad):
    """A d(residual) parked in the sink is added to dx whichever backend computes the data gradient."""
    forced = {"convf": "hip", "convd": dgrad, "convw": "hip"}
    monkeypatch.setattr(C, "_pick", lambda key, own, mi, skinny=None, mm=None: forced[key[0]])
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(2, 8, 8, 128, device="cuda", generator=g).bfloat16()
    w = (torch.randn(64, 128, 1, 1, device="cuda", generator=g) * 0.1).bfloat16()
    dres = torch.randn(2, 8, 8, 128, device="cuda", generator=g).bfloat16()
    xx = x.clone().requires_grad_(True)
    with C.residual_grad_sink() as s:
        y = C.conv2d_nhwc(xx, w, None, 1, 0, 1)
    assert s.armed
    s.dres = dres.clone()
    dy = torch.randn(y.shape, device="cuda", generator=g).bfloat16()
    y.backward(dy)
    _, dxr, _ = _ref(x, w, None, 1, 0, dy)
    _close(xx.grad, dxr + dres.float(), "dx + dres")


@pytest.mark.parametrize("cin,cout", [(64, 256), (256, 64), (64, 64)])
def test_conv_nhwc_skinny_1x1(monkeypatch, cin, cout):
    """1x1 forward and data gradient on the memory-bound kernel (gemm_skinny), with the residual sink."""
    forced = {"convf": "skinny", "convd": "skinny", "convw": "hip"}
    monkeypatch.setattr(C, "_pick", lambda key, own, mi, skinny=None, mm=None: forced[key[0]])
    g = torch.Generator(device="cuda").manual_seed(cin + cout)
    x = torch.randn(4, 16, 16, cin, device="cuda", generator=g).bfloat16()
    w = (torch.randn(cout, cin, 1, 1, device="cuda", generator=g) * 0.1).bfloat16()
    dres = torch.randn(x.shape, device="cuda", generator=g).bfloat16()
    assert C._skinny_ok(x, w, 1, False) and C._skinny_ok(x, w, 1, True)
    xx = x.clone().requires_grad_(True)
    ww = w.clone().requires_grad_(True)
    L.CALLS.clear()
    with C.residual_grad_sink() as s:
        y = C.conv2d_nhwc(xx, ww, None, 1, 0, 1)
    s.dres = dres.clone()
    dy = torch.randn(y.shape, device="cuda", generator=g).bfloat16()
    y.backward(dy)
    assert L.calls("pa_gemm_skinny") == 2
    yr, dxr, dwr = _ref(x, w, None, 1, 0, dy)
    _close(y, yr, "y")
    _close(xx.grad, dxr + dres.float(), "dx + dres")
    _close(ww.grad, dwr, "dw")


@pytest.mark.parametrize("stride", [1, 2])
def test_conv_nhwc_skinny_3x3(monkeypatch, stride):
    """3x3 C=Cout=64 forward (stride 1 / 2) and stride-1 data gradient on the skinny implicit-GEMM kernel, padding
    taps read as zeros past the buffer end."""
    forced = {"convf": "skinny", "convd": "skinny", "convw": "hip"}
    monkeypatch.setattr(C, "_pick", lambda key, own, mi, skinny=None, mm=None: forced[key[0]] if skinny is not None or
                        forced[key[0]] != "skinny" else "hip")
    g = torch.Generator(device="cuda").manual_seed(7 + stride)
    x = torch.randn(3, 15, 13, 64, device="cuda", generator=g).bfloat16()
    w = (torch.randn(64, 64, 3, 3, device="cuda", generator=g) * 0.05).bfloat16()
    assert C._skinny_ok(x, w, stride, False, 1, 1) and C._skinny_ok(x, w, 1, True, 1, 1)
    xx = x.clone().requires_grad_(True)
    ww = w.clone().requires_grad_(True)
    L.CALLS.clear()
    y = C.conv2d_nhwc(xx, ww, None, stride, 1, 1)
    dy = torch.randn(y.shape, device="cuda", generator=g).bfloat16()
    y.backward(dy)
    assert L.calls("pa_conv_skinny") == (2 if stride == 1 else 1)
    yr, dxr, dwr = _ref(x, w, None, stride, 1, dy)
    _close(y, yr, "y")
    _close(xx.grad, dxr, "dx")
    _close(ww.grad, dwr, "dw")


@pytest.mark.parametrize("stride", [1, 2])
def test_conv_nhwc_mm_1x1(monkeypatch, stride):
    """1x1 forward / data gradient as hipBLASLt GEMMs (the 'mm' candidate), incl. the residual sink at stride 1."""
    forced = {"convf": "mm", "convd": "mm", "convw": "hip"}
    monkeypatch.setattr(C, "_pick", lambda key, own, mi, skinny=None, mm=None: forced[key[0]] if mm is not None
                        else "hip")
    g = torch.Generator(device="cuda").manual_seed(11 + stride)
    x = torch.randn(4, 16, 16, 128, device="cuda", generator=g).bfloat16()
    w = (torch.randn(64, 128, 1, 1, device="cuda", generator=g) * 0.1).bfloat16()
    dres = torch.randn(x.shape, device="cuda", generator=g).bfloat16()
    xx = x.clone().requires_grad_(True)
    ww = w.clone().requires_grad_(True)
    with C.residual_grad_sink() as s:
        y = C.conv2d_nhwc(xx, ww, None, stride, 0, 1)
    if stride == 1:
        s.dres = dres.clone()
    dy = torch.randn(y.shape, device="cuda", generator=g).bfloat16()
    y.backward(dy)
    yr, dxr, dwr = _ref(x, w, None, stride, 0, dy)
    _close(y, yr, "y")
    _close(xx.grad, dxr + (dres.float() if stride == 1 else 0), "dx")
    _close(ww.grad, dwr, "dw")


@pytest.mark.parametrize("hw", [(15, 16), (12, 40), (8, 64)])
def test_conv_nhwc_skinny_wgrad_3x3(monkeypatch, hw):
    """3x3 C=Cout=64 weight gradient on the halo-tile kernel (transposed LDS reads of dY and the input window,
    fp32 slabs per workgroup) against the fp32 reference, incl. rows wider than one 32-pixel piece."""
    forced = {"convf": "hip", "convd": "hip", "convw": "skinny"}
    monkeypatch.setattr(C, "_pick", lambda key, own, mi, skinny=None, mm=None:
                        forced[key[0]] if (skinny is not None or forced[key[0]] != "skinny") else "hip")
    g = torch.Generator(device="cuda").manual_seed(hw[1])
    x = torch.randn(4, hw[0], hw[1], 64, device="cuda", generator=g).bfloat16()  # 4 * H * W pixels: multiple of 64
    w = (torch.randn(64, 64, 3, 3, device="cuda", generator=g) * 0.05).bfloat16()
    xx = x.clone().requires_grad_(True)
    ww = w.clone().requires_grad_(True)
    L.CALLS.clear()
    y = C.conv2d_nhwc(xx, ww, None, 1, 1, 1)
    dy = torch.randn(y.shape, device="cuda", generator=g).bfloat16()
    y.backward(dy)
    assert L.calls("pa_conv_skinny_wgrad") == 1
    _, dxr, dwr = _ref(x, w, None, 1, 1, dy)
    _close(ww.grad, dwr, "dw")
    _close(xx.grad, dxr, "dx")
