"""Numerics of every hand-written HIP kernel against a plain PyTorch fp32 reference of the same op.
Each test also asserts the native library is the code path that ran."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from paddlepaddle_amd import ops  # noqa: E402
from paddlepaddle_amd.ops import _loader as L  # noqa: E402

DEV = "cuda"


def _lib_loaded(*launchers):
    """The native library is loaded and each named launcher actually dispatched (ops._loader.CALLS;
    the counters are reset per test by conftest)."""
    assert L._LIB is not None, "HIP kernel library not loaded"
    for n in launchers:
        assert L.calls(n) > 0, f"{n} did not run (calls: {dict(L.CALLS)})"
    if not launchers:
        assert sum(L.CALLS.values()) > 0, "no HIP launcher ran"


def _tol(dt):
    return {torch.float32: 2e-5, torch.bfloat16: 2e-2, torch.float16: 2e-3}[dt]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("cols", [64, 512, 1000, 5120, 12288])
def test_rms_norm(dt, cols):
    torch.manual_seed(0)
    x = torch.randn(37, cols, device=DEV, dtype=dt, requires_grad=True)
    w = (torch.rand(cols, device=DEV) + 0.5).to(dt).requires_grad_(True)
    if cols % 8:
        pytest.skip("cols must be a multiple of 8 for the HIP path")
    y = ops.rms_norm(x, w, 1e-6)
    _lib_loaded("pa_rms_norm_fwd")
    xr, wr = x.detach().float().requires_grad_(True), w.detach().float().requires_grad_(True)
    yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6) * wr
    torch.testing.assert_close(y.float(), yr, atol=_tol(dt) * 4, rtol=_tol(dt))
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    yr.backward(g)
    _lib_loaded("pa_rms_norm_bwd")
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=_tol(dt) * 8, rtol=_tol(dt) * 2)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=_tol(dt) * 40, rtol=_tol(dt) * 4)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cols,shift", [(256, 1.0), (3072, 1.0), (4096, 1.0), (5120, 1.0), (16384, 1.0),
                                        (5120, 300.0), (3072, 300.0)])
def test_layer_norm(dt, cols, shift):
    """Wave-per-row kernels up to 3072 columns, workgroup-per-row kernels above; shift = 300: rows whose mean is
    large against their spread (the wide kernel's shifted moments must not cancel)."""
    torch.manual_seed(1)
    x = (torch.randn(29, cols, device=DEV) * 3 + shift).to(dt).requires_grad_(True)
    w = torch.randn(cols, device=DEV).to(dt).requires_grad_(True)
    b = torch.randn(cols, device=DEV).to(dt).requires_grad_(True)
    y = ops.layer_norm(x, w, b, 1e-5)
    _lib_loaded("pa_layer_norm_fwd")
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = F.layer_norm(xr, (cols,), wr, br, 1e-5)
    # forward against a float64 reference (an fp32 LayerNorm of rows with mean 300 is itself ~1e-4 off)
    y64 = F.layer_norm(xr.detach().double(), (cols,), wr.detach().double(), br.detach().double(), 1e-5)
    torch.testing.assert_close(y.double(), y64, atol=_tol(dt) * 8, rtol=_tol(dt))
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    yr.backward(g)
    _lib_loaded("pa_layer_norm_bwd")
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=_tol(dt) * 10, rtol=_tol(dt) * 2)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=_tol(dt) * 60, rtol=_tol(dt) * 4)
    torch.testing.assert_close(b.grad.float(), br.grad, atol=_tol(dt) * 60, rtol=_tol(dt) * 4)


@pytest.mark.parametrize("op", ["layer_norm", "rms_norm"])
def test_norm_without_affine_params(op):
    """weight = bias = None (paddle.nn.functional.layer_norm(x, shape)): the kernels take null pointers and
    the backward produces no parameter gradients."""
    torch.manual_seed(2)
    x = torch.randn(33, 512, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = ops.layer_norm(x, None, None, 1e-5) if op == "layer_norm" else ops.rms_norm(x, None, 1e-6)
    xr = x.detach().float().requires_grad_(True)
    yr = F.layer_norm(xr, (512,), None, None, 1e-5) if op == "layer_norm" else \
        xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    _lib_loaded(f"pa_{op}_fwd", f"pa_{op}_bwd")
    torch.testing.assert_close(y.float(), yr, atol=0.05, rtol=0.02)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=0.1, rtol=0.04)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cols", [8, 128, 4096, 50304])
def test_softmax(dt, cols):
    x = (torch.randn(13, cols, device=DEV) * 4).to(dt).requires_grad_(True)
    y = ops.softmax(x, -1)
    _lib_loaded("pa_softmax_fwd")
    xr = x.detach().float().requires_grad_(True)
    yr = torch.softmax(xr, -1)
    torch.testing.assert_close(y.float(), yr, atol=_tol(dt), rtol=_tol(dt) * 2)
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=_tol(dt) * 2, rtol=_tol(dt) * 4)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("V", [64, 50304])
def test_softmax_cross_entropy(dt, V):
    torch.manual_seed(3)
    logits = (torch.randn(33, V, device=DEV) * 3).to(dt).requires_grad_(True)
    labels = torch.randint(0, V, (33,), device=DEV)
    labels[5] = -100
    l = ops.softmax_cross_entropy(logits, labels, -100)
    _lib_loaded("pa_softmax_ce_fwd")
    lr = logits.detach().float().requires_grad_(True)
    ref = F.cross_entropy(lr, labels, ignore_index=-100, reduction="none")
    torch.testing.assert_close(l, ref, atol=1e-3 if dt == torch.float32 else 3e-2, rtol=1e-3)
    g = torch.rand(33, device=DEV)
    l.backward(g)
    ref.backward(g)
    torch.testing.assert_close(logits.grad.float(), lr.grad, atol=1e-5 if dt == torch.float32 else 3e-3,
                               rtol=1e-3 if dt == torch.float32 else 3e-2)


@pytest.mark.parametrize("approx", [False, True])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gelu(approx, dt):
    x = (torch.randn(4, 1024, device=DEV) * 3).to(dt).requires_grad_(True)
    y = ops.gelu(x, approx)
    _lib_loaded("pa_gelu_fwd")
    xr = x.detach().float().requires_grad_(True)
    yr = F.gelu(xr, approximate="tanh" if approx else "none")
    torch.testing.assert_close(y.float(), yr, atol=_tol(dt) * 2, rtol=_tol(dt))
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=_tol(dt) * 4, rtol=_tol(dt) * 2)


def test_bias_gelu():
    x = torch.randn(64, 2048, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(2048, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = ops.bias_gelu(x, b)
    _lib_loaded("pa_bias_gelu_fwd")
    xr, br = x.detach().float().requires_grad_(True), b.detach().float().requires_grad_(True)
    yr = F.gelu(xr + br, approximate="tanh")
    torch.testing.assert_close(y.float(), yr, atol=4e-2, rtol=2e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=6e-2, rtol=3e-2)
    torch.testing.assert_close(b.grad.float(), br.grad, atol=0.5, rtol=3e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_swiglu_packed(dt):
    xy = torch.randn(40, 2 * 512, device=DEV).to(dt).requires_grad_(True)
    a, b = xy.chunk(2, -1)
    y = ops.swiglu(a, b)
    _lib_loaded("pa_swiglu_fwd")
    xr = xy.detach().float().requires_grad_(True)
    ar, br = xr.chunk(2, -1)
    yr = F.silu(ar) * br
    torch.testing.assert_close(y.float(), yr, atol=_tol(dt) * 4, rtol=_tol(dt))
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    yr.backward(g)
    torch.testing.assert_close(xy.grad.float(), xr.grad, atol=_tol(dt) * 4, rtol=_tol(dt) * 2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_swiglu_one_input(dt):
    """swiglu(x) with x = [gate | up]: one-buffer gradient straight from the kernel (no autograd cat)."""
    xy = torch.randn(3, 40, 2 * 512, device=DEV).to(dt).requires_grad_(True)
    y = ops.swiglu(xy)
    _lib_loaded("pa_swiglu_fwd")
    assert type(y.grad_fn).__name__ == "_SwigluPackedHIPBackward"
    xr = xy.detach().float().requires_grad_(True)
    ar, br = xr.chunk(2, -1)
    yr = F.silu(ar) * br
    torch.testing.assert_close(y.float(), yr, atol=_tol(dt) * 4, rtol=_tol(dt))
    g = torch.randn_like(yr)
    y.backward(g.to(dt))
    yr.backward(g)
    torch.testing.assert_close(xy.grad.float(), xr.grad, atol=_tol(dt) * 4, rtol=_tol(dt) * 2)


@pytest.mark.parametrize("neox", [True, False])
def test_rope(neox):
    from paddlepaddle_amd.ops.rope import rope_tables, _rotate_ref
    B, S, H, D = 2, 64, 4, 128
    cos, sin = rope_tables(S, D, device=DEV, neox=neox)
    x = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = ops.apply_rotary(x, cos, sin, neox)
    _lib_loaded("pa_rope_fwd")
    xr = x.detach().float().requires_grad_(True)
    yr = _rotate_ref(xr, cos, sin, neox, False)
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=2e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=5e-2, rtol=3e-2)


def test_adamw_multi_tensor_master_weights():
    import paddlepaddle_amd as paddle
    torch.manual_seed(5)
    shapes = [(1000,), (33, 17), (4096, 8), (7,)]
    ps = [paddle.Parameter(torch.randn(s, device=DEV).bfloat16()) for s in shapes]
    ref = [p._t.detach().float().clone().requires_grad_(True) for p in ps]
    opt = paddle.optimizer.AdamW(1e-2, parameters=ps, weight_decay=0.1, multi_precision=True)
    topt = torch.optim.AdamW(ref, lr=1e-2, weight_decay=0.1, eps=1e-8)
    for step in range(3):
        gs = [torch.randn(s, device=DEV) for s in shapes]
        for p, g in zip(ps, gs):
            p._t.grad = g.bfloat16()
        for r, g in zip(ref, gs):
            r.grad = g.bfloat16().float()
        opt.step()
        topt.step()
    _lib_loaded("pa_adamw_multi")
    for p, r in zip(ps, ref):
        m = opt._master_weights[id(p)]
        torch.testing.assert_close(m, r.detach(), atol=2e-5, rtol=1e-5)
        torch.testing.assert_close(p._t.float(), r.detach(), atol=1e-2, rtol=1e-2)


def test_global_norm_multi():
    from paddlepaddle_amd.ops.optim import global_sq_norm
    ts = [torch.randn(n, device=DEV, dtype=dt) for n, dt in [(100000, torch.float32), (333, torch.bfloat16),
                                                              (70000, torch.bfloat16)]]
    got = global_sq_norm(ts)
    _lib_loaded("pa_sq_norm_multi")
    ref = sum(t.float().pow(2).sum() for t in ts)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-3)


@pytest.fixture(params=["hip", "blas"])
def gemm_backend(request):
    from paddlepaddle_amd.framework.flags import get_flags, set_flags
    old = get_flags(["FLAGS_gemm_backend"])["FLAGS_gemm_backend"]
    set_flags({"FLAGS_gemm_backend": request.param})
    yield request.param
    set_flags({"FLAGS_gemm_backend": old})


def _gemm_dispatch(backend):
    if backend == "hip":
        _lib_loaded("pa_gemm_bf16")
    else:
        assert L.calls("pa_gemm_bf16") == 0, "FLAGS_gemm_backend=blas must not run the hand-written GEMM"


def test_linear_fused_bias_grad(gemm_backend):
    x = torch.randn(4, 96, 256, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(256, 512, device=DEV) * 0.05).bfloat16().requires_grad_(True)
    b = torch.randn(512, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = ops.fused_linear(x, w, b)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = xr @ wr + br
    torch.testing.assert_close(y.float(), yr, atol=5e-2, rtol=2e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    torch.testing.assert_close(b.grad.float(), br.grad, atol=0.5, rtol=2e-2)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=0.5, rtol=3e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=0.1, rtol=3e-2)
    _gemm_dispatch(gemm_backend)


def test_linear_bias_gelu_fused(gemm_backend):
    x = torch.randn(128, 256, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(256, 1024, device=DEV) * 0.05).bfloat16().requires_grad_(True)
    b = torch.randn(1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = ops.fused_linear(x, w, b, act="gelu")
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = F.gelu(xr @ wr + br, approximate="tanh")
    torch.testing.assert_close(y.float(), yr, atol=5e-2, rtol=3e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    torch.testing.assert_close(b.grad.float(), br.grad, atol=0.6, rtol=3e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=0.15, rtol=3e-2)
    _gemm_dispatch(gemm_backend)


def test_colsum():
    x = torch.randn(3000, 5120, device=DEV, dtype=torch.bfloat16)
    got = ops.colsum(x)
    _lib_loaded("pa_colsum")
    torch.testing.assert_close(got.float(), x.float().sum(0), atol=0.3, rtol=1e-2)


def test_dropout_add_statistics_and_grad():
    torch.manual_seed(0)
    x = torch.ones(1 << 20, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    r = torch.zeros(1 << 20, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = ops.dropout_add(x, r, 0.1, True)
    _lib_loaded("pa_dropout_add_fwd")
    kept = (y != 0).float().mean().item()
    assert abs(kept - 0.9) < 0.005
    vals = y[y != 0].float()
    assert torch.allclose(vals, torch.full_like(vals, 1 / 0.9), rtol=1e-2)
    y.backward(torch.ones_like(y))
    # grad mask == forward mask, scaled
    torch.testing.assert_close(x.grad.float(), y.detach().float(), atol=1e-2, rtol=1e-2)
    assert torch.all(r.grad == 1)
    # recompute determinism: same seed state -> same mask
    torch.manual_seed(5)
    a = ops.dropout_add(x.detach(), None, 0.3, True)
    torch.manual_seed(5)
    b = ops.dropout_add(x.detach(), None, 0.3, True)
    assert torch.equal(a, b)


def test_dropout_backward_writes_linear_bias_grad_partials():
    """linear(+bias) -> dropout_add: after the first backward the dropout backward writes the column partials of
    its gradient and the linear only folds them; the bias gradient equals the plain column sum, and the dropout
    mask matches the unfused kernel (same seed)."""
    from paddlepaddle_amd.ops import dropout as D
    torch.manual_seed(0)
    rows, k, n = 1000, 64, 96
    x = torch.randn(rows, k, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(k, n, device=DEV) / 8).to(torch.bfloat16).requires_grad_(True)
    b = torch.zeros(n, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    gy = torch.randn(rows, n, device=DEV, dtype=torch.bfloat16)
    D._WANT_CS.discard((rows, n, torch.bfloat16))
    grads = []
    for it in range(2):
        torch.manual_seed(11)
        lin = ops.fused_linear(x, w, b)
        y = ops.dropout_add(lin, None, 0.25, True)
        w.grad, b.grad = None, None
        L.CALLS.clear()
        y.backward(gy)
        grads.append((w.grad.clone(), b.grad.clone()))
        if it == 0:
            assert (rows, n, torch.bfloat16) in D._WANT_CS and L.calls("pa_dropout_bwd") > 0
        else:
            _lib_loaded("pa_dropout_bwd_colsum", "pa_fold_partials")
    mask = (y.detach() != 0) | (lin.detach() == 0)
    dx_ref = gy.float() * mask.float() / 0.75
    torch.testing.assert_close(grads[1][1].float(), dx_ref.sum(0), atol=0.25, rtol=1e-2)
    assert torch.equal(grads[0][0], grads[1][0])  # same mask / dX as the unfused kernel
    torch.testing.assert_close(grads[0][1].float(), grads[1][1].float(), atol=0.25, rtol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("shape,k,s,p", [((2, 17, 15, 64), 3, 2, 1), ((3, 12, 12, 32), 2, 2, 0), ((1, 9, 11, 16), 3, 1, 1)])
def test_maxpool_nhwc_matches_torch(shape, k, s, p):
    from paddlepaddle_amd.ops import pool as P
    g = torch.Generator().manual_seed(7)
    x = torch.randn(*shape, generator=g).to("cuda", torch.bfloat16).requires_grad_(True)
    assert P.maxpool2d_nhwc_supported(x, k, s, p)
    y = P.maxpool2d_nhwc(x, k, s, p)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = torch.nn.functional.max_pool2d(xr, k, s, p)
    assert torch.equal(y.float(), yr.permute(0, 2, 3, 1))
    gy = torch.randn(yr.shape, generator=g).to("cuda")
    y.backward(gy.permute(0, 2, 3, 1).to(torch.bfloat16))
    yr.backward(gy.to(torch.bfloat16).float())
    torch.testing.assert_close(x.grad.float(), xr.grad.permute(0, 2, 3, 1), atol=2e-2, rtol=1e-2)
    _lib_loaded("pa_maxpool_nhwc_fwd", "pa_maxpool_nhwc_bwd")


def _maxpool_paddle_ref(x, k, s, p, gy):
    """numpy max pool with the reference's semantics (pooling.h MaxPool / pooling.cu KernelMaxPool2DGrad): the
    in-bounds window only, y = y > x ? y : x from the type's lowest value, gradient to the first x == y."""
    import numpy as np
    N, H, W, C = x.shape
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    y = np.full((N, Ho, Wo, C), -np.inf, dtype=np.float64)
    dx = np.zeros_like(x, dtype=np.float64)
    for n in range(N):
        for i in range(Ho):
            for j in range(Wo):
                hs, ws = i * s - p, j * s - p
                hh = range(max(hs, 0), min(hs + k, H))
                ww = range(max(ws, 0), min(ws + k, W))
                for c in range(C):
                    best = -np.inf
                    for a in hh:
                        for b in ww:
                            v = x[n, a, b, c]
                            best = best if best > v else v
                    y[n, i, j, c] = best
                    done = False
                    for a in hh:
                        for b in ww:
                            if not done and x[n, a, b, c] == best:
                                dx[n, a, b, c] += gy[n, i, j, c]
                                done = True
    return y, dx


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("k,s,p", [(3, 2, 1), (2, 3, 0), (3, 1, 1)])
def test_maxpool_nhwc_through_functional(dtype, k, s, p):
    """paddle.nn.functional.max_pool2d(data_format='NHWC') (the path ResNet takes) against the reference's
    semantics, with border windows whose in-bounds inputs are all -inf and a NaN input; tuple kernel sizes and
    ceil_mode take the fallback and must agree with the NCHW path."""
    import numpy as np
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.ops import _loader as L
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 9, 10, 8, generator=g).to(dtype)
    x[0, 0, :, :] = -float("inf")
    x[0, 0:2, 0:2, 3] = -float("inf")
    x[1, 4, 4, 5] = float("nan")
    xt = paddle.Tensor(x.to("cuda").requires_grad_(True))
    xt.stop_gradient = False
    before = L.calls("pa_maxpool_nhwc_fwd")
    y = paddle.nn.functional.max_pool2d(xt, k, s, p, data_format="NHWC")
    assert L.calls("pa_maxpool_nhwc_fwd") > before, "the NHWC HIP kernel must serve int kernel / stride"
    gy = torch.randn(tuple(y.shape), generator=g).to(dtype)
    y.backward(paddle.Tensor(gy.to("cuda")))
    want_y, want_dx = _maxpool_paddle_ref(x.float().numpy(), k, s, p, gy.float().numpy())
    np.testing.assert_array_equal(y._t.detach().float().cpu().numpy(), want_y.astype(np.float32))
    np.testing.assert_allclose(xt.grad._t.float().cpu().numpy(), want_dx, atol=2e-2, rtol=1e-2)
    # fallback forms agree with the NCHW path on finite data
    xf = paddle.Tensor(torch.randn(2, 9, 10, 8, generator=g).to("cuda", dtype))
    for kk, ss, cm in (((2, 3), (2, 2), False), (3, 2, True)):
        a = paddle.nn.functional.max_pool2d(xf, kk, ss, 0, ceil_mode=cm, data_format="NHWC")
        b = paddle.nn.functional.max_pool2d(xf.transpose([0, 3, 1, 2]), kk, ss, 0, ceil_mode=cm)
        assert torch.equal(a._t, b._t.permute(0, 2, 3, 1))


@pytest.mark.gpu
@pytest.mark.parametrize("act", [None, "gelu"])
def test_fused_linear_dx_hook_runs_between_dgrad_and_wgrad(act):
    """The column-parallel dX hook (tensor_parallel._async_allreduce_hook) sees dX right after its GEMM; the
    finisher runs after the dW GEMM was issued; dW is unaffected by what the hook does to dX."""
    from paddlepaddle_amd.ops import linear as Lin
    torch.manual_seed(0)
    x = torch.randn(256, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(128, 192, device="cuda") * 0.05).to(torch.bfloat16).requires_grad_(True)
    b = torch.randn(192, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    events = []

    def hook(dx):
        events.append("hook")
        dx.mul_(2.0)
        return lambda: events.append("finish")
    y = Lin.fused_linear(x, w, b, act=act, dx_hook=hook)
    g = torch.randn_like(y)
    y.backward(g)
    xr, wr, br = (t.detach().clone().requires_grad_(True) for t in (x, w, b))
    yr = Lin.fused_linear(xr, wr, br, act=act)
    yr.backward(g)
    assert events == ["hook", "finish"]
    torch.testing.assert_close(x.grad, 2 * xr.grad)
    torch.testing.assert_close(w.grad, wr.grad)


@pytest.mark.gpu
def test_layer_norm_residual_grad_fused():
    """(r, LN(x)) with r's gradient summed into dx by the LN backward kernel == LN + separate residual add."""
    from paddlepaddle_amd.ops import norm as N
    torch.manual_seed(0)
    x = torch.randn(64, 1024, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(1024, device="cuda")).to(torch.bfloat16).requires_grad_(True)
    b = (0.1 * torch.randn(1024, device="cuda")).to(torch.bfloat16).requires_grad_(True)
    gr, gy = torch.randn_like(x), torch.randn_like(x)
    before = L.calls("pa_layer_norm_bwd")
    r, y = N.layer_norm_residual(x, w, b, 1e-5)
    torch.autograd.backward([r, y], [gr, gy])
    assert L.calls("pa_layer_norm_bwd") == before + 1
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (1024,), wr, br, 1e-5)
    torch.autograd.backward([xr, yr], [gr.float(), gy.float()])
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=5e-2, rtol=2e-2)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=5e-1, rtol=2e-2)
    torch.testing.assert_close(b.grad.float(), br.grad, atol=5e-1, rtol=2e-2)


@pytest.mark.gpu
def test_native_launch_path_is_active():
    """Launches go through the generated METH_FASTCALL entry points (csrc/dispatch), not ctypes."""
    from paddlepaddle_amd.ops import _loader as L
    from paddlepaddle_amd.ops import norm as N
    assert L.native_launch(), "csrc/dispatch module _C_dispatch not loaded"
    x = torch.randn(4, 256, device="cuda", dtype=torch.bfloat16)
    w = torch.rand(256, device="cuda", dtype=torch.bfloat16)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):  # the current-stream sentinel resolves to the side stream
        y = N.rms_norm(x, w, 1e-6)
    s.synchronize()
    ref = (x.float() * torch.rsqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-6)) * w.float()
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
