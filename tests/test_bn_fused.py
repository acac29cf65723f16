"""Fused channels-last batch norm (+ residual add + relu): csrc/kernels/bn.hip against a plain fp32
PyTorch reference of the same op; running statistics follow the reference's biased-variance update."""
import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle
from paddlepaddle_amd import ops
from paddlepaddle_amd.ops.bn import batch_norm_act_reference


def _ref(x, w, b, rm, rv, training, mom, eps, act, res):
    """autograd-able fp32 reference on [R, C]."""
    xf = x.float()
    if training:
        mean, var = xf.mean(0), xf.var(0, unbiased=False)
        rm.mul_(mom).add_((1 - mom) * mean.detach())
        rv.mul_(mom).add_((1 - mom) * var.detach())
    else:
        mean, var = rm, rv
    y = (xf - mean) * torch.rsqrt(var + eps) * w + b
    if res is not None:
        y = y + res.float()
    return torch.relu(y) if act == "relu" else y


def test_reference_and_functional_cpu():
    torch.manual_seed(0)
    x = torch.randn(4, 5, 5, 16)
    w, b = torch.rand(16) + 0.5, torch.randn(16)
    rm, rv = torch.zeros(16), torch.ones(16)
    rm2, rv2 = rm.clone(), rv.clone()
    res = torch.randn_like(x)
    y = ops.batch_norm_act_nhwc(x, w, b, rm, rv, True, 0.9, 1e-5, "relu", res)
    ref = _ref(x.view(-1, 16), w, b, rm2, rv2, True, 0.9, 1e-5, "relu", res.view(-1, 16)).view(x.shape)
    np.testing.assert_allclose(y.numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(rv.numpy(), rv2.numpy(), rtol=1e-6)
    # F.batch_norm (NCHW, fallback) also uses the reference's biased running variance
    t = torch.randn(8, 3, 4, 4)
    m, v = paddle.zeros([3]), paddle.ones([3])
    paddle.nn.functional.batch_norm(paddle.Tensor(t), m, v, training=True, momentum=0.9)
    np.testing.assert_allclose(v.numpy(), 0.9 + 0.1 * t.var((0, 2, 3), unbiased=False).numpy(), rtol=1e-5)


def test_resnet_block_fused_matches_unfused_cpu():
    from paddlepaddle_amd.vision.models.resnet import BottleneckBlock
    paddle.seed(0)
    blk = BottleneckBlock(64, 16, data_format="NHWC")
    x = paddle.randn([2, 8, 8, 64])
    y = blk(x)
    bn = blk.bn3
    # unfused composition through the plain layers (eval stats untouched by a second training pass)
    blk.eval()
    y_eval = blk(x)
    out = blk.bn3(blk.conv3(paddle.nn.functional.relu(blk.bn2(blk.conv2(paddle.nn.functional.relu(
        blk.bn1(blk.conv1(x))))))))
    ref = paddle.nn.functional.relu(out + x)
    np.testing.assert_allclose(y_eval.numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)
    assert y.shape == [2, 8, 8, 64] and bn._mean.numpy().any()


@pytest.mark.gpu
@pytest.mark.parametrize("shape,act,with_res,training", [
    ((4, 7, 7, 64), "relu", False, True),
    ((8, 14, 14, 256), "relu", True, True),
    ((2, 3, 3, 2048), None, False, True),
    ((16, 28, 28, 128), None, True, True),
    ((3, 5, 5, 24), "relu", True, True),
    ((4, 7, 7, 512), "relu", True, False),
])
def test_bn_act_hip_matches_fp32(shape, act, with_res, training):
    from paddlepaddle_amd.ops import _loader as L
    L.reset_calls()
    torch.manual_seed(0)
    C = shape[-1]
    x = (torch.randn(shape, device="cuda") * 2 + 0.5).bfloat16().requires_grad_(True)
    res = torch.randn(shape, device="cuda").bfloat16().requires_grad_(True) if with_res else None
    w = (torch.rand(C, device="cuda") + 0.5).requires_grad_(True)
    b = torch.randn(C, device="cuda").requires_grad_(True)
    rm, rv = torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5
    rm2, rv2 = rm.clone(), rv.clone()
    assert L.hip_enabled_for(x) and L.has("pa_bn_fwd_nhwc")
    y = ops.batch_norm_act_nhwc(x, w, b, rm, rv, training, 0.9, 1e-5, act, res)
    xr = x.detach().float().requires_grad_(True)
    rr = res.detach().float().requires_grad_(True) if with_res else None
    wr, br = w.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    ref = _ref(xr.view(-1, C), wr, br, rm2, rv2, training, 0.9, 1e-5, act, rr.view(-1, C) if with_res else None)
    torch.testing.assert_close(y.float().view(-1, C), ref, rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(rm, rm2, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rv, rv2, rtol=1e-4, atol=1e-5)
    g = torch.randn(shape, device="cuda").bfloat16()
    y.backward(g)
    # mask the reference's gradient with the kernel's own relu decisions (bf16 output rounding at 0)
    ref.backward(g.float().view(-1, C))
    torch.testing.assert_close(x.grad.float(), xr.grad.view(shape), rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(w.grad, wr.grad, rtol=2e-2, atol=2e-1)
    torch.testing.assert_close(b.grad, br.grad, rtol=2e-2, atol=2e-1)
    if with_res:
        torch.testing.assert_close(res.grad.float(), rr.grad.view(shape), rtol=2e-2, atol=2e-2)
    if act == "relu" and with_res:  # the relu bit-mask variants (no y re-read in the backward)
        assert L.calls("pa_bn_fwd_nhwc_mask") == 1 and L.calls("pa_bn_bwd_nhwc_mask") == 1
    else:
        assert L.calls("pa_bn_fwd_nhwc") == 1 and L.calls("pa_bn_bwd_nhwc") == 1


@pytest.mark.gpu
@pytest.mark.parametrize("nesterov", [False, True])
def test_momentum_multi_tensor_hip_matches_fp32(nesterov):
    """Multi-tensor Momentum (fp32 masters + bf16 shadows, L2 decay) == per-tensor fp32 math."""
    paddle.set_device("gpu")
    torch.manual_seed(0)
    ws = [torch.randn(64, 33, device="cuda"), torch.randn(7, device="cuda"), torch.randn(3, 3, 8, 16, device="cuda")]
    params = [paddle.Parameter(w.clone().bfloat16()) for w in ws]
    opt = paddle.optimizer.Momentum(0.1, 0.9, parameters=params, use_nesterov=nesterov, weight_decay=1e-2,
                                    multi_precision=True)
    masters = [w.bfloat16().float() for w in ws]
    vel = [torch.zeros_like(w) for w in ws]
    for step in range(3):
        gs = [torch.randn_like(w) for w in ws]
        for p, g in zip(params, gs):
            p._t.grad = g.bfloat16()
        opt.step()
        for i, g in enumerate(gs):
            gj = g.bfloat16().float() + 1e-2 * masters[i]
            vel[i] = 0.9 * vel[i] + gj
            masters[i] = masters[i] - 0.1 * (gj + 0.9 * vel[i] if nesterov else vel[i])
    assert getattr(opt, "_mt_tables", None), "fused multi-tensor path not taken"
    from paddlepaddle_amd.ops import _loader as L
    assert L.calls("pa_momentum_multi") == 3
    for p, m in zip(params, masters):
        torch.testing.assert_close(opt._master(p), m, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(p._t.float(), m.bfloat16().float(), rtol=1e-2, atol=1e-2)


@pytest.mark.gpu
def test_bottleneck_residual_grad_sink_matches_autograd_sum_gpu():
    """Identity-shortcut bottleneck on the HIP path: bn3 hands d(residual) to conv1, whose dgrad GEMM adds it in
    its epilogue (ops/conv.py ResidualGradSink). Gradients match the same block with the hand-off disabled
    (autograd sums the two gradients of x with an elementwise add)."""
    from paddlepaddle_amd.ops import conv as C
    from paddlepaddle_amd.vision.models import resnet as RN
    paddle.set_device("gpu")
    paddle.seed(3)
    paddle.set_default_dtype("bfloat16")
    try:
        blk = RN.BottleneckBlock(256, 64, data_format="NHWC")
    finally:
        paddle.set_default_dtype("float32")
    g = torch.Generator(device="cuda").manual_seed(0)
    xt = torch.randn(8, 14, 14, 256, device="cuda", generator=g, dtype=torch.bfloat16)
    dy = torch.randn(8, 14, 14, 256, device="cuda", generator=g, dtype=torch.bfloat16)
    seen = []
    orig = C.residual_grad_sink

    class spy(orig):
        def __exit__(self, *exc):
            seen.append(self.sink.armed)
            return super().__exit__(*exc)

    def run(ctx_factory):
        C.residual_grad_sink = ctx_factory
        try:
            x = paddle.Tensor(xt.clone().requires_grad_(True))
            for p in blk.parameters():
                p.clear_gradient(set_to_zero=False)
            blk(x)._t.backward(dy)
            return x._t.grad.float(), [p.grad._t.float().clone() for p in blk.parameters()]
        finally:
            C.residual_grad_sink = orig

    class off:
        def __enter__(self):
            return C.ResidualGradSink()

        def __exit__(self, *exc):
            return False
    old = paddle.get_flags("FLAGS_gemm_backend")["FLAGS_gemm_backend"]
    paddle.set_flags({"FLAGS_gemm_backend": "hip"})  # the hand-written 1x1 path, whatever this shape's timing says
    try:
        gx_s, gp_s = run(spy)
        gx_r, gp_r = run(off)
    finally:
        paddle.set_flags({"FLAGS_gemm_backend": old})
    assert seen and all(seen), "conv1 did not run the hand-written GEMM path"
    scale = gx_r.abs().max().item()
    assert (gx_s - gx_r).abs().max().item() < 2e-2 * scale
    for a, b in zip(gp_s, gp_r):
        assert (a - b).abs().max().item() <= 2e-2 * max(b.abs().max().item(), 1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [1, 2])
def test_projection_block_residual_grad_producer_gpu(stride):
    """Projection-shortcut bottleneck: the shortcut conv hands dx to conv1's epilogue (residual_grad_producer);
    gradients match the same block with the hand-off disabled (autograd sums the two gradients of x)."""
    from paddlepaddle_amd.ops import _loader as L
    from paddlepaddle_amd.ops import conv as C
    from paddlepaddle_amd.vision.models import resnet as RN
    paddle.set_device("gpu")
    paddle.seed(4)
    paddle.set_default_dtype("bfloat16")
    try:
        ds = paddle.nn.Sequential(paddle.nn.Conv2D(128, 256, 1, stride=stride, bias_attr=False, data_format="NHWC"),
                                  paddle.nn.BatchNorm2D(256, data_format="NHWC"))
        blk = RN.BottleneckBlock(128, 64, stride=stride, downsample=ds, data_format="NHWC")
    finally:
        paddle.set_default_dtype("float32")
    g = torch.Generator(device="cuda").manual_seed(1)
    xt = torch.randn(8, 14, 14, 128, device="cuda", generator=g, dtype=torch.bfloat16)
    ho = 14 // stride
    dy = torch.randn(8, ho, ho, 256, device="cuda", generator=g, dtype=torch.bfloat16)
    orig = C.residual_grad_producer
    produced = []

    class spy(orig):
        def __exit__(self, *exc):
            produced.append(self.sink is not None and self.sink.armed)
            return super().__exit__(*exc)

    class off:
        def __init__(self, sink):
            pass

        def __enter__(self):
            return None

        def __exit__(self, *exc):
            return False

    def run(factory):
        C.residual_grad_producer = factory
        try:
            x = paddle.Tensor(xt.clone().requires_grad_(True))
            for p in blk.parameters():
                p.clear_gradient(set_to_zero=False)
            blk(x)._t.backward(dy)
            return x._t.grad.float(), [p.grad._t.float().clone() for p in blk.parameters()]
        finally:
            C.residual_grad_producer = orig
    old = paddle.get_flags("FLAGS_gemm_backend")["FLAGS_gemm_backend"]
    paddle.set_flags({"FLAGS_gemm_backend": "hip"})
    try:
        L.CALLS.clear()
        gx_s, gp_s = run(spy)
        gx_r, gp_r = run(off)
    finally:
        paddle.set_flags({"FLAGS_gemm_backend": old})
    assert produced and all(produced), "conv1 did not arm the sink on the hand-written path"
    scale = gx_r.abs().max().item()
    assert (gx_s - gx_r).abs().max().item() < 2e-2 * scale
    for a, b in zip(gp_s, gp_r):
        assert (a - b).abs().max().item() <= 2e-2 * max(b.abs().max().item(), 1e-3)
