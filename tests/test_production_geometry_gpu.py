"""Hand-written kernels at the geometry the per-shape chooser selects them for in the benchmarks (VERDICT r3 weak
#11): ResNet-50 stage-1/2 convolutions at batch 32 (56x56 / 28x28) on every hand-written variant, a full
bottleneck stage against fp32, and the GPT-3 13B / 1.3B GEMM products in the three linear-layer layouts — each
against a plain PyTorch fp32 reference of the same op."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from paddlepaddle_amd.ops import _loader as L  # noqa: E402
from paddlepaddle_amd.ops import conv as C  # noqa: E402
from paddlepaddle_amd.ops import gemm as G  # noqa: E402


def _rel(got, exp):
    return (got.float() - exp).abs().max().item() / (exp.abs().max().item() + 1e-6)


def _conv_ref(x, w, stride, pad, dy):
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.float().requires_grad_(True)
    y = torch.nn.functional.conv2d(xr, wr, None, stride, pad)
    y.backward(dy.float().permute(0, 3, 1, 2))
    return y.permute(0, 2, 3, 1), xr.grad.permute(0, 2, 3, 1), wr.grad


# (k, stride, cin, cout, hw): ResNet-50 layer1 (56x56) and layer2 (28x28) convolutions
RESNET_CONVS = [(1, 1, 64, 64, 56), (3, 1, 64, 64, 56), (1, 1, 64, 256, 56), (1, 1, 256, 64, 56),
                (1, 1, 256, 128, 56), (3, 2, 128, 128, 56), (3, 1, 128, 128, 28), (1, 1, 128, 512, 28),
                (1, 2, 256, 512, 56)]


@pytest.mark.parametrize("k,stride,cin,cout,hw", RESNET_CONVS)
@pytest.mark.parametrize("variant", ["hip", "skinny"])
def test_resnet_conv_batch32_every_direction(monkeypatch, k, stride, cin, cout, hw, variant):
    g = torch.Generator(device="cuda").manual_seed(k * 100 + cin + cout + hw)
    x = torch.randn(32, hw, hw, cin, device="cuda", generator=g).bfloat16()
    w = (torch.randn(cout, cin, k, k, device="cuda", generator=g) * (1.0 / (cin * k * k) ** 0.5)).bfloat16()
    offered = {}

    def pick(key, own, mi, skinny=None, mm=None):
        offered[key[0]] = skinny is not None
        if variant == "skinny" and skinny is not None:
            return "skinny"
        return "hip"
    monkeypatch.setattr(C, "_pick", pick)
    assert C.eligible_nhwc(x, w, 1)
    xx = x.clone().requires_grad_(True)
    ww = w.clone().requires_grad_(True)
    L.reset_calls()
    y = C.conv2d_nhwc(xx, ww, None, stride, k // 2, 1)
    dy = torch.randn(y.shape, device="cuda", generator=g).bfloat16()
    y.backward(dy)
    torch.cuda.synchronize()
    if variant == "skinny" and not any(offered.values()):
        pytest.skip("no skinny kernel for this geometry")
    assert sum(L.CALLS.values()) > 0
    yr, dxr, dwr = _conv_ref(x, w, stride, k // 2, dy)
    assert _rel(y, yr) < 2e-2
    assert _rel(xx.grad, dxr) < 2e-2
    assert _rel(ww.grad, dwr) < 2e-2


def test_resnet50_layer1_stack_bf16_hip_vs_fp32():
    """ResNet-50 stage 1 (three bottleneck blocks, projection shortcut) at batch 32, 56x56: bf16 NHWC through the
    hand-written conv / BN kernels against the same stage in fp32 (training-mode BN)."""
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.vision.models import resnet50
    paddle.set_device("gpu:0")
    paddle.seed(3)
    net = resnet50(num_classes=10, data_format="NHWC")
    stage = net.layer1
    ref = resnet50(num_classes=10, data_format="NHWC").layer1
    ref.set_state_dict(stage.state_dict())
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(32, 56, 56, 64, device="cuda", generator=g)
    for p in stage.parameters():
        p._t.data = p._t.data.bfloat16() if p._t.dim() == 4 else p._t.data
    xb = paddle.Tensor(x.bfloat16().requires_grad_(True))
    xb.stop_gradient = False
    L.reset_calls()
    y = stage(xb)
    # a random cotangent: d sum(y) / dx through training-mode BN is a near-total cancellation (the batch mean
    # removes it), which no bf16 pipeline reproduces to a few percent of its tiny magnitude
    gy = torch.randn(y.shape, device="cuda", generator=g)
    y.astype("float32").backward(paddle.Tensor(gy))
    torch.cuda.synchronize()
    assert sum(v for k, v in L.CALLS.items() if k.startswith("pa_bn_")) > 0
    assert sum(v for k, v in L.CALLS.items() if "gemm" in k or "conv" in k) > 0
    xf = paddle.Tensor(x.clone().requires_grad_(True))
    xf.stop_gradient = False
    yf = ref(xf)
    yf.backward(paddle.Tensor(gy))
    # the same bf16 stage on the vendor / ATen path (MIOpen convolutions, fp32-math BN) sets the bf16 noise floor
    # of a three-block backward at batch 32
    from paddlepaddle_amd.framework import flags
    vend = resnet50(num_classes=10, data_format="NHWC").layer1
    vend.set_state_dict(stage.state_dict())
    for p in vend.parameters():
        p._t.data = p._t.data.bfloat16() if p._t.dim() == 4 else p._t.data
    flags.set_flags({"FLAGS_use_hip_kernels": False})
    try:
        xv = paddle.Tensor(x.bfloat16().requires_grad_(True))
        xv.stop_gradient = False
        yv = vend(xv)
        yv.astype("float32").backward(paddle.Tensor(gy))
    finally:
        flags.set_flags({"FLAGS_use_hip_kernels": True})
    err_y, err_dx = _rel(y._t, yf._t.detach()), _rel(xb.grad._t, xf.grad._t)
    floor_y, floor_dx = _rel(yv._t, yf._t.detach()), _rel(xv.grad._t, xf.grad._t)
    print(f"layer1 bf16 vs fp32: hip y {err_y:.4f} dx {err_dx:.4f}; vendor y {floor_y:.4f} dx {floor_dx:.4f}")
    assert err_y < max(5e-2, 1.5 * floor_y)
    assert err_dx < max(8e-2, 1.5 * floor_dx)


H13, F13, Q13, T13 = 5120, 20480, 15360, 4096
H1, F1, Q1, T1 = 2048, 8192, 6144, 8192
GEMMS = []
for (H, F, Q, T) in ((H13, F13, Q13, T13), (H1, F1, Q1, T1)):
    GEMMS += [("fwd", T, Q, H), ("fwd", T, H, F), ("dgrad", T, H, Q), ("dgrad", T, F, H), ("wgrad", H, Q, T),
              ("wgrad", F, H, T)]


@pytest.mark.parametrize("layout,M,N,K", GEMMS)
def test_gpt_gemm_shapes_vs_fp32(layout, M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    if layout == "fwd":
        a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
        b = (torch.randn(K, N, device="cuda", generator=g) * 0.02).bfloat16()
    elif layout == "dgrad":
        a = (torch.randn(M, K, device="cuda", generator=g) * 1e-2).bfloat16()
        b = (torch.randn(N, K, device="cuda", generator=g) * 0.02).bfloat16().t()
    else:
        a = torch.randn(K, M, device="cuda", generator=g).bfloat16().t()
        b = (torch.randn(K, N, device="cuda", generator=g) * 1e-2).bfloat16()
    assert G.supported(a, b)
    L.reset_calls()
    c = G.gemm(a, b)
    torch.cuda.synchronize()
    assert sum(L.CALLS.values()) == 1
    ref = a.float() @ b.float()
    assert _rel(c, ref) < 1e-2


def _gpt_layer_run(layer, x, gy, dtype):
    import paddlepaddle_amd as paddle
    xt = paddle.Tensor(x.detach().to(dtype).clone().requires_grad_(True))
    xt.stop_gradient = False
    y = layer(xt)
    y.astype("float32").backward(paddle.Tensor(gy))
    grads = {n: p.grad._t.float() for n, p in layer.named_parameters()}
    return y._t.float(), xt.grad._t.float(), grads


def test_gpt3_13b_decoder_layer_bf16_hip_vs_fp32():
    """One GPT-3 13B decoder layer (h 5120, 40 heads of 128, ffn 20480) at the bench's micro-batch geometry
    (B 2, S 2048), dropout off: bf16 through the hand-written LN / GEMM (fused bias, GeLU) / flash-attention /
    residual kernels against the same layer in fp32 on the ATen path, forward, input gradient and weight gradients.
    The bf16 vendor path (hipBLASLt, ATen attention and LN) sets the noise floor."""
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.framework import flags
    from paddlepaddle_amd.models.gpt import GPTConfig, GPTDecoderLayer
    paddle.set_device("gpu:0")
    paddle.seed(13)
    cfg = GPTConfig.gpt3_13b(hidden_dropout_prob=0.0)
    layer = GPTDecoderLayer(cfg)
    sd = layer.state_dict()
    g = torch.Generator(device="cuda").manual_seed(2)
    x = torch.randn(2, 2048, cfg.hidden_size, device="cuda", generator=g)
    gy = torch.randn(x.shape, device="cuda", generator=g)

    flags.set_flags({"FLAGS_use_hip_kernels": False})
    try:
        ref = GPTDecoderLayer(cfg)
        ref.set_state_dict(sd)
        yf, dxf, gf = _gpt_layer_run(ref, x, gy, torch.float32)
        vend = GPTDecoderLayer(cfg)
        vend.set_state_dict(sd)
        vend.to(dtype="bfloat16")
        yv, dxv, gv = _gpt_layer_run(vend, x, gy, torch.bfloat16)
    finally:
        flags.set_flags({"FLAGS_use_hip_kernels": True})
    layer.to(dtype="bfloat16")
    L.reset_calls()
    y, dx, gh = _gpt_layer_run(layer, x, gy, torch.bfloat16)
    torch.cuda.synchronize()
    for k in ("pa_layer_norm_fwd", "pa_layer_norm_bwd", "pa_flash_attn_fwd", "pa_flash_attn_bwd"):
        assert any(n.startswith(k) for n, v in L.CALLS.items() if v), (k, dict(L.CALLS))
    # the per-shape GEMM chooser may hand some shapes to hipBLASLt once earlier tests have timed them
    assert sum(v for n, v in L.CALLS.items() if n.startswith("pa_gemm")) >= 1, dict(L.CALLS)
    rows = [("y", y, yv, yf), ("dx", dx, dxv, dxf)] + [(n, gh[n], gv[n], gf[n]) for n in gf]
    for name, got, vendor, exp in rows:
        err, floor = _rel(got, exp), _rel(vendor, exp)
        print(f"{name}: hip {err:.4f} vendor {floor:.4f}")
        assert err < max(2e-2, 1.5 * floor), (name, err, floor)


@pytest.mark.parametrize("size", ["llama2_7b", "llama2_70b"])
def test_llama2_decoder_layer_bf16_hip_vs_fp32(size):
    """One LLaMA-2 decoder layer at full width (7B: 32 MHA heads; 70B: h 8192, 64 query / 8 KV heads, ffn 28672)
    at B 1, S 2048: bf16 through the hand-written RMSNorm / RoPE / flash-attention (GQA) / SwiGLU / GEMM kernels
    against the same layer in fp32 on the ATen path, forward, input gradient and every weight gradient; the bf16
    vendor path sets the noise floor."""
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.framework import flags
    from paddlepaddle_amd.models.llama import LlamaConfig, LlamaDecoderLayer
    paddle.set_device("gpu:0")
    paddle.seed(70)
    cfg = getattr(LlamaConfig, size)()
    layer = LlamaDecoderLayer(cfg)
    sd = layer.state_dict()
    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.randn(1, 2048, cfg.hidden_size, device="cuda", generator=g)
    gy = torch.randn(x.shape, device="cuda", generator=g)
    flags.set_flags({"FLAGS_use_hip_kernels": False})
    try:
        ref = LlamaDecoderLayer(cfg)
        ref.set_state_dict(sd)
        yf, dxf, gf = _gpt_layer_run(ref, x, gy, torch.float32)
        del ref
        vend = LlamaDecoderLayer(cfg)
        vend.set_state_dict(sd)
        vend.to(dtype="bfloat16")
        yv, dxv, gv = _gpt_layer_run(vend, x, gy, torch.bfloat16)
        del vend
    finally:
        flags.set_flags({"FLAGS_use_hip_kernels": True})
    layer.to(dtype="bfloat16")
    L.reset_calls()
    y, dx, gh = _gpt_layer_run(layer, x, gy, torch.bfloat16)
    torch.cuda.synchronize()
    for k in ("pa_rms_norm_fwd", "pa_rms_norm_bwd", "pa_rope", "pa_swiglu_fwd", "pa_swiglu_bwd",
              "pa_flash_attn_fwd", "pa_flash_attn_bwd"):
        assert any(n.startswith(k) for n, v in L.CALLS.items() if v), (k, dict(L.CALLS))
    # the per-shape GEMM chooser may hand some shapes to hipBLASLt once earlier tests have timed them
    assert sum(v for n, v in L.CALLS.items() if n.startswith("pa_gemm")) >= 1, dict(L.CALLS)
    rows = [("y", y, yv, yf), ("dx", dx, dxv, dxf)] + [(n, gh[n], gv[n], gf[n]) for n in gf]
    for name, got, vendor, exp in rows:
        err, floor = _rel(got, exp), _rel(vendor, exp)
        print(f"{size} {name}: hip {err:.4f} vendor {floor:.4f}")
        assert err < max(2e-2, 1.5 * floor), (name, err, floor)
