"""Weight-only int8 / int4 and LLM.int8 linears (nn/quant, ops/quant.py, csrc/kernels/wo_gemm.hip) and the
quantised outputs of the fused norms. Reference: python/paddle/nn/quant/quantized_linear.py:56,183,276,
phi/kernels/impl/weight_quantize_kernel_impl.h (layout / rounding), fusion/gpu/fused_layernorm_kernel.cu:996."""
import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle
from paddlepaddle_amd.nn import quant as Q


def _w(k, n, seed=0, dtype="float32"):
    g = torch.Generator().manual_seed(seed)
    return paddle.Tensor((torch.randn(k, n, generator=g) * 0.05).to(getattr(torch, dtype)))


@pytest.mark.parametrize("algo,group", [("weight_only_int8", -1), ("weight_only_int8", 64), ("weight_only_int4", -1),
                                        ("weight_only_int4", 128), ("llm.int8", -1)])
def test_quantize_layout_and_roundtrip(algo, group):
    w = _w(256, 64)
    q, s = Q.weight_quantize(w, algo, group_size=group)
    assert q.dtype == paddle.int8
    if algo == "weight_only_int4":
        assert q.shape == [32, 256]
        u = q._t.view(torch.uint8)
        assert int(u.min()) >= 0 and ((u & 0xF) >= 1).all() and (((u >> 4) & 0xF) >= 1).all()  # values + 8
    else:
        assert q.shape == [64, 256] and int(q._t.abs().max()) <= 127
    assert s.shape == ([64] if group == -1 else [256 // group, 64])
    d = Q.weight_dequantize(q, s, algo, "float32", group)
    bound = 7 if algo == "weight_only_int4" else 127
    step = float(w._t.abs().max()) / bound
    assert d.shape == [256, 64] and float((d._t - w._t).abs().max()) <= 0.5 * step + 1e-6


def test_int4_nibble_order_matches_the_reference_packing():
    """channel 2j in the low nibble, 2j+1 in the high nibble of byte row j (weight_quantize_kernel_impl.h)."""
    w = torch.zeros(64, 16)
    w[:, 0], w[:, 1] = 1.0, -1.0
    q, s = Q.weight_quantize(paddle.Tensor(w), "weight_only_int4")
    b = int(q._t.view(torch.uint8)[0, 0])
    assert (b & 0xF) - 8 == 7 and ((b >> 4) & 0xF) - 8 == -7


def test_arguments_are_validated_not_dropped():
    w = _w(128, 32)
    with pytest.raises(ValueError):
        Q.weight_quantize(w, "weight_only_int8", group_size=32)
    with pytest.raises(ValueError):
        Q.weight_quantize(w, "fp8")
    with pytest.raises(ValueError):
        Q.weight_quantize(_w(100, 32), "weight_only_int8")
    q, s = Q.weight_quantize(w, "weight_only_int8")
    with pytest.raises(ValueError):
        Q.weight_only_linear(paddle.randn([2, 128]), q, weight_scale=s, weight_dtype="int2")
    with pytest.raises(ValueError):
        Q.weight_only_linear(paddle.randn([2, 128]), q)


@pytest.mark.parametrize("wdt,group", [("int8", -1), ("int8", 128), ("int4", 64)])
def test_weight_only_linear_equals_dequantized_product(wdt, group):
    w = _w(256, 64, 1)
    x = paddle.randn([5, 256])
    algo = "weight_only_" + wdt
    q, s = Q.weight_quantize(w, algo, group_size=group)
    bias = paddle.randn([64])
    y = Q.weight_only_linear(x, q, bias, s, wdt, group_size=group)
    ref = x._t @ Q.weight_dequantize(q, s, algo, "float32", group)._t + bias._t
    np.testing.assert_allclose(y.numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)


def test_llm_int8_outlier_decomposition():
    w = _w(128, 32, 2)
    q, s = Q.weight_quantize(w, "llm.int8")
    x = torch.randn(3, 128)
    x[:, 5] *= 40.0  # an outlier feature
    y = Q.llm_int8_linear(paddle.Tensor(x), q, None, s, threshold=6.0)
    wd = Q.weight_dequantize(q, s, "llm.int8", "float32")._t
    # outlier column exact (floating point), inliers through the row-quantised int8 path
    np.testing.assert_allclose(y.numpy(), (x @ wd).numpy(), rtol=0, atol=0.05 * float((x @ wd).abs().max()))
    xo = torch.zeros_like(x)
    xo[:, 5] = x[:, 5]
    inl = x - xo
    sx = inl.abs().amax(-1) / 127
    xq = torch.round(inl / sx[:, None])
    exact = (sx[:, None] * (xq @ q._t.float().t()) + xo @ q._t.float().t()) * s._t.float()
    np.testing.assert_allclose(y.numpy(), exact.numpy(), rtol=1e-5, atol=1e-5)


def test_fused_norm_quantized_outputs():
    from paddlepaddle_amd.incubate.nn import functional as IF
    x = paddle.randn([4, 64])
    w = paddle.ones([64])
    y = IF.fused_rms_norm(x, w, None, 1e-6, 1)
    q = IF.fused_rms_norm(x, w, None, 1e-6, 1, quant_scale=0.5, quant_round_type=1, quant_max_bound=127,
                          quant_min_bound=-127)
    assert q.dtype == paddle.int8
    v = (y._t.float() * 127 * 0.5)
    np.testing.assert_array_equal(q.numpy(), (torch.sign(v) * torch.floor(v.abs() + 0.5)).clamp(-127, 127).numpy())
    lq, res = IF.fused_layer_norm(x, w, paddle.zeros([64]), 1e-5, residual=x, quant_scale=1.0, quant_round_type=0,
                                  quant_max_bound=127, quant_min_bound=-127)
    assert lq.dtype == paddle.int8 and res.dtype == paddle.float32
    with pytest.raises(ValueError):
        IF.fused_rms_norm(x, w, None, 1e-6, 1, quant_scale=0.5)  # bounds missing: not silently ignored


def test_masked_mha_unsupported_arguments_raise():
    from paddlepaddle_amd.incubate.nn import functional as IF
    x = paddle.randn([2, 3 * 2 * 16])
    cache = paddle.zeros([2, 2, 2, 8, 16])
    with pytest.raises(NotImplementedError):
        IF.masked_multihead_attention(x, cache, cum_offsets=paddle.zeros([2], dtype="int32"))
    out, _ = IF.masked_multihead_attention(x, cache, sequence_lengths=paddle.to_tensor([0, 0]), out_scale=0.1,
                                           quant_round_type=1, quant_max_bound=127.0, quant_min_bound=-127.0)
    assert out.dtype == paddle.int8


def test_masked_mha_beam_cache_offset_reads_parent_beams():
    """beam_cache_offset[b, t] = w (non-zero) reads key / value t from beam w of b's batch entry; the current step
    is the row's own (reference masked_multihead_attention_kernel.cu beam_offsets)."""
    from paddlepaddle_amd.incubate.nn import functional as IF
    torch.manual_seed(0)
    bsz, W, H, D, Lmax, step = 2, 3, 2, 16, 8, 5
    B = bsz * W
    x = torch.randn(B, 3 * H * D)
    cache = torch.randn(2, B, H, Lmax, D)
    off = torch.randint(0, W, (bsz, W, Lmax), dtype=torch.int32)
    ref_cache = cache.clone()
    out, cache_out, off_out = IF.masked_multihead_attention(
        paddle.to_tensor(x), paddle.to_tensor(cache), sequence_lengths=paddle.to_tensor([step] * B),
        beam_cache_offset=paddle.to_tensor(off))
    q, k, v = x.view(B, 3, H, D).unbind(1)
    ref_cache[0][:, :, step] = k
    ref_cache[1][:, :, step] = v
    for b in range(B):
        ks, vs = [], []
        for t in range(step + 1):
            o = int(off[b // W, b % W, t])
            r = (b // W) * W + o if (o != 0 and t < step) else b
            ks.append(ref_cache[0][r, :, t])
            vs.append(ref_cache[1][r, :, t])
        K, V = torch.stack(ks, 1), torch.stack(vs, 1)        # [H, T, D]
        p = torch.softmax(torch.einsum("hd,htd->ht", q[b], K) / D ** 0.5, -1)
        ref = torch.einsum("ht,htd->hd", p, V).reshape(-1)
        np.testing.assert_allclose(out.numpy()[b], ref.numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(cache_out.numpy(), ref_cache.numpy())
    assert off_out is not None


# ------------------------------------------------------------------------------------------------ GPU kernels
def _ref_gpu(x, q, s, algo, group, bias):
    wd = Q.weight_dequantize(q, s, algo, "float32", group)._t.cuda()
    y = x.float() @ wd
    return y + bias.float() if bias is not None else y


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 7, 16, 33, 64, 200])
@pytest.mark.parametrize("algo,group", [("weight_only_int8", -1), ("weight_only_int8", 64), ("weight_only_int4", -1),
                                        ("weight_only_int4", 128)])
def test_wo_gemm_kernel_matches_fp32_dequantized_reference(M, algo, group):
    from paddlepaddle_amd.ops import _loader as L
    paddle.set_device("gpu:0")
    K, N = 1024, 1536
    w = _w(K, N, 3)
    q, s = Q.weight_quantize(w, algo, group_size=group)
    q, s = paddle.Tensor(q._t.cuda()), paddle.Tensor(s._t.cuda())
    g = torch.Generator(device="cuda").manual_seed(M)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    bias = (torch.randn(N, device="cuda", generator=g) * 0.1).bfloat16()
    L.reset_calls()
    paddle.set_flags({"FLAGS_weight_only_dequant_cache_mb": 0})  # the decode kernel itself / per-call dequant
    try:
        y = Q.weight_only_linear(paddle.Tensor(x), q, paddle.Tensor(bias), s, algo.split("_")[-1], group_size=group)
    finally:
        paddle.set_flags({"FLAGS_weight_only_dequant_cache_mb": 4096})
    torch.cuda.synchronize()
    assert L.calls("pa_wo_gemm" if M <= 64 else "pa_wo_dequant") == 1
    ref = _ref_gpu(x, q, s, algo, group, bias)
    err = (y._t.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 16, 40])
def test_llm_int8_kernel_matches_decomposition(M):
    from paddlepaddle_amd.ops import _loader as L
    paddle.set_device("gpu:0")
    K, N = 2048, 1024
    q, s = Q.weight_quantize(_w(K, N, 4), "llm.int8")
    q, s = paddle.Tensor(q._t.cuda()), paddle.Tensor(s._t.cuda())
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(M, K, device="cuda", generator=g)
    x[:, 17] *= 30
    x[:, 900] *= 25
    xb = x.bfloat16()
    L.reset_calls()
    paddle.set_flags({"FLAGS_weight_only_dequant_cache_mb": 0})  # the LLM.int8 decode kernel itself
    try:
        y = Q.llm_int8_linear(paddle.Tensor(xb), q, None, s, threshold=6.0)
    finally:
        paddle.set_flags({"FLAGS_weight_only_dequant_cache_mb": 4096})
    torch.cuda.synchronize()
    assert L.calls("pa_wo_gemm") == 1
    xq, xo, sx, outl = Q._llm_split(xb, 6.0)
    assert int(outl.sum()) == 2
    exact = (sx[:, None] * (xq @ q._t.float().t()) + xo @ q._t.float().t()) * s._t.float()
    err = (y._t.float() - exact).abs().max().item() / exact.abs().max().item()
    assert err < 1e-2, err


@pytest.mark.gpu
def test_llm_int8_long_inputs_run_the_mfma_gemm():
    """LLM.int8 above 64 rows runs on device kernels (the MFMA GEMM on the exact int8 values, outlier
    columns as x / sx), matching the exact decomposition."""
    from paddlepaddle_amd.ops import _loader as L
    paddle.set_device("gpu:0")
    K, N, M = 2048, 1024, 512
    q, s = Q.weight_quantize(_w(K, N, 4), "llm.int8")
    q, s = paddle.Tensor(q._t.cuda()), paddle.Tensor(s._t.cuda())
    g = torch.Generator(device="cuda").manual_seed(9)
    x = torch.randn(M, K, device="cuda", generator=g)
    x[:, 33] *= 30
    xb = x.bfloat16()
    L.reset_calls()
    y = Q.llm_int8_linear(paddle.Tensor(xb), q, None, s, threshold=6.0)
    torch.cuda.synchronize()
    assert sum(L.calls(n) for n in ("pa_gemm_bf16", "pa_gemm_bf16_pp")) >= 1
    xq, xo, sx, outl = Q._llm_split(xb, 6.0)
    exact = (sx[:, None] * (xq @ q._t.float().t()) + xo @ q._t.float().t()) * s._t.float()
    err = (y._t.float() - exact).abs().max().item() / exact.abs().max().item()
    assert err < 1e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize("M", [8, 48, 256])
def test_weight_only_dispatch_uses_cached_image_and_stays_exact(M):
    """Per-shape choice between the decode kernel and the bf16 GEMM on the cached dequantised image: every choice
    matches the fp32 reference, and a long input dequantises the weight once, not per call."""
    from paddlepaddle_amd.ops import _loader as L
    from paddlepaddle_amd.ops import quant as OQ
    paddle.set_device("gpu:0")
    K, N = 4096, 4096
    q, s = Q.weight_quantize(_w(K, N, 5), "weight_only_int8")
    q, s = paddle.Tensor(q._t.cuda()), paddle.Tensor(s._t.cuda())
    x = torch.randn(M, K, device="cuda").bfloat16()
    OQ._DQ_CACHE.clear()
    ys = [Q.weight_only_linear(paddle.Tensor(x), q, None, s, "int8") for _ in range(3)]
    L.reset_calls()
    y = Q.weight_only_linear(paddle.Tensor(x), q, None, s, "int8")
    torch.cuda.synchronize()
    assert L.calls("pa_wo_dequant") == 0  # the image is cached
    ref = _ref_gpu(x, q, s, "weight_only_int8", -1, None)
    for out in ys + [y]:
        err = (out._t.float() - ref).abs().max().item() / ref.abs().max().item()
        assert err < 1e-2, err
