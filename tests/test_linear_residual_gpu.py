"""Residual add in the output-projection GEMM (csrc/kernels/gemm.hip pa_gemm_bf16_res, ops.fused_linear
residual=) and the LLaMA training layer that uses it, against fp32 references and the unfused layer.
Reference: incubate/nn/functional/fused_rms_norm.py:59 (residual=)."""
import numpy as np
import pytest
import torch

from paddlepaddle_amd.ops import _loader as Ld
from paddlepaddle_amd.ops import gemm as G
from paddlepaddle_amd.ops import linear as LIN

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()


@pytest.mark.parametrize("bias", [False, True])
@pytest.mark.parametrize("M,N,K", [(4096, 4096, 4096), (1000, 768, 512), (4096, 5120, 1024)])
def test_gemm_res_matches_fp32(M, N, K, bias):
    torch.manual_seed(0)
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(K, N, device="cuda") * 0.05).to(torch.bfloat16)
    r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16) if bias else None
    assert G.res_supported(a, w, r)
    before = Ld.CALLS.get("pa_gemm_bf16_res", 0)
    y = G.gemm_res(a, w, r, bias=b)
    assert Ld.CALLS["pa_gemm_bf16_res"] == before + 1
    ref = a.float() @ w.float() + r.float() + (b.float() if bias else 0)
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("backend", ["hip", "blas"])
def test_fused_linear_residual_forward_backward_vs_fp32(backend):
    from paddlepaddle_amd.framework.flags import flag, set_flags
    prev = flag("FLAGS_gemm_backend", "auto")
    set_flags({"FLAGS_gemm_backend": backend})
    try:
        torch.manual_seed(1)
        x = torch.randn(2, 512, 1024, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        w = (torch.randn(1024, 2048, device="cuda") * 0.03).to(torch.bfloat16).requires_grad_(True)
        r = torch.randn(2, 512, 2048, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        before = Ld.CALLS.get("pa_gemm_bf16_res", 0)
        y = LIN.fused_linear(x, w, residual=r)
        if backend == "hip":
            assert Ld.CALLS["pa_gemm_bf16_res"] == before + 1
        g = torch.randn_like(y)
        y.backward(g)
        xr, wr, rr = (t.detach().float().requires_grad_(True) for t in (x, w, r))
        yr = xr @ wr + rr
        yr.backward(g.float())
        assert _rel(y, yr) < 1e-2
        for t, ref in ((x, xr), (w, wr), (r, rr)):
            assert _rel(t.grad, ref.grad) < 2e-2
    finally:
        set_flags({"FLAGS_gemm_backend": prev})


def test_llama_layer_fused_residual_matches_unfused():
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.models import llama as LM
    paddle.set_device("gpu")
    paddle.seed(0)
    cfg = LM.LlamaConfig.tiny(hidden_size=512, num_attention_heads=4, num_key_value_heads=2, intermediate_size=1024)
    model = LM.LlamaForCausalLM(cfg)
    model.to(dtype="bfloat16")
    ids = torch.randint(0, cfg.vocab_size, (2, 256), generator=torch.Generator().manual_seed(1))
    x = paddle.to_tensor(ids.numpy(), place=paddle.CUDAPlace(0))
    crit = LM.LlamaPretrainingCriterion(cfg)

    def run():
        for p in model.parameters():
            p.clear_gradient()
        loss = crit(model(x[:, :-1]), x[:, 1:])
        loss.backward()
        return float(loss), {n: p.grad._t.float().clone() for n, p in model.named_parameters()}

    before = LIN.CALLS["linear_residual"]
    l1, g1 = run()
    assert LIN.CALLS["linear_residual"] == before + 2 * cfg.num_hidden_layers  # o_proj and down_proj per layer
    orig = LM._proj_res
    LM._proj_res = lambda layer, h, residual: orig(layer, h, None) if residual is None else \
        LM._wrap(layer(h)._t + residual._t)
    try:
        l0, g0 = run()
    finally:
        LM._proj_res = orig
    np.testing.assert_allclose(l1, l0, rtol=2e-3)
    for n in g0:
        assert _rel(g1[n], g0[n]) < 3e-2, n
