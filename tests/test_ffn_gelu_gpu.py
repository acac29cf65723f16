"""GELU backward fused into the data-gradient GEMM epilogue (csrc/kernels/gemm.hip pa_gemm_bf16_dgelu) and the
fused-backward FFN op built on it (ops/linear.py ffn_gelu / _FFNGeluFn), against fp32 references.
Reference: incubate/nn/functional/fused_transformer.py fused_feedforward (+ its _grad kernel)."""
import pytest
import torch

from paddlepaddle_amd.ops import _loader as Ld
from paddlepaddle_amd.ops import gemm as G
from paddlepaddle_amd.ops import linear as LIN

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()


def _gelu_grad(x):
    x = x.float()
    u = 0.7978845608028654 * (x + 0.044715 * x ** 3)
    t = torch.tanh(u)
    return 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * x * x)


@pytest.mark.parametrize("kern", [1, 2])
@pytest.mark.parametrize("M,N,K", [(4096, 2048, 1024), (1000, 768, 512), (512, 4096, 256)])
def test_gemm_dgelu_matches_fp32(M, N, K, kern):
    torch.manual_seed(kern)
    dy = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w2 = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)  # fc2 weight [in = N, out = K]
    pre = torch.randn(M, N, device="cuda", dtype=torch.bfloat16) * 2
    b = w2.t()  # dY . W2^T: B = W2^T read K-major in place
    assert G.gemm_dgelu_supported(dy, b, pre)
    dh, parts = G.gemm_dgelu(dy, b, pre, kern)
    ref = (dy.float() @ b.float()) * _gelu_grad(pre)
    assert _rel(dh, ref) < 1e-2
    assert parts.shape == (-(-M // 256), N)
    db = torch.empty(N, dtype=torch.float32, device="cuda")
    Ld.call("pa_fold_partials", Ld.ptr(parts), Ld.ptr(db), N, parts.shape[0], 0, Ld.stream_ptr())
    assert _rel(db, ref.sum(0)) < 1e-2


@pytest.mark.parametrize("backend", ["hip", "blas"])
def test_ffn_gelu_forward_backward_vs_fp32(backend):
    from paddlepaddle_amd.framework.flags import flag, set_flags
    prev = flag("FLAGS_gemm_backend", "auto")
    set_flags({"FLAGS_gemm_backend": backend})
    try:
        _ffn_case(backend)
    finally:
        set_flags({"FLAGS_gemm_backend": prev})


def _ffn_case(backend):
    torch.manual_seed(3)
    B, S, H, F = 2, 512, 1024, 4096
    x = torch.randn(B, S, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w1 = (torch.randn(H, F, device="cuda") * 0.03).to(torch.bfloat16).requires_grad_(True)
    b1 = (torch.randn(F, device="cuda") * 0.1).to(torch.bfloat16).requires_grad_(True)
    w2 = (torch.randn(F, H, device="cuda") * 0.03).to(torch.bfloat16).requires_grad_(True)
    b2 = (torch.randn(H, device="cuda") * 0.1).to(torch.bfloat16).requires_grad_(True)
    before = LIN.CALLS["dgrad_gelu_fused"]
    y = LIN.ffn_gelu(x, w1, b1, w2, b2)
    g = torch.randn_like(y)
    y.backward(g)
    if backend == "hip":
        assert LIN.CALLS["dgrad_gelu_fused"] == before + 1  # the fused epilogue ran, not the split fallback
    ps = [t.detach().float().requires_grad_(True) for t in (x, w1, b1, w2, b2)]
    xr, w1r, b1r, w2r, b2r = ps
    yr = torch.nn.functional.gelu(xr @ w1r + b1r, approximate="tanh") @ w2r + b2r
    yr.backward(g.float())
    assert _rel(y, yr) < 1e-2
    for t, r in zip((x, w1, b1, w2, b2), ps):
        assert _rel(t.grad, r.grad) < 3e-2
