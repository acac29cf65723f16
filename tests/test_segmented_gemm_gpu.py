"""Segmented-operand GEMMs on the ping-pong kernel (csrc/kernels/gemm.hip pa_gemm_bf16_pp_segs) and the
sibling-linear op built on them (ops/linear.py multi_linear), against fp32 references."""
import pytest
import torch

from paddlepaddle_amd.ops import gemm as G
from paddlepaddle_amd.ops import linear as LIN

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()


@pytest.mark.parametrize("M,K,widths", [(4096, 1024, [512, 256, 128]), (2048, 4096, [4096, 512, 512]),
                                        (1000, 512, [256, 136])])
def test_gemm_nseg_matches_fp32(M, K, widths):
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    ws = [torch.randn(K, n, device="cuda", dtype=torch.bfloat16) * 0.05 for n in widths]
    assert G.gemm_nseg_supported(x, ws)
    out = G.gemm_nseg(x, ws)
    ref = x.float() @ torch.cat([w.float() for w in ws], 1)
    assert out.shape == (M, sum(widths)) and _rel(out, ref) < 1e-2


@pytest.mark.parametrize("M,N,ks", [(4096, 1024, [512, 256, 128]), (2048, 4096, [4096, 512, 512])])
def test_gemm_kseg_matches_fp32_with_own_leading_dims(M, N, ks):
    torch.manual_seed(1)
    # dx = sum_i dy_i W_i^T: A_i [M, k_i] K-major with ld k_i, B_i = W_i^T (W_i [N, k_i]: K-major, ld k_i)
    dys = [torch.randn(M, k, device="cuda", dtype=torch.bfloat16) for k in ks]
    ws = [torch.randn(N, k, device="cuda", dtype=torch.bfloat16) * 0.05 for k in ks]
    As, Bs = dys, [w.t() for w in ws]
    assert G.gemm_kseg_supported(As, Bs)
    out = G.gemm_kseg(As, Bs)
    ref = sum(a.float() @ b.float() for a, b in zip(As, Bs))
    assert _rel(out, ref) < 1e-2


def test_multi_linear_forward_backward_vs_fp32():
    torch.manual_seed(2)
    x = torch.randn(2, 1024, 1024, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    ws = [(torch.randn(1024, n, device="cuda") * 0.03).to(torch.bfloat16).requires_grad_(True)
          for n in (1024, 256, 256)]
    outs = LIN.multi_linear(x, ws)
    assert len(outs) == 3 and outs[0].shape == (2, 1024, 1024) and outs[2].shape == (2, 1024, 256)
    gs = [torch.randn_like(o) for o in outs[:2]]  # the third output is unused: its gradient is None
    torch.autograd.backward(outs[:2], gs)
    xr = x.detach().float().requires_grad_(True)
    wr = [w.detach().float().requires_grad_(True) for w in ws]
    refs = [xr @ w for w in wr]
    torch.autograd.backward(refs[:2], [g.float() for g in gs])
    for o, r in zip(outs, refs):
        assert _rel(o, r) < 1e-2
    assert _rel(x.grad, xr.grad) < 2e-2
    for w, r in zip(ws[:2], wr[:2]):
        assert _rel(w.grad, r.grad) < 2e-2
    assert ws[2].grad is None or float(ws[2].grad.float().abs().max()) == 0.0
