"""SyncBatchNorm's split-phase HIP kernels (pa_bn_reduce_nhwc + pa_bn_fwd_nhwc apply + pa_bn_bwd_apply_nhwc)
against fp32 batch norm. One process: the cross-rank all-reduce is the identity here (its cross-rank
semantics are covered by the 2-rank gloo test in test_distributed_cpu.py)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(8, 14, 14, 64), (4, 7, 7, 256), (2, 28, 28, 40)])
def test_sync_bn_hip_matches_fp32(shape, monkeypatch):
    import torch.distributed as dist
    from paddlepaddle_amd.ops import _loader as L
    from paddlepaddle_amd.ops.bn import sync_batch_norm
    monkeypatch.setattr(dist, "all_reduce", lambda t, *a, **k: None)
    g = torch.Generator().manual_seed(3)
    C = shape[-1]
    x = (torch.randn(*shape, generator=g) * 2 + 0.3).to("cuda", torch.bfloat16).requires_grad_(True)
    w = torch.linspace(0.5, 1.5, C, device="cuda").requires_grad_(True)
    b = torch.linspace(-0.3, 0.2, C, device="cuda").requires_grad_(True)
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    y = sync_batch_norm(x, w, b, rm, rv, 0.9, 1e-5, channel_last=True, pg=None)
    gy = torch.randn(*shape, generator=g).to("cuda", torch.bfloat16)
    y.backward(gy)
    assert L.calls("pa_bn_reduce_nhwc") == 2 and L.calls("pa_bn_fwd_nhwc") == 1
    assert L.calls("pa_bn_bwd_apply_nhwc") == 1
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_(True)
    wr, br = w.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    rmr, rvr = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    yr = F.batch_norm(xr, rmr, rvr, wr, br, True, 0.1, 1e-5)
    yr.backward(gy.float().permute(0, 3, 1, 2))
    torch.testing.assert_close(y.float(), yr.permute(0, 2, 3, 1), atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad.permute(0, 2, 3, 1), atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(w.grad, wr.grad, atol=5e-2, rtol=1e-2)
    torch.testing.assert_close(b.grad, br.grad, atol=5e-2, rtol=1e-2)
    torch.testing.assert_close(rm, rmr, atol=1e-3, rtol=1e-3)
    # torch's running var uses the unbiased batch variance; paddle's keeps the biased one
    n = x.numel() // C
    torch.testing.assert_close(rv, 0.9 + (rvr - 0.9) * (n - 1) / n, atol=1e-3, rtol=1e-3)
