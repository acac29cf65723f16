"""Grouped (all-experts) MoE GEMM + device routing: HIP kernels vs per-expert fp32 references.
Reference: paddle/phi/kernels/fusion/cutlass/fused_moe_kernel.cu, incubate/nn/functional/fused_moe.py:20."""
import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle
from paddlepaddle_amd.ops import _loader as L
from paddlepaddle_amd.ops import moe as M


def _offs(counts):
    o = np.zeros(len(counts) + 1, dtype=np.int32)
    o[1:] = np.cumsum(counts)
    return o


def _ref_grouped(x, w, offs, b=None):
    out = torch.zeros(x.shape[0], w.shape[2], dtype=torch.float32)
    for e in range(w.shape[0]):
        s, t = int(offs[e]), int(offs[e + 1])
        if t > s:
            y = x[s:t].float() @ w[e].float()
            if b is not None:
                y = y + b[e].float()
            out[s:t] = y
    return out


# ----------------------------------------------------------------------------------------- CPU
def test_route_fallback_groups_stably():
    eid = torch.tensor([2, 0, 1, 0, -1, 2, 1, 0])
    offs, perm = M.route(eid, 3)
    assert offs.tolist() == [0, 3, 5, 7]
    assert perm[:7].tolist() == [1, 3, 7, 2, 6, 0, 5]


def test_grouped_experts_cpu_matches_loop():
    paddle.seed(0)
    ge = paddle.incubate.distributed.models.moe.GroupedExperts(4, 16, 32, activation="gelu")
    x = paddle.randn([10, 16])
    ei = paddle.to_tensor(np.array([0, 3, 3, 1, 0, 2, 2, 2, 1, 0]))
    y = ge(x, ei).numpy()
    for r in range(10):
        e = int(ei.numpy()[r])
        h = torch.nn.functional.gelu(x._t[r] @ ge.w1._t[e] + ge.b1._t[e])
        np.testing.assert_allclose(y[r], (h @ ge.w2._t[e] + ge.b2._t[e]).detach().cpu().numpy(), rtol=1e-4,
                                   atol=1e-4)


def test_moe_layer_grouped_matches_layerlist():
    """MoELayer with GroupedExperts == MoELayer with the same experts as separate Layers."""
    paddle.seed(1)
    E, d, h = 4, 16, 24
    ge = paddle.incubate.distributed.models.moe.GroupedExperts(E, d, h, activation="relu")

    class FFN(paddle.nn.Layer):
        def __init__(self, e):
            super().__init__()
            self.fc1 = paddle.nn.Linear(d, h)
            self.fc2 = paddle.nn.Linear(h, d)
            self.fc1.weight.set_value(ge.w1[e])
            self.fc1.bias.set_value(ge.b1[e])
            self.fc2.weight.set_value(ge.w2[e])
            self.fc2.bias.set_value(ge.b2[e])

        def forward(self, x):
            return self.fc2(paddle.nn.functional.relu(self.fc1(x)))
    experts = paddle.nn.LayerList([FFN(e) for e in range(E)])
    gate = {"type": "naive", "top_k": 2}
    m1 = paddle.incubate.distributed.models.moe.MoELayer(d, ge, gate=gate)
    m2 = paddle.incubate.distributed.models.moe.MoELayer(d, experts, gate=gate)
    m2.gate.set_state_dict(m1.gate.state_dict())
    x = paddle.randn([2, 5, d])
    np.testing.assert_allclose(m1(x).numpy(), m2(x).numpy(), rtol=1e-5, atol=1e-5)


# ----------------------------------------------------------------------------------------- GPU
gpu = pytest.mark.gpu


def _need():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@gpu
@pytest.mark.parametrize("counts", [[300, 0, 129, 64, 1, 511, 128, 7], [5] * 64, [0, 0, 1000]])
def test_grouped_linear_fwd_bwd(counts):
    _need()
    torch.manual_seed(0)
    E, K, N = len(counts), 256, 192
    offs = _offs(counts)
    T = int(offs[-1]) + 37  # tail rows past offs[E] (dropped entries) must come out 0
    x = (torch.randn(T, K, device="cuda") * 0.5).bfloat16().requires_grad_()
    w = (torch.randn(E, K, N, device="cuda") * 0.05).bfloat16().requires_grad_()
    b = (torch.randn(E, N, device="cuda") * 0.1).bfloat16().requires_grad_()
    o = torch.tensor(offs, device="cuda")
    L.reset_calls()
    y = M.grouped_linear(x, w, o, b)
    assert L.calls("pa_grouped_gemm") == 1
    ref = _ref_grouped(x.detach().cpu(), w.detach().cpu(), offs, b.detach().cpu())
    torch.testing.assert_close(y.float().cpu(), ref, rtol=2e-2, atol=2e-2)
    dy = torch.randn(T, N, device="cuda").bfloat16()
    dy[int(offs[-1]):] = 0
    y.backward(dy)
    assert L.calls("pa_grouped_gemm") == 3
    xr = x.detach().cpu().float().requires_grad_()
    wr = w.detach().cpu().float().requires_grad_()
    br = b.detach().cpu().float().requires_grad_()
    _ref_grouped(xr, wr, offs, br).backward(dy.cpu().float())
    torch.testing.assert_close(x.grad.float().cpu(), xr.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(w.grad.float().cpu(), wr.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(b.grad.float().cpu(), br.grad, rtol=3e-2, atol=3e-2)


@gpu
def test_route_hip_matches_stable_sort():
    _need()
    torch.manual_seed(1)
    eid = torch.randint(-1, 16, (5000,), device="cuda")
    L.reset_calls()
    offs, perm = M.route(eid, 16)
    assert L.calls("pa_moe_route") == 1
    key = torch.where(eid < 0, torch.full_like(eid, 16), eid)
    ref = torch.argsort(key.cpu(), stable=True)
    n = int(offs[-1])
    assert n == int((eid >= 0).sum())
    assert torch.equal(perm[:n].cpu(), ref[:n])
    cnt = torch.bincount(eid[eid >= 0].cpu(), minlength=16)
    assert torch.equal(offs.cpu()[1:] - offs.cpu()[:-1], cnt.int())


@gpu
def test_fused_moe_matches_reference_and_captures():
    _need()
    torch.manual_seed(2)
    B, S, d, f, E, k = 2, 64, 128, 256, 8, 2
    x = paddle.Tensor((torch.randn(B, S, d, device="cuda") * 0.5).bfloat16())
    gw = paddle.Tensor(torch.randn(B, S, E, device="cuda"))
    w1 = paddle.Tensor((torch.randn(E, d, 2 * f, device="cuda") * 0.05).bfloat16())
    w2 = paddle.Tensor((torch.randn(E, f, d, device="cuda") * 0.05).bfloat16())
    L.reset_calls()
    out = paddle.incubate.nn.functional.fused_moe(x, gw, w1, w2, moe_topk=k)
    assert L.calls("pa_grouped_gemm") == 2 and L.calls("pa_moe_route") == 1
    xf = x._t.float().reshape(-1, d)
    p = torch.softmax(gw._t.float().reshape(-1, E), -1)
    val, idx = p.topk(k, -1)
    val = val / val.sum(-1, keepdim=True)
    ref = torch.zeros_like(xf)
    for t in range(xf.shape[0]):
        for j in range(k):
            e = int(idx[t, j])
            h = xf[t] @ w1._t[e].float()
            a, g = h.chunk(2)
            ref[t] += val[t, j] * ((torch.nn.functional.silu(a) * g) @ w2._t[e].float())
    torch.testing.assert_close(out._t.float().reshape(-1, d), ref, rtol=3e-2, atol=3e-2)
    # whole layer in a hipGraph: no host synchronisation inside
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        paddle.incubate.nn.functional.fused_moe(x, gw, w1, w2, moe_topk=k)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        o2 = paddle.incubate.nn.functional.fused_moe(x, gw, w1, w2, moe_topk=k)
    g.replay()
    torch.cuda.synchronize()
    torch.testing.assert_close(o2._t.float(), out._t.float(), rtol=0, atol=0)


@gpu
def test_moe_layer_grouped_gpu_backward():
    _need()
    paddle.seed(3)
    E, d, h = 8, 128, 256
    ge = paddle.incubate.distributed.models.moe.GroupedExperts(E, d, h, activation="gelu")
    layer = paddle.incubate.distributed.models.moe.MoELayer(d, ge, gate={"type": "naive", "top_k": 2})
    layer.to(dtype="bfloat16")
    x = paddle.randn([4, 32, d]).astype("bfloat16")
    x.stop_gradient = False
    L.reset_calls()
    y = layer(x)
    y.astype("float32").sum().backward()
    assert L.calls("pa_grouped_gemm") >= 6
    assert ge.w1.grad is not None and float(ge.w1.grad.astype("float32").abs().sum()) > 0
    assert x.grad is not None
