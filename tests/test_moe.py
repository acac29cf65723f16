"""MoE: expert-parallel MoELayer (gloo, 2 ranks x 2 local experts) == single-process layer with all 4
experts; gates (naive / gshard capacity / switch); fused_moe vs a per-token reference.
Reference test strategy: test/collective/fleet/test_moe_api.py / test_fused_moe_op.py."""
import os
import sys

import numpy as np
import torch

from test_distributed_cpu import ROOT, _setup, _spawn


class _Expert:
    @staticmethod
    def make(paddle, d, h):
        return paddle.nn.Sequential(paddle.nn.Linear(d, h), paddle.nn.GELU(), paddle.nn.Linear(h, d))


def _build(paddle, world, rank, group):
    from paddlepaddle_amd.parallel.moe import MoELayer, NaiveGate
    paddle.seed(3)
    d, h, E = 8, 16, 4
    experts_all = [_Expert.make(paddle, d, h) for _ in range(E)]
    gate = NaiveGate(d, E // world, world, topk=2)
    local = paddle.nn.LayerList(experts_all[rank * (E // world):(rank + 1) * (E // world)])
    return MoELayer(d, local, gate=gate, moe_group=group), experts_all


def _tokens(rank):
    return torch.randn(2, 5, 8, generator=torch.Generator().manual_seed(10 + rank))


def _moe_worker(rank, world, port, q):
    paddle = _setup(rank, world, port)
    group = paddle.distributed.new_group([0, 1])
    layer, _ = _build(paddle, world, rank, group)
    x = paddle.Tensor(_tokens(rank).requires_grad_(True))
    x.stop_gradient = False
    y = layer(x)
    (y * y).sum().backward()
    grads = {f"{rank * 2 + i}.{k}": p.grad.numpy() for i, e in enumerate(layer.experts)
             for k, p in e.named_parameters()}
    q.put((rank, y.numpy(), x.grad.numpy(), grads))
    paddle.distributed.barrier()


def test_expert_parallel_moe_matches_single_process():
    res = _spawn(_moe_worker)
    sys.path.insert(0, ROOT)
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    layer, experts = _build(paddle, 1, 0, None)
    ref_grads = {}
    for rank, y, gx, grads in res:
        x = paddle.Tensor(_tokens(rank).requires_grad_(True))
        x.stop_gradient = False
        yr = layer(x)
        np.testing.assert_allclose(y, yr.numpy(), rtol=1e-5, atol=1e-6)
        (yr * yr).sum().backward()
        np.testing.assert_allclose(gx, x.grad.numpy(), rtol=1e-5, atol=1e-6)
    for i, e in enumerate(layer.experts):
        for k, p in e.named_parameters():
            ref_grads[f"{i}.{k}"] = p.grad.numpy()
    got = {}
    for _, _, _, g in res:
        got.update(g)
    assert set(got) == set(ref_grads)
    for k in ref_grads:
        np.testing.assert_allclose(got[k], ref_grads[k], rtol=1e-5, atol=1e-6, err_msg=k)


def test_gates_capacity_and_aux_loss():
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.parallel.moe import GShardGate, SwitchGate, MoELayer
    paddle.seed(0)
    g = GShardGate(8, 4, 1, capacity=(0.5, 0.5), random_routing=False)
    val, idx = g(paddle.randn([64, 8]))
    idx = idx.numpy()
    # capacity = ceil(0.5 * 64 / 4) = 8 assignments per expert at most
    counts = np.bincount(idx[idx >= 0], minlength=4)
    assert counts.max() <= 8 and (idx == -1).any()
    assert float(g.get_loss()) > 0
    s = SwitchGate(8, 4, 1, capacity=(2.0, 2.0))
    v, i = s(paddle.randn([32, 8]))
    assert i.shape == [32, 1]
    experts = paddle.nn.LayerList([paddle.nn.Linear(8, 8) for _ in range(4)])
    m = MoELayer(8, experts, gate={"type": "switch", "top_k": 1})
    out = m(paddle.randn([2, 16, 8]))
    assert out.shape == [2, 16, 8]


def test_fused_moe_matches_reference():
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.incubate.nn.functional import fused_moe
    rng = np.random.RandomState(0)
    E, d, f = 4, 8, 6
    x = rng.randn(2, 3, d).astype("float32")
    gl = rng.randn(2, 3, E).astype("float32")
    w1 = rng.randn(E, d, 2 * f).astype("float32") * 0.3
    w2 = rng.randn(E, f, d).astype("float32") * 0.3
    out = fused_moe(paddle.to_tensor(x), paddle.to_tensor(gl), paddle.to_tensor(w1), paddle.to_tensor(w2),
                    moe_topk=2).numpy()
    ref = np.zeros_like(x).reshape(-1, d)
    xf, gf = x.reshape(-1, d), gl.reshape(-1, E)
    for t in range(xf.shape[0]):
        p = np.exp(gf[t] - gf[t].max())
        p /= p.sum()
        top = np.argsort(-p)[:2]
        w = p[top] / p[top].sum()
        for e, we in zip(top, w):
            h = xf[t] @ w1[e]
            a, b = h[:f], h[f:]
            ref[t] += we * ((a / (1 + np.exp(-a)) * b) @ w2[e])
    np.testing.assert_allclose(out.reshape(-1, d), ref, rtol=1e-4, atol=1e-5)
