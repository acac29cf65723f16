"""incubate fused ops vs plain compositions, decode attention (masked / paged block MHA) vs full
attention recompute, LookAhead / ModelAverage / ASP, geometric segment & message passing ops.
Reference test strategy: test/legacy_test/test_fused_*_op.py, test_masked_multihead_attention_op.py,
test_block_multihead_attention.py, test_segment_ops.py, test_graph_send_recv_op.py."""
import math

import numpy as np
import torch

import paddlepaddle_amd as paddle
from paddlepaddle_amd.incubate.nn import functional as IF


def _np(t):
    return t.numpy()


def test_fused_norms_rope_act():
    rng = np.random.RandomState(0)
    x = paddle.to_tensor(rng.randn(4, 16).astype("float32"))
    r = paddle.to_tensor(rng.randn(4, 16).astype("float32"))
    w = paddle.to_tensor(rng.rand(16).astype("float32"))
    out, res = IF.fused_rms_norm(x, w, None, 1e-6, 1, residual=r)
    h = x.numpy() + r.numpy()
    ref = h / np.sqrt((h ** 2).mean(-1, keepdims=True) + 1e-6) * w.numpy()
    np.testing.assert_allclose(out.numpy(), ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(res.numpy(), h)
    ln = IF.fused_layer_norm(x, w, w, 1e-5, begin_norm_axis=1)
    m, v = x.numpy().mean(-1, keepdims=True), x.numpy().var(-1, keepdims=True)
    np.testing.assert_allclose(ln.numpy(), (x.numpy() - m) / np.sqrt(v + 1e-5) * w.numpy() + w.numpy(), rtol=1e-4,
                               atol=1e-5)
    q = paddle.randn([2, 8, 2, 16])
    k = paddle.randn([2, 8, 2, 16])
    qo, ko, vo = IF.fused_rotary_position_embedding(q, k, None)
    # rotation preserves per-pair norms
    np.testing.assert_allclose(np.linalg.norm(qo.numpy(), axis=-1), np.linalg.norm(q.numpy(), axis=-1), rtol=1e-4)
    assert vo is None
    a = paddle.randn([3, 8])
    np.testing.assert_allclose(IF.swiglu(a).numpy(),
                               (lambda u, g: u / (1 + np.exp(-u)) * g)(a.numpy()[:, :4], a.numpy()[:, 4:]), rtol=1e-5)
    b = paddle.randn([8])
    y = IF.fused_bias_act(a, b, act_method="relu")
    np.testing.assert_allclose(y.numpy(), np.maximum(a.numpy() + b.numpy(), 0))
    mm = IF.fused_matmul_bias(a, paddle.randn([8, 5]), paddle.zeros([5]))
    assert mm.shape == [3, 5]


def test_fused_layers_forward():
    paddle.seed(0)
    x = paddle.randn([2, 6, 16])
    attn = paddle.incubate.nn.FusedMultiHeadAttention(16, 4, dropout_rate=0.0, attn_dropout_rate=0.0)
    ffn = paddle.incubate.nn.FusedFeedForward(16, 32, dropout_rate=0.0)
    enc = paddle.incubate.nn.FusedTransformerEncoderLayer(16, 4, 32, dropout_rate=0.0)
    for l in (attn, ffn, enc):
        l.eval()
        assert l(x).shape == [2, 6, 16]


def test_masked_mha_decode_matches_full_attention():
    rng = np.random.RandomState(1)
    B, H, D, L = 2, 2, 8, 6
    cache = paddle.zeros([2, B, H, L, D])
    qs, ks, vs = [], [], []
    for t in range(4):
        x = rng.randn(B, 3 * H * D).astype("float32")
        mask = paddle.zeros([B, 1, 1, t + 1])
        out, cache = IF.masked_multihead_attention(paddle.to_tensor(x), cache, src_mask=mask)
        qkv = x.reshape(B, 3, H, D)
        qs.append(qkv[:, 0])
        ks.append(qkv[:, 1])
        vs.append(qkv[:, 2])
        K, V = np.stack(ks, 2), np.stack(vs, 2)  # [B,H,t+1,D]
        s = np.einsum("bhd,bhld->bhl", qkv[:, 0], K) / math.sqrt(D)
        p = np.exp(s - s.max(-1, keepdims=True))
        p /= p.sum(-1, keepdims=True)
        ref = np.einsum("bhl,bhld->bhd", p, V).reshape(B, H * D)
        np.testing.assert_allclose(out.numpy(), ref, rtol=1e-5, atol=1e-5)


def test_block_mha_prefill_then_decode():
    rng = np.random.RandomState(2)
    H, D, bs = 2, 8, 4
    lens = [5, 3]
    nblocks = 8
    kc = paddle.zeros([nblocks, H, bs, D])
    vc = paddle.zeros([nblocks, H, bs, D])
    tables = paddle.to_tensor(np.array([[0, 1, 2], [3, 4, 5]], dtype="int32"))
    toks = rng.randn(sum(lens), 3 * H * D).astype("float32")
    cu = np.array([0, 5, 8], dtype="int32")
    z = paddle.zeros([2], dtype="int32")
    out, _, kc, vc = IF.block_multihead_attention(
        paddle.to_tensor(toks), kc, vc, paddle.to_tensor(np.array(lens, "int32")), z,
        paddle.to_tensor(np.array(lens, "int32")), None, None, paddle.to_tensor(cu), paddle.to_tensor(cu), tables,
        block_size=bs)

    def full_attn(seq):  # seq [n, 3, H, D] causal
        q, k, v = seq[:, 0], seq[:, 1], seq[:, 2]
        s = np.einsum("qhd,khd->hqk", q, k) / math.sqrt(D)
        n = seq.shape[0]
        s = np.where(np.triu(np.ones((n, n), bool), 1)[None], -np.inf, s)
        p = np.exp(s - s.max(-1, keepdims=True))
        p /= p.sum(-1, keepdims=True)
        return np.einsum("hqk,khd->qhd", p, v).reshape(n, H * D)
    seqs = [toks[0:5].reshape(5, 3, H, D), toks[5:8].reshape(3, 3, H, D)]
    np.testing.assert_allclose(out.numpy()[0:5], full_attn(seqs[0]), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(out.numpy()[5:8], full_attn(seqs[1]), rtol=1e-4, atol=1e-5)
    # one decode step for both sequences
    new = rng.randn(2, 3 * H * D).astype("float32")
    out2, _, kc, vc = IF.block_multihead_attention(
        paddle.to_tensor(new), kc, vc, z, paddle.to_tensor(np.array(lens, "int32")),
        paddle.to_tensor(np.array([1, 1], "int32")), None, None, paddle.to_tensor(np.array([0, 1, 2], "int32")),
        paddle.to_tensor(np.array([0, 1, 2], "int32")), tables, block_size=bs)
    for b in range(2):
        full = np.concatenate([seqs[b], new[b].reshape(1, 3, H, D)])
        np.testing.assert_allclose(out2.numpy()[b], full_attn(full)[-1], rtol=1e-4, atol=1e-5)


def test_lookahead_modelaverage_asp():
    paddle.seed(0)
    lin = paddle.nn.Linear(8, 4)
    opt = paddle.incubate.LookAhead(paddle.optimizer.SGD(0.1, parameters=lin.parameters()), alpha=0.5, k=2)
    x = paddle.randn([4, 8])
    for _ in range(4):
        loss = (lin(x) ** 2).mean()
        loss.backward()
        opt.step()
        opt.clear_grad()
    ma = paddle.incubate.ModelAverage(0.5, parameters=lin.parameters(), min_average_window=2, max_average_window=4)
    w0 = lin.weight.numpy().copy()
    ma.step()
    with ma.apply():
        np.testing.assert_allclose(lin.weight.numpy(), w0, rtol=1e-6)
    net = paddle.nn.Sequential(paddle.nn.Linear(16, 8))
    paddle.incubate.asp.prune_model(net)
    w = net[0].weight
    assert abs(paddle.incubate.asp.calculate_density(w) - 0.5) < 1e-6
    assert paddle.incubate.asp.check_sparsity(w, 2, 4)


def test_geometric_ops():
    x = paddle.to_tensor(np.arange(12, dtype="float32").reshape(4, 3))
    seg = paddle.to_tensor(np.array([0, 0, 1, 2]))
    np.testing.assert_allclose(paddle.geometric.segment_sum(x, seg).numpy(), [[3, 5, 7], [6, 7, 8], [9, 10, 11]])
    np.testing.assert_allclose(paddle.geometric.segment_mean(x, seg).numpy()[0], [1.5, 2.5, 3.5])
    np.testing.assert_allclose(paddle.geometric.segment_max(x, seg).numpy()[0], [3, 4, 5])
    src = paddle.to_tensor(np.array([0, 1, 2, 0]))
    dst = paddle.to_tensor(np.array([1, 2, 1, 0]))
    out = paddle.geometric.send_u_recv(x, src, dst, "sum")
    np.testing.assert_allclose(out.numpy()[1], x.numpy()[0] + x.numpy()[2])
    row = paddle.to_tensor(np.array([1, 2, 0, 2, 0, 1]))
    colptr = paddle.to_tensor(np.array([0, 2, 4, 6]))
    nb, cnt = paddle.geometric.sample_neighbors(row, colptr, paddle.to_tensor(np.array([0, 2])), sample_size=1)
    assert cnt.numpy().tolist() == [1, 1]
    s, d, nodes = paddle.geometric.reindex_graph(paddle.to_tensor(np.array([0, 2])), nb, cnt)
    assert nodes.numpy()[0] == 0 and nodes.numpy()[1] == 2


def test_minimize_bfgs_and_lbfgs_match_scipy():
    """incubate.optimizer.functional: BFGS / L-BFGS with strong-Wolfe line search reach scipy's minimum of
    the Rosenbrock function and of a random SPD quadratic (closed-form minimiser)."""
    from scipy.optimize import minimize
    from paddlepaddle_amd.incubate.optimizer.functional import minimize_bfgs, minimize_lbfgs

    def rosen(x):
        t = x._t
        return paddle.Tensor((100 * (t[1:] - t[:-1] ** 2) ** 2 + (1 - t[:-1]) ** 2).sum())
    x0 = np.array([-1.2, 1.0, -1.2, 1.0])
    ref = minimize(lambda v: float(np.sum(100 * (v[1:] - v[:-1] ** 2) ** 2 + (1 - v[:-1]) ** 2)), x0,
                   method="BFGS").x
    for fn, kw in ((minimize_bfgs, {}), (minimize_lbfgs, {"history_size": 8})):
        ok, calls, x, fx, g = fn(rosen, paddle.to_tensor(x0), max_iters=300, dtype="float64", **kw)[:5]
        assert ok and calls > 1
        np.testing.assert_allclose(x.numpy(), ref, atol=1e-4)
        assert float(fx) < 1e-8
    rng = np.random.RandomState(0)
    A = rng.randn(6, 6)
    A = A @ A.T + 6 * np.eye(6)
    b = rng.randn(6)
    At, bt = paddle.to_tensor(A), paddle.to_tensor(b)

    def quad(x):
        return paddle.Tensor(0.5 * x._t @ At._t @ x._t - bt._t @ x._t)
    ok, _, x, _, _, H = minimize_bfgs(quad, paddle.zeros([6], dtype="float64"), dtype="float64")
    np.testing.assert_allclose(x.numpy(), np.linalg.solve(A, b), atol=1e-6)
    np.testing.assert_allclose(H.numpy(), np.linalg.inv(A), atol=5e-2)


def test_asp_add_supported_layer_custom_pruning():
    import numpy as np
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.incubate import asp

    class MyLayer(paddle.nn.Layer):
        def __init__(self):
            super().__init__()
            self.weight = self.create_parameter([8, 8])

        def forward(self, x):
            return x @ self.weight

    calls = []

    def prune(w, m, n, algo, name):  # keep the first n of every m along rows (a custom pattern)
        calls.append(name)
        mask = np.zeros_like(w)
        mask[:, ::m] = 1
        return w * mask, mask

    net = paddle.nn.Sequential(MyLayer(), paddle.nn.Linear(8, 8))
    assert len(asp._prunable(net)) == 1  # only the Linear before registration
    asp.add_supported_layer(MyLayer, prune)
    try:
        assert asp._snake("MyLayer") == "my_layer" and len(asp._prunable(net)) == 2
        masks = asp.prune_model(net, n=2, m=4)
        assert calls == [net[0].weight.name]
        w = net[0].weight.numpy()
        assert (w[:, 1::4] == 0).all() and (w[:, ::4] != 0).any()
        assert asp.check_sparsity(net[1].weight, 2, 4)
        assert len(masks) == 2
    finally:
        asp._supported.pop("my_layer", None)


def test_incubate_distributed_fleet_recompute_exports():
    import importlib
    mod = importlib.import_module("paddlepaddle_amd.incubate.distributed.fleet")
    from paddlepaddle_amd.distributed.fleet.recompute import recompute_sequential
    assert mod.recompute_sequential is recompute_sequential and callable(mod.recompute_hybrid)
