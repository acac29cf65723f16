"""paddle.sparse on its own index / value algorithms vs dense references (rulebook convolutions vs dense
conv restricted to the active sites, SpMM / SpGEMM / SDDMM, reductions, reshapes, sparse attention).
Reference: test/legacy_test/test_sparse_*_op.py (dense-equivalence checks)."""
import numpy as np
import torch
import torch.nn.functional as TF

import paddlepaddle_amd as paddle
from paddlepaddle_amd import sparse


def _rand_sparse(shape, density, seed, dense_dims=0):
    g = torch.Generator().manual_seed(seed)
    d = torch.randn(shape, generator=g)
    keep = torch.rand(shape[:len(shape) - dense_dims], generator=g) < density
    if dense_dims:
        d = d * keep.reshape(keep.shape + (1,) * dense_dims)
    else:
        d = d * keep
    return d


def test_arith_matmul_reductions_match_dense():
    a = _rand_sparse((6, 5), 0.4, 0)
    b = _rand_sparse((6, 5), 0.4, 1)
    sa, sb = paddle.Tensor(a).to_sparse_coo(), paddle.Tensor(b).to_sparse_csr()
    np.testing.assert_allclose(sparse.add(sa, sb).to_dense().numpy(), (a + b).numpy(), rtol=1e-6)
    np.testing.assert_allclose(sparse.subtract(sa, sb).to_dense().numpy(), (a - b).numpy(), rtol=1e-6)
    np.testing.assert_allclose(sparse.multiply(sa, sb).to_dense().numpy(), (a * b).numpy(), rtol=1e-6)
    m = torch.randn(5, 3)
    np.testing.assert_allclose(sparse.matmul(sa, paddle.Tensor(m)).numpy(), (a @ m).numpy(), rtol=1e-5, atol=1e-6)
    c = _rand_sparse((5, 4), 0.5, 2)
    sp = sparse.matmul(sa, paddle.Tensor(c).to_sparse_coo())
    np.testing.assert_allclose(sp.to_dense().numpy(), (a @ c).numpy(), rtol=1e-5, atol=1e-6)
    x, y = torch.randn(6, 7), torch.randn(7, 5)
    mk = paddle.Tensor(b).to_sparse_csr()
    out = sparse.masked_matmul(paddle.Tensor(x), paddle.Tensor(y), mk).to_dense().numpy()
    np.testing.assert_allclose(out, ((x @ y) * (b != 0)).numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(sparse.sum(sa, axis=1).to_dense().numpy(), a.sum(1).numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(sparse.transpose(sa, [1, 0]).to_dense().numpy(), a.t().numpy())
    np.testing.assert_allclose(sparse.reshape(sa, [3, 10]).to_dense().numpy(), a.reshape(3, 10).numpy())
    np.testing.assert_allclose(sparse.slice(sa, [0, 1], [1, 2], [5, 4]).to_dense().numpy(), a[1:5, 2:4].numpy())


def _dense_conv_at_sites(d, w, stride, pad, subm):
    # d [N, D, H, W, C], w [kd, kh, kw, C, Co] -> dense conv, then the sparse output sites
    out = TF.conv3d(d.permute(0, 4, 1, 2, 3), w.permute(4, 3, 0, 1, 2), stride=stride, padding=pad)
    return out.permute(0, 2, 3, 4, 1)


def test_rulebook_conv3d_matches_dense_conv():
    x = _rand_sparse((2, 6, 6, 6, 4), 0.15, 3, dense_dims=1)
    w = torch.randn(3, 3, 3, 4, 5) * 0.2
    sx = paddle.Tensor(x).to_sparse_coo(sparse_dim=4)
    # regular conv: every output reachable from an active input
    out = sparse.nn.functional.conv3d(sx, paddle.Tensor(w), stride=2, padding=1)
    ref = _dense_conv_at_sites(x, w, 2, 1, False)
    np.testing.assert_allclose(out.to_dense().numpy(), ref.numpy(), rtol=1e-4, atol=1e-5)
    # submanifold conv: outputs only at the input's active sites
    out = sparse.nn.functional.subm_conv3d(sx, paddle.Tensor(w))
    ref = _dense_conv_at_sites(x, w, 1, 1, True)
    active = (x.abs().sum(-1) != 0).unsqueeze(-1)
    np.testing.assert_allclose(out.to_dense().numpy(), (ref * active).numpy(), rtol=1e-4, atol=1e-5)
    assert out.nnz() == int(active.sum())


def test_sparse_softmax_and_attention():
    a = _rand_sparse((4, 6), 0.5, 5)
    a[:, 0] = 1.0  # every row has an entry
    sa = paddle.Tensor(a).to_sparse_csr()
    sm = sparse.nn.functional.softmax(sa).to_dense().numpy()
    ref = torch.softmax(a.masked_fill(a == 0, float("-inf")), -1).numpy()
    np.testing.assert_allclose(sm, ref, rtol=1e-5, atol=1e-6)
    B, H, S, D = 1, 2, 6, 8
    q, k, v = torch.randn(B, H, S, D), torch.randn(B, H, S, D), torch.randn(B, H, S, D)
    mask = torch.ones(B * H, S, S).tril()
    sm_ = paddle.Tensor(mask).to_sparse_csr()
    out = sparse.nn.functional.attention(paddle.Tensor(q), paddle.Tensor(k), paddle.Tensor(v), sm_).numpy()
    ref = TF.scaled_dot_product_attention(q, k, v, is_causal=True).numpy()
    np.testing.assert_allclose(out, ref, rtol=1e-4, atol=1e-5)
