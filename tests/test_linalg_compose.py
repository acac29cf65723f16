"""paddle.linalg routines composed from the LU / QR / SVD / eigen / Cholesky / triangular-solve primitives
(tensor/linalg.py), checked against numpy / scipy / torch.linalg in float64."""
import numpy as np
import pytest
import scipy.linalg
import torch

import paddlepaddle_amd as paddle

L = paddle.linalg
rs = np.random.RandomState(0)


def _t(a):
    return paddle.to_tensor(a)


def _n(t):
    return t.numpy()


@pytest.mark.parametrize("p", [None, "fro", "nuc", 1, -1, 2, -2, np.inf, -np.inf])
def test_matrix_norms(p):
    a = rs.randn(3, 4, 5)
    got = _n(L.norm(_t(a), p=p, axis=[1, 2]))
    want = np.linalg.norm(a, ord=p, axis=(1, 2))
    np.testing.assert_allclose(got, want, rtol=1e-10)


@pytest.mark.parametrize("p", [0, 1, 2, 3.5, np.inf, -np.inf])
def test_vector_norms(p):
    a = rs.randn(4, 6)
    a[0, 1] = 0
    np.testing.assert_allclose(_n(L.vector_norm(_t(a), p=p, axis=1)), np.linalg.norm(a, ord=p, axis=1), rtol=1e-10)
    np.testing.assert_allclose(_n(L.vector_norm(_t(a), p=p, axis=1, keepdim=True)).shape, (4, 1))


def test_det_slogdet_solve_inv():
    a = rs.randn(3, 5, 5)
    a[1, 2] = a[1, 0] * 2  # singular member of the batch
    np.testing.assert_allclose(_n(L.det(_t(a))), np.linalg.det(a), rtol=1e-9, atol=1e-12)
    s, l = _n(L.slogdet(_t(a)))
    ws, wl = np.linalg.slogdet(a)
    np.testing.assert_allclose(s[[0, 2]], ws[[0, 2]])
    np.testing.assert_allclose(l[[0, 2]], wl[[0, 2]], rtol=1e-10)
    assert s[1] == 0 or abs(l[1]) > 20  # singular: sign 0 / log|det| -> -inf (or rounding-sized)
    b = rs.randn(3, 5, 2)
    good = a[[0, 2]]
    np.testing.assert_allclose(_n(L.solve(_t(good), _t(b[[0, 2]]))), np.linalg.solve(good, b[[0, 2]]), rtol=1e-9)
    np.testing.assert_allclose(_n(L.solve(_t(good[0]), _t(b[0, :, 0]))), np.linalg.solve(good[0], b[0, :, 0]),
                               rtol=1e-9)
    xr = _n(L.solve(_t(good), _t(b[[0, 2]].transpose(0, 2, 1)), left=False))
    np.testing.assert_allclose(xr @ good, b[[0, 2]].transpose(0, 2, 1), atol=1e-10)
    np.testing.assert_allclose(_n(L.inv(_t(good))), np.linalg.inv(good), rtol=1e-9)
    np.testing.assert_allclose(_n(paddle.inverse(_t(good))), np.linalg.inv(good), rtol=1e-9)


def test_det_and_solve_gradients():
    a = torch.randn(4, 4, dtype=torch.float64) + 4 * torch.eye(4, dtype=torch.float64)
    b = torch.randn(4, 2, dtype=torch.float64)
    torch.autograd.gradcheck(lambda m: L.det(paddle.Tensor(m))._t, (a.requires_grad_(),))
    torch.autograd.gradcheck(lambda m, r: L.solve(paddle.Tensor(m), paddle.Tensor(r))._t,
                             (a.detach().requires_grad_(), b.requires_grad_()))


@pytest.mark.parametrize("upper", [False, True])
def test_cholesky_solve_inverse(upper):
    m = rs.randn(4, 4)
    a = m @ m.T + 4 * np.eye(4)
    u = np.linalg.cholesky(a)
    if upper:
        u = u.T
    b = rs.randn(4, 3)
    np.testing.assert_allclose(_n(L.cholesky_solve(_t(b), _t(u), upper=upper)), np.linalg.solve(a, b), rtol=1e-9)
    np.testing.assert_allclose(_n(L.cholesky_inverse(_t(u), upper=upper)), np.linalg.inv(a), rtol=1e-9)


@pytest.mark.parametrize("shape", [(5, 5), (6, 4), (4, 6), (2, 5, 5)])
def test_lu_unpack_reconstructs(shape):
    a = rs.randn(*shape)
    lu_, piv = L.lu(_t(a))
    P, Lo, U = L.lu_unpack(lu_, piv)
    np.testing.assert_allclose(_n(P) @ _n(Lo) @ _n(U), a, atol=1e-12)
    tp, tl, tu = torch.lu_unpack(*torch.linalg.lu_factor(torch.tensor(a)))
    np.testing.assert_allclose(_n(P), tp.numpy())


def test_matrix_rank_pinv_cond():
    a = rs.randn(6, 4) @ rs.randn(4, 5)  # rank 4
    assert int(L.matrix_rank(_t(a))) == 4
    assert int(L.matrix_rank(_t(a), tol=1e6)) == 0
    h = a @ a.T
    assert int(L.matrix_rank(_t(h), hermitian=True)) == 4
    np.testing.assert_allclose(_n(L.pinv(_t(a))), np.linalg.pinv(a), rtol=1e-7, atol=1e-10)
    np.testing.assert_allclose(_n(L.pinv(_t(h), hermitian=True)), np.linalg.pinv(h, hermitian=True), rtol=1e-6,
                               atol=1e-10)
    sq = rs.randn(2, 4, 4)
    for p in (None, 2, -2, "fro", "nuc", 1, -1, np.inf, -np.inf):
        np.testing.assert_allclose(_n(L.cond(_t(sq), p)), np.linalg.cond(sq, p), rtol=1e-8)


@pytest.mark.parametrize("driver", ["gels", "gelsy", "gelsd", "gelss"])
def test_lstsq_drivers(driver):
    a, b = rs.randn(8, 3), rs.randn(8, 2)
    sol, res, rank, sv = L.lstsq(_t(a), _t(b), driver=driver)
    want, wres, wrank, wsv = np.linalg.lstsq(a, b, rcond=None)
    np.testing.assert_allclose(_n(sol), want, rtol=1e-9)
    np.testing.assert_allclose(_n(res), wres, rtol=1e-9)
    if driver != "gels":
        assert int(rank) == wrank
    if driver in ("gelsd", "gelss"):
        np.testing.assert_allclose(_n(sv), wsv, rtol=1e-10)
    wide = rs.randn(2, 5)  # minimum-norm solution of an under-determined system
    np.testing.assert_allclose(_n(L.lstsq(_t(wide), _t(b[:2]), driver=driver)[0]),
                               np.linalg.lstsq(wide, b[:2], rcond=None)[0], rtol=1e-9)


def test_matrix_power_and_exp():
    a = rs.randn(3, 4, 4)
    for n in (0, 1, 5, 6, -3):
        np.testing.assert_allclose(_n(L.matrix_power(_t(a), n)),
                                   np.linalg.matrix_power(a, n), rtol=1e-8, atol=1e-10)
    big = rs.randn(2, 5, 5) * np.array([0.01, 30.0])[:, None, None]  # scaling: s = 0 and s > 0 in one batch
    want = np.stack([scipy.linalg.expm(m) for m in big])
    np.testing.assert_allclose(_n(L.matrix_exp(_t(big))), want, rtol=1e-9)
    np.testing.assert_allclose(_n(L.matrix_exp(_t(big[:1].astype("float32")))), want[:1], rtol=1e-5)


def test_multi_dot_chain_order_and_vectors():
    mats = [rs.randn(10, 100), rs.randn(100, 5), rs.randn(5, 50), rs.randn(50)]
    np.testing.assert_allclose(_n(L.multi_dot([_t(m) for m in mats])), np.linalg.multi_dot(mats), rtol=1e-10)
    v = rs.randn(10)
    np.testing.assert_allclose(_n(L.multi_dot([_t(v), _t(mats[0]), _t(mats[1])])),
                               np.linalg.multi_dot([v, mats[0], mats[1]]), rtol=1e-10)


def test_householder_product_and_ormqr():
    a = torch.tensor(rs.randn(2, 6, 4))
    geqrf, tau = torch.geqrf(a)
    np.testing.assert_allclose(_n(L.householder_product(_t(geqrf.numpy()), _t(tau.numpy()))),
                               torch.linalg.householder_product(geqrf, tau).numpy(), atol=1e-12)
    c = torch.tensor(rs.randn(2, 6, 3))
    for left, tr in ((True, False), (True, True)):
        np.testing.assert_allclose(_n(L.ormqr(_t(geqrf.numpy()), _t(tau.numpy()), _t(c.numpy()), left, tr)),
                                   torch.ormqr(geqrf, tau, c, left, tr).numpy(), atol=1e-12)
    c2 = torch.tensor(rs.randn(2, 3, 6))
    np.testing.assert_allclose(_n(L.ormqr(_t(geqrf.numpy()), _t(tau.numpy()), _t(c2.numpy()), False, False)),
                               torch.ormqr(geqrf, tau, c2, False, False).numpy(), atol=1e-12)


def test_cov_corrcoef_weights():
    x = rs.randn(3, 7)
    fw = rs.randint(1, 4, size=7)
    aw = rs.rand(7)
    np.testing.assert_allclose(_n(L.cov(_t(x))), np.cov(x), rtol=1e-10)
    np.testing.assert_allclose(_n(L.cov(_t(x), ddof=False)), np.cov(x, ddof=0), rtol=1e-10)
    np.testing.assert_allclose(_n(L.cov(_t(x.T), rowvar=False)), np.cov(x.T, rowvar=False), rtol=1e-10)
    np.testing.assert_allclose(_n(L.cov(_t(x), fweights=_t(fw), aweights=_t(aw))),
                               np.cov(x, fweights=fw, aweights=aw), rtol=1e-10)
    np.testing.assert_allclose(_n(L.corrcoef(_t(x))), np.corrcoef(x), rtol=1e-10)


def test_vecdot_and_lowrank():
    a, b = rs.randn(3, 4), rs.randn(3, 4)
    np.testing.assert_allclose(_n(L.vecdot(_t(a), _t(b))), (a * b).sum(-1), rtol=1e-12)
    paddle.seed(1)
    lr = rs.randn(40, 3) @ rs.randn(3, 30)
    u, s, v = L.svd_lowrank(_t(lr), q=5)
    np.testing.assert_allclose(_n(u) @ np.diag(_n(s)) @ _n(v).T, lr, atol=1e-8)
    u, s, v = L.pca_lowrank(_t(lr.T), q=4)
    c = lr.T - lr.T.mean(0, keepdims=True)
    np.testing.assert_allclose(_n(s)[:3], np.linalg.svd(c, compute_uv=False)[:3], rtol=1e-8)
