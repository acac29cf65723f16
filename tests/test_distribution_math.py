"""paddle.distribution with its own formulas, checked against scipy.stats (independent implementation) and
sample moments. Reference: python/paddle/distribution/*.py; test/distribution/ (scipy-based parity tests)."""
import numpy as np
import pytest
import scipy.stats as st

import paddlepaddle_amd as paddle
from paddlepaddle_amd import distribution as D

x = np.array([0.2, 0.5, 1.3], "float32")


def _np(t):
    return t.numpy()


@pytest.mark.parametrize("dist,ref,vals", [
    (lambda: D.Normal(0.3, 1.7), st.norm(0.3, 1.7), x),
    (lambda: D.Uniform(-1.0, 2.0), st.uniform(-1.0, 3.0), x),
    (lambda: D.Exponential(1.5), st.expon(scale=1 / 1.5), x),
    (lambda: D.Gamma(2.5, 1.5), st.gamma(2.5, scale=1 / 1.5), x),
    (lambda: D.Chi2(3.0), st.chi2(3.0), x),
    (lambda: D.Beta(2.0, 3.0), st.beta(2.0, 3.0), np.array([0.1, 0.5, 0.8], "float32")),
    (lambda: D.Laplace(0.5, 2.0), st.laplace(0.5, 2.0), x),
    (lambda: D.Cauchy(0.5, 2.0), st.cauchy(0.5, 2.0), x),
    (lambda: D.Gumbel(0.5, 2.0), st.gumbel_r(0.5, 2.0), x),
    (lambda: D.StudentT(4.0, 0.5, 2.0), st.t(4.0, 0.5, 2.0), x),
    (lambda: D.LogNormal(0.2, 0.7), st.lognorm(0.7, scale=np.exp(0.2)), x),
])
def test_continuous_log_prob_entropy_match_scipy(dist, ref, vals):
    d = dist()
    np.testing.assert_allclose(_np(d.log_prob(paddle.to_tensor(vals))), ref.logpdf(vals), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(float(d.entropy()), ref.entropy(), rtol=1e-4, atol=1e-5)
    if hasattr(d, "cdf"):
        try:
            c = d.cdf(paddle.to_tensor(vals))
        except NotImplementedError:
            return
        np.testing.assert_allclose(_np(c), ref.cdf(vals), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("dist,ref,vals", [
    (lambda: D.Poisson(3.5), st.poisson(3.5), np.array([0, 2, 7], "float32")),
    (lambda: D.Binomial(10, 0.3), st.binom(10, 0.3), np.array([0, 3, 10], "float32")),
    (lambda: D.Bernoulli(0.3), st.bernoulli(0.3), np.array([0, 1, 1], "float32")),
])
def test_discrete_log_prob_entropy_match_scipy(dist, ref, vals):
    d = dist()
    np.testing.assert_allclose(_np(d.log_prob(paddle.to_tensor(vals))), ref.logpmf(vals), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(float(d.entropy()), ref.entropy(), rtol=1e-4, atol=1e-5)


def test_dirichlet_mvn_multinomial_against_scipy():
    a = np.array([1.5, 2.0, 3.0], "float32")
    v = np.array([0.2, 0.3, 0.5], "float32")
    d = D.Dirichlet(paddle.to_tensor(a))
    np.testing.assert_allclose(float(d.log_prob(paddle.to_tensor(v))), st.dirichlet(a).logpdf(v), rtol=1e-4)
    np.testing.assert_allclose(float(d.entropy()), st.dirichlet(a).entropy(), rtol=1e-4)
    cov = np.array([[2.0, 0.3], [0.3, 1.0]], "float32")
    mvn = D.MultivariateNormal(paddle.to_tensor([0.5, -1.0]), covariance_matrix=paddle.to_tensor(cov))
    pt = np.array([0.1, 0.2], "float32")
    ref = st.multivariate_normal([0.5, -1.0], cov)
    np.testing.assert_allclose(float(mvn.log_prob(paddle.to_tensor(pt))), ref.logpdf(pt), rtol=1e-4)
    np.testing.assert_allclose(float(mvn.entropy()), ref.entropy(), rtol=1e-4)
    m = D.Multinomial(6, paddle.to_tensor([0.2, 0.3, 0.5]))
    c = np.array([1.0, 2.0, 3.0], "float32")
    np.testing.assert_allclose(float(m.log_prob(paddle.to_tensor(c))), st.multinomial(6, [0.2, 0.3, 0.5]).logpmf(c),
                               rtol=1e-4)
    np.testing.assert_allclose(float(m.entropy()), st.multinomial(6, [0.2, 0.3, 0.5]).entropy(), rtol=1e-4)


def test_kl_closed_forms_match_monte_carlo():
    paddle.seed(0)
    pairs = [(D.Normal(0.0, 1.0), D.Normal(0.5, 2.0)), (D.Gamma(2.0, 1.0), D.Gamma(3.0, 2.0)),
             (D.Beta(2.0, 3.0), D.Beta(1.5, 1.5)), (D.Laplace(0.0, 1.0), D.Laplace(1.0, 2.0)),
             (D.Exponential(1.0), D.Exponential(2.0))]
    for p, q in pairs:
        kl = float(D.kl_divergence(p, q))
        s = p.sample([200000])
        mc = float((p.log_prob(s) - q.log_prob(s)).mean())
        assert abs(kl - mc) < 0.02 + 0.02 * abs(kl), (type(p).__name__, kl, mc)
    # generic exponential-family (Bregman) KL == the closed form
    g1, g2 = D.Gamma(2.0, 1.0), D.Gamma(3.0, 2.0)
    from paddlepaddle_amd.distribution.kl import _kl_expfamily
    np.testing.assert_allclose(float(_kl_expfamily(g1, g2)), float(D.kl_divergence(g1, g2)), rtol=1e-5)


def test_rsample_carries_gradients_and_moments():
    paddle.seed(1)
    loc = paddle.to_tensor(0.5, stop_gradient=False)
    s = D.Normal(loc, 2.0).rsample([4096])
    s.mean().backward()
    np.testing.assert_allclose(float(loc.grad), 1.0, rtol=1e-6)
    g = D.Gamma(paddle.to_tensor(3.0), paddle.to_tensor(2.0)).sample([100000])
    np.testing.assert_allclose(float(g.mean()), 1.5, rtol=0.02)
    lkj = D.LKJCholesky(3, 2.0)
    L = lkj.sample([5])
    corr = L.numpy() @ np.swapaxes(L.numpy(), -1, -2)
    np.testing.assert_allclose(np.diagonal(corr, axis1=-2, axis2=-1), np.ones((5, 3)), rtol=1e-5)
    assert np.isfinite(lkj.log_prob(L).numpy()).all()


def test_transforms_roundtrip_and_log_det():
    xs = paddle.to_tensor([[0.3, -1.2, 2.0]])
    for t in [D.ExpTransform(), D.SigmoidTransform(), D.TanhTransform(), D.AffineTransform(1.0, 2.5),
              D.PowerTransform(2.0), D.StickBreakingTransform()]:
        inp = xs.abs() if isinstance(t, D.PowerTransform) else xs
        y = t.forward(inp)
        np.testing.assert_allclose(t.inverse(y).numpy(), inp.numpy(), rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(t.inverse_log_det_jacobian(y).numpy(),
                                   -np.broadcast_to(t.forward_log_det_jacobian(inp).numpy(),
                                                    t.inverse_log_det_jacobian(y).numpy().shape), rtol=1e-4, atol=1e-5)
    td = D.TransformedDistribution(D.Normal(0.0, 1.0), [D.AffineTransform(1.0, 2.0)])
    v = paddle.to_tensor([0.3, 2.0])
    np.testing.assert_allclose(td.log_prob(v).numpy(), st.norm(1.0, 2.0).logpdf(v.numpy()), rtol=1e-5)
