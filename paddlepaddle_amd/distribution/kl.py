"""KL divergence registry. Reference: python/paddle/distribution/kl.py (register_kl, kl_divergence and the
registered pairs: Bernoulli, Beta, Binomial, Categorical, Cauchy, ContinuousBernoulli, Dirichlet, Normal,
MultivariateNormal, Uniform, Laplace, Geometric, Exponential, Gamma, LogNormal, Poisson, and the generic
exponential-family Bregman divergence)."""
from __future__ import annotations

import functools
import math

import torch

from ..framework.tensor import _wrap
from .distribution import Distribution, ExponentialFamily

_REGISTRY = {}


def register_kl(cls_p, cls_q):
    if not (issubclass(cls_p, Distribution) and issubclass(cls_q, Distribution)):
        raise TypeError("cls_p and cls_q must be subclass of Distribution")

    def deco(f):
        _REGISTRY[(cls_p, cls_q)] = f
        _dispatch.cache_clear()
        return f
    return deco


@functools.lru_cache(maxsize=None)
def _dispatch(tp, tq):
    matches = [(p, q) for p, q in _REGISTRY if issubclass(tp, p) and issubclass(tq, q)]
    if not matches:
        return None
    # most specific pair (shortest MRO distance)
    best = min(matches, key=lambda pq: (tp.__mro__.index(pq[0]), tq.__mro__.index(pq[1])))
    return _REGISTRY[best]


def kl_divergence(p, q):
    fn = _dispatch(type(p), type(q))
    if fn is None:
        raise NotImplementedError(f"No KL(p || q) is implemented for {type(p).__name__} and {type(q).__name__}")
    return fn(p, q)


from .bernoulli import Bernoulli  # noqa: E402
from .beta import Beta  # noqa: E402
from .binomial import Binomial  # noqa: E402
from .categorical import Categorical  # noqa: E402
from .cauchy import Cauchy  # noqa: E402
from .continuous_bernoulli import ContinuousBernoulli  # noqa: E402
from .dirichlet import Dirichlet  # noqa: E402
from .exponential import Exponential  # noqa: E402
from .gamma import Gamma  # noqa: E402
from .geometric import Geometric  # noqa: E402
from .laplace import Laplace  # noqa: E402
from .lognormal import LogNormal  # noqa: E402
from .multivariate_normal import MultivariateNormal  # noqa: E402
from .normal import Normal  # noqa: E402
from .poisson import Poisson  # noqa: E402
from .uniform import Uniform  # noqa: E402


@register_kl(Bernoulli, Bernoulli)
def _kl_bernoulli(p, q):
    a, b = p._p, q._p
    eps = torch.finfo(a.dtype).eps
    a, b = a.clamp(eps, 1 - eps), b.clamp(eps, 1 - eps)
    return _wrap(a * (torch.log(a) - torch.log(b)) + (1 - a) * (torch.log1p(-a) - torch.log1p(-b)))


@register_kl(Beta, Beta)
def _kl_beta(p, q):
    a1, b1, a2, b2 = p._a, p._b, q._a, q._b
    s1 = a1 + b1
    return _wrap(torch.lgamma(a2) + torch.lgamma(b2) - torch.lgamma(a2 + b2)
                 - (torch.lgamma(a1) + torch.lgamma(b1) - torch.lgamma(s1))
                 + (a1 - a2) * torch.digamma(a1) + (b1 - b2) * torch.digamma(b1)
                 + (a2 - a1 + b2 - b1) * torch.digamma(s1))


@register_kl(Binomial, Binomial)
def _kl_binomial(p, q):
    return p.kl_divergence(q)


@register_kl(Categorical, Categorical)
def _kl_categorical(p, q):
    return p.kl_divergence(q)


@register_kl(Cauchy, Cauchy)
def _kl_cauchy(p, q):
    num = (p._scale + q._scale).pow(2) + (p._loc - q._loc).pow(2)
    return _wrap(torch.log(num) - torch.log(4 * p._scale * q._scale))


@register_kl(ContinuousBernoulli, ContinuousBernoulli)
def _kl_cb(p, q):
    m = p.mean._t
    t1 = m * (torch.log(p._p) - torch.log(q._p)) + (1 - m) * (torch.log1p(-p._p) - torch.log1p(-q._p))
    return _wrap(t1 + p._log_norm() - q._log_norm())


@register_kl(Dirichlet, Dirichlet)
def _kl_dirichlet(p, q):
    a, b = p._c, q._c
    s = a.sum(-1)
    return _wrap(torch.lgamma(s) - torch.lgamma(b.sum(-1)) - (torch.lgamma(a) - torch.lgamma(b)).sum(-1)
                 + ((a - b) * (torch.digamma(a) - torch.digamma(s).unsqueeze(-1))).sum(-1))


@register_kl(Normal, Normal)
def _kl_normal(p, q):
    vr = (p._scale / q._scale).pow(2)
    t = ((p._loc - q._loc) / q._scale).pow(2)
    return _wrap(0.5 * (vr + t - 1 - torch.log(vr)))


@register_kl(MultivariateNormal, MultivariateNormal)
def _kl_mvn(p, q):
    k = p._loc.shape[-1]
    lp, lq = p._L, q._L
    shape = torch.broadcast_shapes(lp.shape, lq.shape)
    lp, lq = lp.expand(shape), lq.expand(shape)
    m = torch.linalg.solve_triangular(lq, lp, upper=False)
    diff = (q._loc - p._loc).expand(shape[:-1])
    y = torch.linalg.solve_triangular(lq, diff.unsqueeze(-1), upper=False).squeeze(-1)
    logdet = torch.log(torch.diagonal(lq, dim1=-2, dim2=-1)).sum(-1) - torch.log(
        torch.diagonal(lp, dim1=-2, dim2=-1)).sum(-1)
    return _wrap(0.5 * (m.pow(2).sum((-2, -1)) + y.pow(2).sum(-1) - k) + logdet)


@register_kl(Uniform, Uniform)
def _kl_uniform(p, q):
    inside = (q._low <= p._low) & (p._high <= q._high)
    r = torch.log((q._high - q._low) / (p._high - p._low))
    return _wrap(torch.where(inside, r, torch.full_like(r, float("inf"))))


@register_kl(Laplace, Laplace)
def _kl_laplace(p, q):
    r = p._scale / q._scale
    d = (p._loc - q._loc).abs()
    return _wrap(-torch.log(r) + d / q._scale + r * torch.exp(-d / p._scale) - 1)


@register_kl(Geometric, Geometric)
def _kl_geometric(p, q):
    return p.kl_divergence(q)


@register_kl(ExponentialFamily, ExponentialFamily)
def _kl_expfamily(p, q):
    """Bregman divergence of the log normaliser between the natural parameters (same family only)."""
    if type(p) is not type(q):
        raise NotImplementedError(f"KL between {type(p).__name__} and {type(q).__name__}")
    with torch.enable_grad():
        np_ = [t.detach().requires_grad_(True) for t in p._natural_parameters]
        ap = p._log_normalizer(*np_)
        grads = torch.autograd.grad(ap.sum(), np_)
    nq = [t.detach() for t in q._natural_parameters]
    aq = q._log_normalizer(*nq)
    kl = aq - ap.detach()
    for a, b, g in zip(np_, nq, grads):
        term = (b - a.detach()) * g
        extra = term.dim() - kl.dim()
        kl = kl - (term.sum(list(range(-extra, 0))) if extra > 0 else term)
    return _wrap(kl)


@register_kl(Exponential, Exponential)
def _kl_exponential(p, q):
    r = q._rate / p._rate
    return _wrap(r - torch.log(r) - 1)


@register_kl(Gamma, Gamma)
def _kl_gamma(p, q):
    a1, b1, a2, b2 = p._conc, p._rate, q._conc, q._rate
    return _wrap((a1 - a2) * torch.digamma(a1) - torch.lgamma(a1) + torch.lgamma(a2)
                 + a2 * (torch.log(b1) - torch.log(b2)) + a1 * (b2 - b1) / b1)


@register_kl(LogNormal, LogNormal)
def _kl_lognormal(p, q):
    return _kl_normal(p._base_normal, q._base_normal)


@register_kl(Poisson, Poisson)
def _kl_poisson(p, q):
    return p.kl_divergence(q)
