"""paddle.distribution. Reference: python/paddle/distribution/ (distribution.py, normal.py, uniform.py,
categorical.py, ..., kl.py, transform.py, transformed_distribution.py).

Each distribution keeps its parameters as device tensors and evaluates densities / samples with the
reparameterised device samplers (gradients flow through ``rsample``)."""
from __future__ import annotations

import math

import torch
import torch.distributions as D
from torch.distributions import transforms as _T

from ..framework.tensor import Tensor, _wrap

__all__ = ["Bernoulli", "Beta", "Categorical", "Cauchy", "Chi2", "ContinuousBernoulli", "Dirichlet", "Distribution",
           "Exponential", "ExponentialFamily", "Multinomial", "MultivariateNormal", "Normal", "Uniform",
           "kl_divergence", "register_kl", "Independent", "TransformedDistribution", "Laplace", "LogNormal",
           "LKJCholesky", "Gamma", "Gumbel", "Geometric", "Binomial", "Poisson", "StudentT"]


def _t(x, like=None):
    if x is None:
        return None
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, torch.Tensor):
        return x
    t = torch.as_tensor(x, dtype=torch.float32 if not isinstance(x, torch.Tensor) else None)
    if like is not None:
        t = t.to(like.device)
    return t


def _shape(s):
    if s is None:
        return torch.Size()
    if isinstance(s, int):
        return torch.Size([s])
    return torch.Size(list(s))


class Distribution:
    """Base: subclasses set ``self._d`` (a device distribution object)."""

    def __init__(self, batch_shape=(), event_shape=()):
        self._batch_shape = tuple(batch_shape)
        self._event_shape = tuple(event_shape)

    @property
    def batch_shape(self):
        return tuple(self._d.batch_shape) if hasattr(self, "_d") else self._batch_shape

    @property
    def event_shape(self):
        return tuple(self._d.event_shape) if hasattr(self, "_d") else self._event_shape

    @property
    def mean(self):
        return _wrap(self._d.mean)

    @property
    def variance(self):
        return _wrap(self._d.variance)

    @property
    def stddev(self):
        return _wrap(self._d.stddev)

    def sample(self, shape=()):
        with torch.no_grad():
            return _wrap(self._d.sample(_shape(shape)))

    def rsample(self, shape=()):
        return _wrap(self._d.rsample(_shape(shape)))

    def log_prob(self, value):
        return _wrap(self._d.log_prob(_t(value)))

    def prob(self, value):
        return _wrap(self._d.log_prob(_t(value)).exp())

    probs_fn = prob

    def entropy(self):
        return _wrap(self._d.entropy())

    def cdf(self, value):
        return _wrap(self._d.cdf(_t(value)))

    def icdf(self, value):
        return _wrap(self._d.icdf(_t(value)))

    def kl_divergence(self, other):
        return kl_divergence(self, other)

    def __repr__(self):
        return f"{type(self).__name__}(batch_shape={self.batch_shape}, event_shape={self.event_shape})"


class ExponentialFamily(Distribution):
    pass


class Normal(ExponentialFamily):
    def __init__(self, loc, scale, name=None):
        l = _t(loc)
        s = _t(scale, l)
        if not l.is_floating_point():
            l = l.float()
        self.loc, self.scale = _wrap(l), _wrap(s.to(l.dtype))
        self._d = D.Normal(l, s.to(l.dtype))

    def probs(self, value):
        return self.prob(value)


class LogNormal(Distribution):
    def __init__(self, loc, scale):
        l, s = _t(loc), _t(scale)
        self.loc, self.scale = _wrap(l), _wrap(s)
        self._d = D.LogNormal(l.float() if not l.is_floating_point() else l, s)


class Uniform(Distribution):
    def __init__(self, low, high, name=None):
        lo, hi = _t(low), _t(high)
        self.low, self.high = _wrap(lo), _wrap(hi)
        self._d = D.Uniform(lo.float() if not lo.is_floating_point() else lo, hi, validate_args=False)

    def log_prob(self, value):
        v = _t(value)
        lo, hi = self._d.low, self._d.high
        inside = (v >= lo) & (v < hi)
        shape = torch.broadcast_shapes(v.shape, lo.shape)
        lp = (-torch.log(hi - lo)).expand(shape)
        return _wrap(torch.where(inside.expand(shape), lp, torch.full(shape, float("-inf"), device=lp.device)))

    def probs(self, value):
        return self.prob(value)


class Categorical(Distribution):
    """paddle's Categorical takes (unnormalised, non-negative) ``logits`` treated as probabilities
    after normalisation, like the reference."""

    def __init__(self, logits, name=None):
        lg = _t(logits).float()
        self.logits = _wrap(lg)
        self._d = D.Categorical(probs=lg / lg.sum(-1, keepdim=True))

    def probs(self, value):
        v = _t(value).long()
        p = self._d.probs
        return _wrap(p.gather(-1, v.unsqueeze(-1) if v.dim() == p.dim() - 1 else v).squeeze(-1)
                     if v.dim() == p.dim() - 1 else p[..., v])

    def sample(self, shape=()):
        with torch.no_grad():
            return _wrap(self._d.sample(_shape(shape)))


class Bernoulli(ExponentialFamily):
    def __init__(self, probs, name=None):
        p = _t(probs).float()
        self.probs = _wrap(p)
        self._d = D.Bernoulli(probs=p)

    def rsample(self, shape=(), temperature=1.0):
        """Relaxed (Gumbel-softmax / concrete) sample, differentiable in ``probs``."""
        rd = D.RelaxedBernoulli(torch.as_tensor(temperature, device=self._d.probs.device), probs=self._d.probs)
        return _wrap(rd.rsample(_shape(shape)))


class ContinuousBernoulli(ExponentialFamily):
    def __init__(self, probs, lims=(0.499, 0.501)):
        self._d = D.ContinuousBernoulli(probs=_t(probs).float(), lims=lims)


class Beta(ExponentialFamily):
    def __init__(self, alpha, beta):
        a, b = _t(alpha).float(), _t(beta).float()
        self.alpha, self.beta = _wrap(a), _wrap(b)
        self._d = D.Beta(a, b)


class Dirichlet(ExponentialFamily):
    def __init__(self, concentration):
        c = _t(concentration).float()
        self.concentration = _wrap(c)
        self._d = D.Dirichlet(c)


class Exponential(ExponentialFamily):
    def __init__(self, rate):
        r = _t(rate).float()
        self.rate = _wrap(r)
        self._d = D.Exponential(r)


class Gamma(ExponentialFamily):
    def __init__(self, concentration, rate):
        c, r = _t(concentration).float(), _t(rate).float()
        self.concentration, self.rate = _wrap(c), _wrap(r)
        self._d = D.Gamma(c, r)


class Chi2(Gamma):
    def __init__(self, df):
        d = _t(df).float()
        self.df = _wrap(d)
        self._d = D.Chi2(d)


class Gumbel(Distribution):
    def __init__(self, loc, scale):
        l, s = _t(loc).float(), _t(scale).float()
        self.loc, self.scale = _wrap(l), _wrap(s)
        self._d = D.Gumbel(l, s)


class Laplace(Distribution):
    def __init__(self, loc, scale):
        l, s = _t(loc).float(), _t(scale).float()
        self.loc, self.scale = _wrap(l), _wrap(s)
        self._d = D.Laplace(l, s)


class Cauchy(Distribution):
    def __init__(self, loc, scale, name=None):
        l, s = _t(loc).float(), _t(scale).float()
        self.loc, self.scale = _wrap(l), _wrap(s)
        self._d = D.Cauchy(l, s)


class StudentT(Distribution):
    def __init__(self, df, loc, scale, name=None):
        self._d = D.StudentT(_t(df).float(), _t(loc).float(), _t(scale).float())


class Geometric(Distribution):
    """Number of failures before the first success (support {0, 1, ...}), like the reference."""

    def __init__(self, probs):
        p = _t(probs).float()
        self.probs = _wrap(p)
        self._d = D.Geometric(probs=p)

    def pmf(self, k):
        return self.prob(k)


class Binomial(Distribution):
    def __init__(self, total_count, probs):
        self._d = D.Binomial(total_count=_t(total_count).float(), probs=_t(probs).float())


class Poisson(ExponentialFamily):
    def __init__(self, rate):
        r = _t(rate).float()
        self.rate = _wrap(r)
        self._d = D.Poisson(r)


class Multinomial(Distribution):
    def __init__(self, total_count, probs):
        self.total_count = int(total_count)
        p = _t(probs).float()
        self.probs = _wrap(p)
        self._d = D.Multinomial(self.total_count, probs=p)


class MultivariateNormal(Distribution):
    def __init__(self, loc, covariance_matrix=None, precision_matrix=None, scale_tril=None):
        self.loc = _wrap(_t(loc).float())
        self._d = D.MultivariateNormal(_t(loc).float(), covariance_matrix=_t(covariance_matrix),
                                       precision_matrix=_t(precision_matrix), scale_tril=_t(scale_tril))


class LKJCholesky(Distribution):
    def __init__(self, dim=2, concentration=1.0, sample_method="onion"):
        self._d = D.LKJCholesky(dim, _t(concentration).float())


class Independent(Distribution):
    def __init__(self, base, reinterpreted_batch_rank):
        self.base = base
        self._d = D.Independent(base._d, reinterpreted_batch_rank)


class TransformedDistribution(Distribution):
    def __init__(self, base, transforms):
        self.base = base
        self.transforms = list(transforms)
        self._d = D.TransformedDistribution(base._d, [t._impl for t in self.transforms])


# ------------------------------------------------------------------------------ transforms
class Transform:
    _impl = None

    def forward(self, x):
        return _wrap(self._impl(_t(x)))

    def inverse(self, y):
        return _wrap(self._impl.inv(_t(y)))

    def forward_log_det_jacobian(self, x):
        xt = _t(x)
        return _wrap(self._impl.log_abs_det_jacobian(xt, self._impl(xt)))

    def inverse_log_det_jacobian(self, y):
        yt = _t(y)
        return _wrap(-self._impl.log_abs_det_jacobian(self._impl.inv(yt), yt))

    def __call__(self, x):
        if isinstance(x, Distribution):
            return TransformedDistribution(x, [self])
        return self.forward(x)


class AbsTransform(Transform):
    def __init__(self):
        self._impl = _T.AbsTransform()


class AffineTransform(Transform):
    def __init__(self, loc, scale):
        self.loc, self.scale = loc, scale
        self._impl = _T.AffineTransform(_t(loc), _t(scale))


class ExpTransform(Transform):
    def __init__(self):
        self._impl = _T.ExpTransform()


class PowerTransform(Transform):
    def __init__(self, power):
        self._impl = _T.PowerTransform(_t(power))


class SigmoidTransform(Transform):
    def __init__(self):
        self._impl = _T.SigmoidTransform()


class TanhTransform(Transform):
    def __init__(self):
        self._impl = _T.TanhTransform()


class SoftmaxTransform(Transform):
    def __init__(self):
        self._impl = _T.SoftmaxTransform()


class StickBreakingTransform(Transform):
    def __init__(self):
        self._impl = _T.StickBreakingTransform()


class ReshapeTransform(Transform):
    def __init__(self, in_event_shape, out_event_shape):
        self._impl = _T.ReshapeTransform(_shape(in_event_shape), _shape(out_event_shape))


class IndependentTransform(Transform):
    def __init__(self, base, reinterpreted_batch_rank):
        self._impl = _T.IndependentTransform(base._impl, reinterpreted_batch_rank)


class ChainTransform(Transform):
    def __init__(self, transforms):
        self._impl = _T.ComposeTransform([t._impl for t in transforms])


class StackTransform(Transform):
    def __init__(self, transforms, axis=0):
        self._impl = _T.StackTransform([t._impl for t in transforms], axis)


# ------------------------------------------------------------------------------ KL
_KL = {}


def register_kl(cls_p, cls_q):
    def deco(fn):
        _KL[(cls_p, cls_q)] = fn
        return fn
    return deco


def kl_divergence(p, q):
    for (a, b), fn in _KL.items():
        if isinstance(p, a) and isinstance(q, b):
            return fn(p, q)
    return _wrap(D.kl_divergence(p._d, q._d))


__all__ += ["Transform", "AbsTransform", "AffineTransform", "ChainTransform", "ExpTransform", "IndependentTransform",
            "PowerTransform", "ReshapeTransform", "SigmoidTransform", "SoftmaxTransform", "StackTransform",
            "StickBreakingTransform", "TanhTransform"]
