"""Distribution base classes. Reference: python/paddle/distribution/distribution.py,
exponential_family.py.

Every distribution in this package evaluates its densities, moments, entropies and divergences with its own
formulas on device tensors (torch ops on HBM, fp32 / fp64 as given); sampling draws from the device RNG
(paddle.seed) and reparameterises where the distribution allows, so ``rsample`` carries gradients."""
from __future__ import annotations

import math
import numbers

import numpy as np
import torch

from ..framework.tensor import Tensor, _wrap


def _t(x, dtype=None, like=None):
    """Tensor / number / list / ndarray -> torch tensor (floats default to float32, like the reference)."""
    if x is None:
        return None
    if isinstance(x, Tensor):
        t = x._t
    elif isinstance(x, torch.Tensor):
        t = x
    elif isinstance(x, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(x))
        if t.dtype == torch.float64 and dtype is None:
            pass
    else:
        t = torch.as_tensor(x, dtype=torch.float32 if isinstance(x, (numbers.Real, list, tuple)) else None)
    if dtype is not None:
        t = t.to(dtype)
    if like is not None and t.device != like.device:
        t = t.to(like.device)
    return t


def _ft(x, like=None):
    """Floating parameter tensor."""
    t = _t(x, like=like)
    if not t.is_floating_point():
        t = t.float()
    return t


def _shape(s):
    if s is None:
        return ()
    if isinstance(s, (int, np.integer)):
        return (int(s),)
    if isinstance(s, Tensor):
        return tuple(int(v) for v in s._t.reshape(-1).tolist())
    return tuple(int(v) for v in s)


def _bshape(*ts):
    return tuple(torch.broadcast_shapes(*[t.shape for t in ts]))


def _eps(t):
    return torch.finfo(t.dtype).eps


def _tiny(t):
    return torch.finfo(t.dtype).tiny


class Distribution:
    """Base of all distributions: ``batch_shape`` (independent draws) x ``event_shape`` (one draw)."""

    has_rsample = False

    def __init__(self, batch_shape=(), event_shape=()):
        self._batch_shape = tuple(batch_shape)
        self._event_shape = tuple(event_shape)

    @property
    def batch_shape(self):
        return self._batch_shape

    @property
    def event_shape(self):
        return self._event_shape

    def _extend_shape(self, sample_shape):
        return tuple(_shape(sample_shape)) + self._batch_shape + self._event_shape

    @property
    def mean(self):
        raise NotImplementedError

    @property
    def variance(self):
        raise NotImplementedError

    @property
    def stddev(self):
        return _wrap(self.variance._t.sqrt())

    def sample(self, shape=()):
        with torch.no_grad():
            out = self.rsample(shape)
        return _wrap(out._t.detach())

    def rsample(self, shape=()):
        raise NotImplementedError(f"{type(self).__name__} has no reparameterised sampler")

    def log_prob(self, value):
        raise NotImplementedError

    def prob(self, value):
        return _wrap(self.log_prob(value)._t.exp())

    def probs(self, value):
        return self.prob(value)

    def entropy(self):
        raise NotImplementedError

    def cdf(self, value):
        raise NotImplementedError

    def icdf(self, value):
        raise NotImplementedError

    def kl_divergence(self, other):
        from .kl import kl_divergence
        return kl_divergence(self, other)

    # helpers for subclasses
    @staticmethod
    def _validate_args(*args):
        return all(isinstance(a, (Tensor, torch.Tensor)) for a in args)

    @staticmethod
    def _to_tensor(*args):
        ts = [_ft(a) for a in args]
        if len(ts) > 1:
            shape = _bshape(*ts)
            dt = torch.float64 if any(t.dtype == torch.float64 for t in ts) else ts[0].dtype
            ts = [t.to(dt).expand(shape) for t in ts]
        return [_wrap(t) for t in ts]

    @staticmethod
    def _logits_to_probs(logits, is_binary=False):
        lt = _t(logits)
        return _wrap(torch.sigmoid(lt) if is_binary else torch.softmax(lt, -1))

    @staticmethod
    def _probs_to_logits(probs, is_binary=False):
        p = _t(probs)
        eps = _eps(p)
        p = p.clamp(eps, 1 - eps)
        return _wrap(torch.log(p) - torch.log1p(-p) if is_binary else torch.log(p))

    def __repr__(self):
        return f"{type(self).__name__}(batch_shape={self.batch_shape}, event_shape={self.event_shape})"


class ExponentialFamily(Distribution):
    """p(x; theta) = h(x) exp(<eta(theta), T(x)> - A(eta)). Subclasses give the natural parameters and the
    log normaliser A; the entropy (and the generic exponential-family KL in kl.py) follow by autograd:
    H = A(eta) - <eta, grad A(eta)> - E[log h(x)] (reference exponential_family.py)."""

    @property
    def _natural_parameters(self):
        raise NotImplementedError

    def _log_normalizer(self, *natural):
        raise NotImplementedError

    @property
    def _mean_carrier_measure(self):
        raise NotImplementedError

    def entropy(self):
        with torch.enable_grad():
            nat = [p.detach().requires_grad_(True) for p in self._natural_parameters]
            a = self._log_normalizer(*nat)
            grads = torch.autograd.grad(a.sum(), nat, create_graph=True)
        ent = a.detach() - self._mean_carrier_measure
        for n, g in zip(nat, grads):
            ent = ent - (n.detach() * g.detach()).reshape(a.shape + (-1,)).sum(-1) if n.dim() > a.dim() \
                else ent - n.detach() * g.detach()
        return _wrap(ent)
