"""Random sampling ops. Reference: python/paddle/tensor/random.py."""
from __future__ import annotations

import torch

from ..framework import dtype as _dt
from ..framework.place import _get_torch_device
from ..framework.tensor import Tensor, _wrap
from ._helpers import T, dtype_arg, shape_arg


def _fd(dtype):
    return dtype_arg(dtype) if dtype is not None else _dt.default_dtype().torch_dtype


def rand(shape, dtype=None, name=None):
    return _wrap(torch.rand(shape_arg(shape), dtype=_fd(dtype), device=_get_torch_device()))


def randn(shape, dtype=None, name=None):
    return _wrap(torch.randn(shape_arg(shape), dtype=_fd(dtype), device=_get_torch_device()))


standard_normal = randn


def randint(low=0, high=None, shape=[1], dtype=None, name=None):
    if high is None:
        low, high = 0, low
    return _wrap(torch.randint(low, high, shape_arg(shape), dtype=dtype_arg(dtype or "int64"),
                               device=_get_torch_device()))


def randint_like(x, low=0, high=None, dtype=None, name=None):
    if high is None:
        low, high = 0, low
    t = T(x)
    return _wrap(torch.randint(low, high, t.shape, dtype=dtype_arg(dtype) if dtype else t.dtype, device=t.device))


def randperm(n, dtype="int64", name=None):
    return _wrap(torch.randperm(n, dtype=dtype_arg(dtype), device=_get_torch_device()))


def uniform(shape, dtype=None, min=-1.0, max=1.0, seed=0, name=None):  # noqa: A002
    g = None
    if seed:
        g = torch.Generator(device=_get_torch_device()).manual_seed(seed)
    t = torch.empty(shape_arg(shape), dtype=_fd(dtype), device=_get_torch_device())
    t.uniform_(min, max, generator=g)
    return _wrap(t)


def uniform_(x, min=-1.0, max=1.0, seed=0, name=None):  # noqa: A002
    with torch.no_grad():
        x._t.uniform_(min, max)
    return x


def normal(mean=0.0, std=1.0, shape=None, name=None):
    if isinstance(mean, Tensor) or isinstance(std, Tensor):
        m = T(mean) if isinstance(mean, Tensor) else torch.tensor(mean)
        s = T(std) if isinstance(std, Tensor) else torch.tensor(std)
        m, s = torch.broadcast_tensors(m.float(), s.float().to(m.device))
        return _wrap(torch.normal(m, s))
    return _wrap(torch.normal(float(mean), float(std), shape_arg(shape), device=_get_torch_device(),
                              dtype=_dt.default_dtype().torch_dtype))


def normal_(x, mean=0.0, std=1.0, name=None):
    with torch.no_grad():
        x._t.normal_(mean, std)
    return x


def log_normal(mean=1.0, std=2.0, shape=None, name=None):
    return _wrap(torch.exp(normal(mean, std, shape)._t))


def log_normal_(x, mean=1.0, std=2.0, name=None):
    with torch.no_grad():
        x._t.log_normal_(mean, std)
    return x


def bernoulli(x, p=None, name=None):
    t = T(x)
    return _wrap(torch.bernoulli(t) if p is None else torch.bernoulli(torch.full_like(t, p)))


def bernoulli_(x, p=0.5, name=None):
    with torch.no_grad():
        x._t.bernoulli_(T(p) if isinstance(p, Tensor) else p)
    return x


def binomial(count, prob, name=None):
    return _wrap(torch.binomial(T(count).float(), T(prob).float()).to(torch.int64))


def poisson(x, name=None):
    return _wrap(torch.poisson(T(x)))


def standard_gamma(x, name=None):
    return _wrap(torch._standard_gamma(T(x)))


def multinomial(x, num_samples=1, replacement=False, name=None):
    return _wrap(torch.multinomial(T(x), num_samples, replacement))


def exponential_(x, lam=1.0, name=None):
    with torch.no_grad():
        x._t.exponential_(lam)
    return x


def cauchy_(x, loc=0, scale=1, name=None):
    with torch.no_grad():
        x._t.cauchy_(loc, scale)
    return x


def geometric_(x, probs, name=None):
    with torch.no_grad():
        x._t.geometric_(probs)
    return x


def uniform_random_batch_size_like(input, shape, dtype="float32", input_dim_idx=0, output_dim_idx=0, min=-1.0,  # noqa: A002
                                   max=1.0, seed=0):  # noqa: A002
    """U(min, max) samples of ``shape`` with dim ``output_dim_idx`` replaced by ``input.shape[input_dim_idx]``.
    Reference: python/paddle/tensor/random.py uniform_random_batch_size_like."""
    shp = list(shape)
    shp[output_dim_idx] = T(input).shape[input_dim_idx]
    return uniform(shp, dtype=dtype, min=min, max=max, seed=seed)
