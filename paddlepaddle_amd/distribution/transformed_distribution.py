"""TransformedDistribution. Reference: python/paddle/distribution/transformed_distribution.py."""
from __future__ import annotations

import torch

from ..framework.tensor import _wrap
from .distribution import Distribution, _shape, _t
from .transform import ChainTransform, Transform


class TransformedDistribution(Distribution):
    def __init__(self, base, transforms):
        if not isinstance(base, Distribution):
            raise TypeError(f"Expected type of 'base' is Distribution, but got {type(base)}.")
        if not all(isinstance(t, Transform) for t in transforms):
            raise TypeError("All element of transforms must be Transform type.")
        self._base = base
        self._transforms = list(transforms)
        chain = ChainTransform(self._transforms)
        self._chain = chain
        shape = tuple(base.batch_shape) + tuple(base.event_shape)
        out_shape = chain.forward_shape(shape)
        ev_rank = max(chain._event_rank, len(base.event_shape))
        cut = len(out_shape) - ev_rank
        super().__init__(out_shape[:cut], out_shape[cut:])

    @property
    def base(self):
        return self._base

    @property
    def transforms(self):
        return self._transforms

    def sample(self, shape=()):
        x = self._base.sample(shape)._t
        return _wrap(self._chain._forward(x).detach())

    def rsample(self, shape=()):
        x = self._base.rsample(shape)._t
        return _wrap(self._chain._forward(x))

    def log_prob(self, value):
        y = _t(value)
        if not y.is_floating_point():
            y = y.float()
        lp = 0.0
        ev = len(self.event_shape)
        for t in reversed(self._transforms):
            x = t._inverse(y)
            ld = t._forward_log_det_jacobian(x)
            extra = ev - t._event_rank
            if extra > 0 and ld.dim() >= extra:
                ld = ld.sum(list(range(-extra, 0)))
            lp = lp - ld
            y = x
        base_lp = self._base.log_prob(_wrap(y))._t
        extra = ev - len(self._base.event_shape)
        if extra > 0:
            base_lp = base_lp.sum(list(range(-extra, 0)))
        return _wrap(lp + base_lp)
