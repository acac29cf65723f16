"""Independent: reinterpret batch dims of a base distribution as event dims. Reference:
python/paddle/distribution/independent.py."""
from __future__ import annotations

from ..framework.tensor import _wrap
from .distribution import Distribution


class Independent(Distribution):
    def __init__(self, base, reinterpreted_batch_rank):
        if not isinstance(base, Distribution):
            raise TypeError(f"Expected type of 'base' is Distribution, but got {type(base)}")
        if not 0 < reinterpreted_batch_rank <= len(base.batch_shape):
            raise ValueError(f"Expected 0 < reinterpreted_batch_rank <= {len(base.batch_shape)}, but got "
                             f"{reinterpreted_batch_rank}")
        self._base = base
        self._reinterpreted_batch_rank = reinterpreted_batch_rank
        shape = tuple(base.batch_shape) + tuple(base.event_shape)
        cut = len(base.batch_shape) - reinterpreted_batch_rank
        super().__init__(shape[:cut], shape[cut:])

    @property
    def mean(self):
        return self._base.mean

    @property
    def variance(self):
        return self._base.variance

    def sample(self, shape=()):
        return self._base.sample(shape)

    def rsample(self, shape=()):
        return self._base.rsample(shape)

    def _sum_rightmost(self, t):
        n = self._reinterpreted_batch_rank
        return t.sum(list(range(-n, 0))) if n > 0 else t

    def log_prob(self, value):
        return _wrap(self._sum_rightmost(self._base.log_prob(value)._t))

    def prob(self, value):
        return _wrap(self.log_prob(value)._t.exp())

    def entropy(self):
        return _wrap(self._sum_rightmost(self._base.entropy()._t))
