"""Reference: python/paddle/nn/functional/distance.py."""
from __future__ import annotations

import torch.nn.functional as F

from ...framework.tensor import _wrap
from ...tensor._helpers import T


def pairwise_distance(x, y, p=2.0, epsilon=1e-6, keepdim=False, name=None):
    return _wrap(F.pairwise_distance(T(x), T(y), p, epsilon, keepdim))


def pdist(x, p=2.0, name=None):
    return _wrap(F.pdist(T(x), p))
