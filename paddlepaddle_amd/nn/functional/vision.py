"""Vision functional ops. Reference: python/paddle/nn/functional/vision.py."""
from __future__ import annotations

import torch.nn.functional as F

from ...framework.tensor import _wrap
from ...tensor._helpers import T, shape_arg


def affine_grid(theta, out_shape, align_corners=True, name=None):
    return _wrap(F.affine_grid(T(theta), list(shape_arg(out_shape)), align_corners=align_corners))


def grid_sample(x, grid, mode="bilinear", padding_mode="zeros", align_corners=True, name=None):
    return _wrap(F.grid_sample(T(x), T(grid), mode=mode, padding_mode=padding_mode, align_corners=align_corners))
