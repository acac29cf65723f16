"""paddle.einsum. Reference: python/paddle/tensor/einsum.py. Contractions lower to hipBLASLt GEMMs."""
from __future__ import annotations

import torch

from ..amp.state import maybe_cast
from ..framework.tensor import _wrap
from ._helpers import T


def einsum(equation, *operands):
    if len(operands) == 1 and isinstance(operands[0], (list, tuple)):
        operands = operands[0]
    ts = maybe_cast("einsum", *[T(o) for o in operands])
    return _wrap(torch.einsum(equation, *ts))
