"""Random state. Reference: python/paddle/framework/random.py (seed, get/set_rng_state,
get/set_cuda_rng_state)."""
from __future__ import annotations

import random as _pyrandom

import numpy as np
import torch

_seed = None


def seed(seed):
    global _seed
    _seed = int(seed)
    torch.manual_seed(_seed)
    np.random.seed(_seed % (2**32))
    _pyrandom.seed(_seed)
    from .tensor import _wrap  # noqa: F401  (keeps import graph simple)
    return _Generator(_seed)


class _Generator:
    def __init__(self, s):
        self._seed = s

    def initial_seed(self):
        return self._seed

    def manual_seed(self, s):
        seed(s)
        return self


def get_rng_state(device=None):
    states = [torch.get_rng_state()]
    if torch.cuda.is_available():
        states += torch.cuda.get_rng_state_all()
    return states


def set_rng_state(state_list, device=None):
    torch.set_rng_state(state_list[0])
    if torch.cuda.is_available() and len(state_list) > 1:
        torch.cuda.set_rng_state_all(state_list[1:])


def get_cuda_rng_state():
    return torch.cuda.get_rng_state_all() if torch.cuda.is_available() else []


def set_cuda_rng_state(state_list):
    if torch.cuda.is_available():
        torch.cuda.set_rng_state_all(state_list)


def _default_generator(device):
    if device.type == "cuda":
        return torch.cuda.default_generators[device.index or 0]
    return torch.default_generator
