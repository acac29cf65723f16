"""paddle.incubate.framework: per-device RNG states with index registration.

Reference: python/paddle/incubate/framework/random.py:54 (get_rng_state), :137 (set_rng_state), :218
(register_rng_state_as_index). ``use_index=True`` works on indices of states registered with
``register_rng_state_as_index`` instead of the state tensors themselves."""
from __future__ import annotations

import torch

from ..framework import random as _random

_REGISTERED: dict = {}   # device kind -> list of registered state lists


def _kind(device):
    if device is None:
        from ..framework.place import get_device
        device = get_device()
    d = str(device).lower()
    return "cpu" if d.startswith("cpu") else "gpu"


def _states(kind):
    if kind == "cpu":
        return [torch.get_rng_state()]
    return torch.cuda.get_rng_state_all() if torch.cuda.is_available() else []


def _apply(kind, states):
    if kind == "cpu":
        torch.set_rng_state(states[0])
    elif torch.cuda.is_available():
        torch.cuda.set_rng_state_all(list(states))


def get_rng_state(device=None, use_index=False):
    """Generator states of the device (one per card for gpu); with use_index, the index of the state list the
    device currently runs (the last one set or registered, 0 if none)."""
    kind = _kind(device)
    if use_index:
        reg = _REGISTERED.setdefault(kind, [])
        cur = _states(kind)
        for i, st in enumerate(reg):
            if len(st) == len(cur) and all(torch.equal(a, b) for a, b in zip(st, cur)):
                return [i] * max(1, len(cur))
        return [0] * max(1, len(cur))
    return _states(kind)


def set_rng_state(state_list, device=None, use_index=False):
    kind = _kind(device)
    if use_index:
        reg = _REGISTERED.get(kind, [])
        idx = state_list[0] if isinstance(state_list, (list, tuple)) else int(state_list)
        if not 0 <= idx < len(reg):
            raise IndexError(f"set_rng_state: no registered rng state with index {idx} on {kind}")
        _apply(kind, reg[idx])
        return
    _apply(kind, state_list)


def register_rng_state_as_index(state_list=None, device=None):
    """Registers ``state_list`` (default: the current states) and returns its index per generator."""
    kind = _kind(device)
    reg = _REGISTERED.setdefault(kind, [])
    st = [s.clone() for s in (state_list if state_list is not None else _states(kind))]
    reg.append(st)
    return [len(reg) - 1] * max(1, len(st))


_ = _random
