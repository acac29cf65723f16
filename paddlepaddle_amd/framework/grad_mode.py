"""Gradient-mode switches. Reference: python/paddle/base/dygraph/base.py (no_grad_, enable_grad,
set_grad_enabled, is_grad_enabled)."""
from __future__ import annotations

import functools

import torch


class _GradMode:
    _mode = False

    def __init__(self):
        self._prev = []

    def __enter__(self):
        self._prev.append(torch.is_grad_enabled())
        torch.set_grad_enabled(self._mode)
        return self

    def __exit__(self, *exc):
        torch.set_grad_enabled(self._prev.pop())
        return False

    def __call__(self, func):
        mode = self._mode

        @functools.wraps(func)
        def wrapper(*a, **k):
            prev = torch.is_grad_enabled()
            torch.set_grad_enabled(mode)
            try:
                return func(*a, **k)
            finally:
                torch.set_grad_enabled(prev)
        return wrapper


class no_grad(_GradMode):
    """``with paddle.no_grad():`` / ``@paddle.no_grad()`` / ``@paddle.no_grad``."""
    _mode = False

    def __new__(cls, func=None):
        self = super().__new__(cls)
        if callable(func):
            self.__init__()
            return self(func)
        return self

    def __init__(self, func=None):
        super().__init__()


class enable_grad(_GradMode):
    _mode = True


class set_grad_enabled:
    """Sets the mode on construction, so both ``paddle.set_grad_enabled(False)`` (a plain call) and
    ``with paddle.set_grad_enabled(False):`` (restores the previous mode on exit) work."""

    def __init__(self, mode):
        self._prev = torch.is_grad_enabled()
        self._mode = bool(mode)
        torch.set_grad_enabled(self._mode)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        torch.set_grad_enabled(self._prev)
        return False

    def __call__(self, func):
        torch.set_grad_enabled(self._prev)  # as a decorator the mode applies only inside func
        mode = self._mode

        @functools.wraps(func)
        def wrapper(*a, **k):
            prev = torch.is_grad_enabled()
            torch.set_grad_enabled(mode)
            try:
                return func(*a, **k)
            finally:
                torch.set_grad_enabled(prev)
        return wrapper


def is_grad_enabled():
    """False in static-graph mode (gradients come from append_backward there), else the dygraph mode."""
    from ..static.executor import _static_mode
    return False if _static_mode.enabled else torch.is_grad_enabled()


no_grad_ = no_grad
