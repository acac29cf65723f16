"""incubate optimizers. Reference: python/paddle/incubate/optimizer/{lookahead.py,modelaverage.py}."""
from __future__ import annotations

import torch

from ..framework.grad_mode import no_grad


class LookAhead:
    """k fast steps of the inner optimizer, then slow weights move alpha toward the fast ones."""

    def __init__(self, inner_optimizer, alpha=0.5, k=5, name=None):
        assert 0.0 <= alpha <= 1.0 and k >= 1
        self.inner_optimizer = inner_optimizer
        self.alpha, self.k = alpha, k
        self._step = 0
        self._slow = {}
        self._parameter_list = inner_optimizer._parameter_list

    @no_grad()
    def step(self):
        self.inner_optimizer.step()
        self._step += 1
        if self._step % self.k == 0:
            for p in self._parameter_list:
                slow = self._slow.get(id(p))
                if slow is None:
                    slow = self._slow[id(p)] = p._t.detach().clone()
                    continue
                slow.add_(p._t.detach() - slow, alpha=self.alpha)
                p._t.detach().copy_(slow)
        elif self._step == 1:
            for p in self._parameter_list:
                self._slow.setdefault(id(p), p._t.detach().clone())

    def clear_grad(self, set_to_zero=True):
        self.inner_optimizer.clear_grad(set_to_zero)

    clear_gradients = clear_grad

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        loss.backward()
        self.step()

    def state_dict(self):
        sd = dict(self.inner_optimizer.state_dict())
        sd["@lookahead_step"] = self._step
        return sd

    def set_state_dict(self, sd):
        self._step = int(sd.get("@lookahead_step", 0))
        self.inner_optimizer.set_state_dict({k: v for k, v in sd.items() if k != "@lookahead_step"})


class ModelAverage:
    """Sliding-window parameter averaging; apply() swaps averaged weights in, restore() swaps back."""

    def __init__(self, average_window_rate, parameters=None, min_average_window=10000, max_average_window=10000,
                 name=None):
        self.rate = average_window_rate
        self.min_w, self.max_w = min_average_window, max_average_window
        self._params = list(parameters) if parameters is not None else []
        self._sum = {id(p): torch.zeros_like(p._t, dtype=torch.float32) for p in self._params}
        self._n = 0
        self._backup = None

    @no_grad()
    def step(self):
        self._n += 1
        for p in self._params:
            self._sum[id(p)].add_(p._t.detach().float())
        window = max(self.min_w, min(self.max_w, int(self._n * self.rate) or 1))
        if self._n > window:  # restart accumulation from the current average
            for p in self._params:
                self._sum[id(p)].mul_(window / self._n)
            self._n = window

    @no_grad()
    def apply(self, executor=None, need_restore=True):
        self._backup = {id(p): p._t.detach().clone() for p in self._params} if need_restore else None
        if self._n:
            for p in self._params:
                p._t.detach().copy_((self._sum[id(p)] / self._n).to(p._t.dtype))
        outer = self

        class _Ctx:
            def __enter__(self):
                return outer

            def __exit__(self, *a):
                if need_restore:
                    outer.restore()
        return _Ctx()

    @no_grad()
    def restore(self, executor=None):
        if self._backup is None:
            return
        for p in self._params:
            p._t.detach().copy_(self._backup[id(p)])
        self._backup = None

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        self.step()

from ..optimizer import LBFGS  # noqa: F401,E402  (reference keeps an incubate alias)


import sys as _sys  # noqa: E402
from . import optimizer_functional as functional  # noqa: E402
_sys.modules[__name__ + ".functional"] = functional
__path__ = []  # submodules above are importable by dotted name
