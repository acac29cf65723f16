"""Dynamic loss scaling. Reference: python/paddle/amp/grad_scaler.py:62 AmpScaler, :657 GradScaler.
The found-inf check and the unscale are fused into the multi-tensor path: grads are checked with
one torch._amp_foreach_non_finite_check_and_unscale_ launch (device-side found_inf flag, no host
sync until update())."""
from __future__ import annotations

from enum import Enum

import torch

from ..framework.tensor import Tensor, _wrap


class OptimizerState(Enum):
    INIT = 0
    UNSCALED = 1
    STEPPED = 2


class AmpScaler:
    def __init__(self, enable=True, init_loss_scaling=2.0 ** 15, incr_ratio=2.0, decr_ratio=0.5,
                 incr_every_n_steps=1000, decr_every_n_nan_or_inf=1, use_dynamic_loss_scaling=True):
        self._enable = enable
        self._scale = float(init_loss_scaling) if enable else 1.0
        self._incr_ratio, self._decr_ratio = incr_ratio, decr_ratio
        self._incr_every_n_steps, self._decr_every_n_nan_or_inf = incr_every_n_steps, decr_every_n_nan_or_inf
        self._use_dynamic = use_dynamic_loss_scaling
        self._incr_count = 0
        self._decr_count = 0
        self._found_inf = None
        self._opt_states = {}
        self._scale_t = None

    def is_enable(self):
        return self._enable

    def is_use_dynamic_loss_scaling(self):
        return self._use_dynamic

    def get_init_loss_scaling(self):
        return self._scale

    def set_init_loss_scaling(self, v):
        self._scale = float(v)

    def scale(self, var):
        if not self._enable:
            return var
        return _wrap(var._t * self._scale)

    def unscale_(self, optimizer):
        if not self._enable:
            return
        st = self._opt_states.get(id(optimizer), OptimizerState.INIT)
        if st == OptimizerState.UNSCALED:
            return
        grads = [p._t.grad for p in optimizer._parameter_list if p._t.grad is not None]
        if not grads:
            self._found_inf = torch.zeros(1)
            return
        dev = grads[0].device
        found = torch.zeros(1, dtype=torch.float32, device=dev)
        inv = torch.full((1,), 1.0 / self._scale, dtype=torch.float32, device=dev)
        by_dtype = {}
        for g in grads:
            by_dtype.setdefault((g.device, g.dtype), []).append(g)
        for gs in by_dtype.values():
            torch._amp_foreach_non_finite_check_and_unscale_(gs, found, inv)
        self._found_inf = found
        self._opt_states[id(optimizer)] = OptimizerState.UNSCALED

    def minimize(self, optimizer, *args, **kwargs):
        self.step(optimizer)
        self.update()
        return None, None

    def step(self, optimizer):
        if not self._enable:
            optimizer.step()
            return
        self.unscale_(optimizer)
        if self._found_inf is not None and bool(self._found_inf.item()):
            self._opt_states[id(optimizer)] = OptimizerState.STEPPED
            self._skip = True
            return
        self._skip = False
        optimizer.step()
        self._opt_states[id(optimizer)] = OptimizerState.STEPPED

    def update(self):
        if not self._enable:
            return
        found = self._found_inf is not None and bool(self._found_inf.item())
        if self._use_dynamic:
            if found:
                self._incr_count = 0
                self._decr_count += 1
                if self._decr_count >= self._decr_every_n_nan_or_inf:
                    self._scale = max(self._scale * self._decr_ratio, 1.0)
                    self._decr_count = 0
            else:
                self._decr_count = 0
                self._incr_count += 1
                if self._incr_count >= self._incr_every_n_steps:
                    self._scale *= self._incr_ratio
                    self._incr_count = 0
        self._opt_states = {}
        self._found_inf = None

    def state_dict(self):
        return {"scale": self._scale, "incr_ratio": self._incr_ratio, "decr_ratio": self._decr_ratio,
                "incr_every_n_steps": self._incr_every_n_steps,
                "decr_every_n_nan_or_inf": self._decr_every_n_nan_or_inf, "incr_count": self._incr_count,
                "decr_count": self._decr_count, "use_dynamic_loss_scaling": self._use_dynamic}

    def load_state_dict(self, sd):
        self._scale = float(sd["scale"])
        self._incr_count = sd.get("incr_count", 0)
        self._decr_count = sd.get("decr_count", 0)

    set_state_dict = load_state_dict


class GradScaler(AmpScaler):
    def __init__(self, enable=True, init_loss_scaling=65536.0, incr_ratio=2.0, decr_ratio=0.5,
                 incr_every_n_steps=2000, decr_every_n_nan_or_inf=1, use_dynamic_loss_scaling=True):
        super().__init__(enable, init_loss_scaling, incr_ratio, decr_ratio, incr_every_n_steps,
                         decr_every_n_nan_or_inf, use_dynamic_loss_scaling)

    def get_loss_scaling(self):
        return self._scale
