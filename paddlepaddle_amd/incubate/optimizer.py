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

from ..optimizer.others import Lamb as _Lamb, _PerParam  # noqa: E402


class LarsMomentumOptimizer(_PerParam):
    """Momentum with layer-wise adaptive rate scaling. Reference: incubate/optimizer/lars_momentum.py:25 and
    paddle/phi/kernels/gpu/lars_momentum_kernel.cu:233 —
    local_lr = lr * lars_coeff * ||p|| / (lars_weight_decay * ||p|| + ||g|| + epsilon) (lr when a norm is 0),
    v = mu * v + local_lr * (g * rescale_grad + lars_weight_decay * p), p -= v. Parameters whose name contains
    an entry of exclude_from_weight_decay use lars_weight_decay = 0."""
    _acc_names = ("velocity",)

    def __init__(self, learning_rate, momentum, lars_coeff=0.001, lars_weight_decay=0.0005, parameter_list=None,
                 regularization=None, grad_clip=None, name=None, exclude_from_weight_decay=None, epsilon=0,
                 multi_precision=False, rescale_grad=1.0):
        super().__init__(learning_rate, parameter_list, regularization, grad_clip, name, multi_precision)
        self._momentum, self._lars_coeff = float(momentum), float(lars_coeff)
        self._lars_weight_decay, self._epsilon = float(lars_weight_decay), float(epsilon)
        self._exclude = list(exclude_from_weight_decay or [])
        self._rescale = float(rescale_grad)

    def _update_param(self, group, p):
        master = self._master(p)
        w = master if master is not None else p._t.detach()
        g = p._t.grad.to(w.dtype) * self._rescale
        g = self._regularized_grad(p, g, group)
        lr = self._group_lr(group, p)
        wd = 0.0 if any(n in (getattr(p, "name", "") or "") for n in self._exclude) else self._lars_weight_decay
        pn, gn = w.norm(), g.norm()
        local = torch.where((pn > 0) & (gn > 0),
                            lr * self._lars_coeff * pn / (wd * pn + gn + self._epsilon),
                            torch.full_like(pn, lr))
        v = self._acc("velocity", p, dtype=w.dtype)
        v.mul_(self._momentum).add_(local * (g + wd * w))
        w.sub_(v)
        self._fin(p, master)


class GradientMergeOptimizer:
    """Gradient merge (accumulation) around an inner optimizer. Reference: incubate/optimizer/gradient_merge.py:30
    (static-graph pass: the inner update runs every k_steps on the summed, optionally averaged gradients).
    Here it works in both modes: ``step()`` counts micro-steps and applies the inner optimizer on every k-th with
    the accumulated gradients (divided by k when avg), ``clear_grad()`` only clears after an applied step."""

    def __init__(self, inner_optimizer, k_steps=1, avg=True):
        if k_steps < 1:
            raise ValueError("k_steps must be >= 1")
        self.inner_optimizer = inner_optimizer
        self.k_steps, self.avg = int(k_steps), bool(avg)
        self._micro = 0
        self.type = "gradient_merge"

    def __getattr__(self, name):
        return getattr(self.inner_optimizer, name)

    @no_grad()
    def step(self):
        self._micro += 1
        if self._micro % self.k_steps:
            return
        if self.avg and self.k_steps > 1:
            for p in self.inner_optimizer._parameter_list:
                if p._t.grad is not None:
                    p._t.grad.mul_(1.0 / self.k_steps)
        self.inner_optimizer.step()

    def clear_grad(self, set_to_zero=True):
        if self._micro % self.k_steps == 0:
            self.inner_optimizer.clear_grad(set_to_zero)

    clear_gradients = clear_grad

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        from ..static import _static_mode
        if _static_mode.enabled:
            from ..static import default_main_program
            default_main_program()._set_optimizer(self, loss)
            return None, None
        loss.backward()
        self.step()
        self.clear_grad()
        return None, None


class _Wrapper:
    def __init__(self, optimizer):
        self._optimizer = optimizer
        self.inner_opt = optimizer

    def __getattr__(self, name):
        return getattr(self._optimizer, name)

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        return self._optimizer.minimize(loss, startup_program, parameters, no_grad_set)


class RecomputeOptimizer(_Wrapper):
    """Reference: incubate/optimizer/recompute.py:24 (static-graph activation recompute around checkpoint
    variables). Activation recompute in this framework is applied to layers (paddle.distributed.fleet.recompute,
    fleet strategy ``recompute``); this wrapper records the checkpoints and delegates the update."""

    def __init__(self, optimizer):
        super().__init__(optimizer)
        self._checkpoints = None

    def _set_checkpoints(self, checkpoints):
        self._checkpoints = list(checkpoints)

    def backward(self, loss, startup_program=None, parameter_list=None, no_grad_set=None, callbacks=None):
        return self._optimizer.backward(loss, startup_program, parameter_list, no_grad_set, callbacks)

    def apply_optimize(self, loss, startup_program, params_grads):
        return self._optimizer.apply_gradients(params_grads)


class PipelineOptimizer(_Wrapper):
    """Reference: incubate/optimizer/pipeline.py:34 (static-graph pipeline over device_guard sections). Pipeline
    training here runs through fleet's PipelineParallel (1F1B / VPP / FThenB / ZBH1) with ``num_microbatches``
    as accumulate_steps; this wrapper carries that setting and delegates the update."""

    def __init__(self, optimizer, num_microbatches=1, start_cpu_core_id=0):
        super().__init__(optimizer)
        if num_microbatches < 1:
            raise ValueError("num_microbatches must be >= 1")
        self._num_microbatches = int(num_microbatches)
        self._start_cpu_core_id = int(start_cpu_core_id)


class DistributedFusedLamb(_Lamb):
    """LAMB over data-parallel ranks. Reference: incubate/optimizer/distributed_fused_lamb.py:115 (a static-graph op
    that all-reduces the flattened gradients, clips by the global norm, and applies LAMB). Here: the gradients are
    flattened per dtype into one buffer and all-reduced over the default group (averaged unless
    is_grad_scaled_by_nranks), clipped by the global norm before or after the all-reduce (clip_after_allreduce),
    and every gradient_accumulation_steps-th step applies the LAMB update."""

    def __init__(self, learning_rate=0.001, lamb_weight_decay=0.01, beta1=0.9, beta2=0.999, epsilon=1e-6,
                 parameters=None, grad_clip=None, exclude_from_weight_decay_fn=None, clip_after_allreduce=True,
                 is_grad_scaled_by_nranks=True, alignment=128, use_master_param_norm=True,
                 gradient_accumulation_steps=1, use_master_acc_grad=True, nproc_per_node=None,
                 use_hierarchical_allreduce=False, name=None):
        from ..nn import ClipGradByGlobalNorm
        if grad_clip is not None and not isinstance(grad_clip, ClipGradByGlobalNorm):
            raise TypeError("Only ClipGradByGlobalNorm is supported in DistributedFusedLamb")
        super().__init__(learning_rate, lamb_weight_decay, beta1, beta2, epsilon, parameters, None,
                         exclude_from_weight_decay_fn, True, False, name)
        self._dfl_clip = grad_clip
        self._clip_after_allreduce = clip_after_allreduce
        self._is_grad_scaled_by_nranks = is_grad_scaled_by_nranks
        self._gradient_accumulation_steps = int(gradient_accumulation_steps)
        if self._gradient_accumulation_steps < 1:
            raise ValueError("gradient_accumulation_steps must be >= 1")
        self._acc_micro = 0

    def _allreduce(self, params):
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() < 2:
            return
        by_dt = {}
        for p in params:
            by_dt.setdefault(p._t.grad.dtype, []).append(p._t.grad)
        n = dist.get_world_size()
        for grads in by_dt.values():
            flat = torch.cat([g.reshape(-1) for g in grads])
            dist.all_reduce(flat)
            if not self._is_grad_scaled_by_nranks:
                flat.mul_(1.0 / n)
            off = 0
            for g in grads:
                g.copy_(flat[off:off + g.numel()].view_as(g))
                off += g.numel()

    @no_grad()
    def step(self):
        self._acc_micro += 1
        if self._acc_micro % self._gradient_accumulation_steps:
            return
        params = [p for p in self._parameter_list if p._t.grad is not None]
        if self._dfl_clip is not None and not self._clip_after_allreduce:
            self._dfl_clip._clip_inplace(params)
        self._allreduce(params)
        if self._dfl_clip is not None and self._clip_after_allreduce:
            self._dfl_clip._clip_inplace(params)
        super().step()

    def clear_grad(self, set_to_zero=True):
        if self._acc_micro % self._gradient_accumulation_steps == 0:
            super().clear_grad(set_to_zero)


from ..optimizer import LBFGS  # noqa: F401,E402  (reference keeps an incubate alias)


import sys as _sys  # noqa: E402
from . import optimizer_functional as functional  # noqa: E402
_sys.modules[__name__ + ".functional"] = functional
__path__ = []  # submodules above are importable by dotted name
