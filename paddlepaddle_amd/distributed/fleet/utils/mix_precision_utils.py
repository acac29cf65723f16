"""fleet.utils.mix_precision_utils: pure 16-bit parameters with fp32 gradient accumulation ("main_grad").
Reference: python/paddle/distributed/fleet/utils/mix_precision_utils.py (MixPrecisionLayer :35,
MixPrecisionOptimizer :97, MixPrecisionScaler :244).

MixPrecisionLayer gives every parameter an fp32 ``main_grad``: each backward's 16-bit gradient is added into it in
fp32 (a post-accumulate hook, so micro-batch accumulation does not round in bf16 / fp16) and the 16-bit ``.grad``
is released. MixPrecisionOptimizer steps its inner optimizer on those fp32 gradients; MixPrecisionScaler unscales
them. fused_allreduce_gradients (hybrid_parallel_util) reduces ``main_grad`` where it exists.
"""
from __future__ import annotations

import torch

from ....framework.tensor import Tensor, _wrap
from ....nn.layer.layers import Layer
from .hybrid_parallel_util import obtain_optimizer_parameters_list


class MixPrecisionLayer(Layer):
    def __init__(self, layers, dtype="float16"):
        super().__init__()
        if dtype not in ("float16", "bfloat16"):
            raise ValueError(f"MixPrecisionLayer dtype must be float16 or bfloat16, got {dtype!r}")
        self._layers = layers
        self._dtype = dtype
        for p in self._layers.parameters():
            if not hasattr(p, "main_grad"):
                p.main_grad = None
                if p._t.requires_grad:
                    p._t.register_post_accumulate_grad_hook(self._update_main_grad_hook(p))

    @staticmethod
    def _update_main_grad_hook(param):
        def hook(t):
            g = t.grad
            if g is None:
                return
            with torch.no_grad():
                if param.main_grad is None:
                    param.main_grad = _wrap(g.detach().float().clone())
                else:
                    param.main_grad._t.add_(g.detach().float())
            t.grad = None
        return hook

    def forward(self, *inputs, **kwargs):
        return self._layers(*inputs, **kwargs)

    def state_dict(self, destination=None, include_sublayers=True, structured_name_prefix="", **kw):
        return self._layers.state_dict(destination=destination, include_sublayers=include_sublayers,
                                       structured_name_prefix=structured_name_prefix)

    def set_state_dict(self, state_dict, use_structured_name=True):
        return self._layers.set_state_dict(state_dict, use_structured_name=use_structured_name)


class MixPrecisionOptimizer:
    """Steps the inner optimizer with each parameter's fp32 ``main_grad`` as its gradient (parameters without a
    main gradient are skipped, as in the reference). The inner optimizer keeps its fp32 master weights
    (multi_precision); the gradient it reads is the fp32 sum rounded once to the parameter dtype."""

    def __init__(self, optimizer):
        self._inner_opt = optimizer
        self._parameter_list = obtain_optimizer_parameters_list(optimizer)

    @torch.no_grad()
    def step(self):
        used = []
        for p in self._parameter_list:
            if p.stop_gradient or getattr(p, "main_grad", None) is None:
                continue
            p._t.grad = p.main_grad._t.to(p._t.dtype)
            used.append(p)
        used_ids = {id(p) for p in used}
        skipped = [p for p in self._parameter_list if id(p) not in used_ids and p._t.grad is not None]
        saved = {id(p): p._t.grad for p in skipped}
        for p in skipped:  # main_grad is the only gradient of a wrapped parameter
            p._t.grad = None
        try:
            self._inner_opt.step()
        finally:
            for p in used:
                p._t.grad = None
            for p in skipped:
                p._t.grad = saved[id(p)]

    def clear_grad(self, set_to_zero=True):
        for p in self._parameter_list:
            if p.stop_gradient:
                continue
            if hasattr(p, "main_grad"):
                if p.main_grad is not None:
                    if set_to_zero:
                        p.main_grad._t.zero_()
                    else:
                        p.main_grad = None
                p._t.grad = None
            else:
                p.clear_gradient(set_to_zero)

    clear_gradients = clear_grad

    def __getattr__(self, item):
        return getattr(self._inner_opt, item)


def _unscale_main_grads(self, optimizer):
    """GradScaler.unscale_ on the fp32 main gradients (reference mix_precision_utils.unscale_method)."""
    from ....amp.grad_scaler import OptimizerState
    if not self._enable:
        return
    if self._opt_states.get(id(optimizer), OptimizerState.INIT) == OptimizerState.UNSCALED:
        return
    params = obtain_optimizer_parameters_list(getattr(optimizer, "_inner_opt", optimizer))
    grads = []
    for p in params:
        mg = getattr(p, "main_grad", None)
        if mg is not None:
            grads.append(mg._t)
        elif p._t.grad is not None:
            grads.append(p._t.grad)
    if not grads:
        self._found_inf = torch.zeros(1)
        return
    dev = grads[0].device
    found = torch.zeros(1, dtype=torch.float32, device=dev)
    inv = torch.full((1,), 1.0 / self._scale, dtype=torch.float32, device=dev)
    by = {}
    for g in grads:
        by.setdefault((g.device, g.dtype), []).append(g)
    for gs in by.values():
        torch._amp_foreach_non_finite_check_and_unscale_(gs, found, inv)
    self._found_inf = found
    self._opt_states[id(optimizer)] = OptimizerState.UNSCALED


class MixPrecisionScaler:
    """A GradScaler whose unscale step works on the fp32 ``main_grad``s (found_inf from them too)."""

    def __init__(self, scaler):
        import types
        self._inner_scaler = scaler
        scaler.unscale_ = types.MethodType(_unscale_main_grads, scaler)

    def __getattr__(self, item):
        return getattr(self._inner_scaler, item)


__all__ = ["MixPrecisionLayer", "MixPrecisionOptimizer", "MixPrecisionScaler"]
