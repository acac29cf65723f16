"""Gradient clipping. Reference: python/paddle/nn/clip.py (ClipGradByGlobalNorm etc.).
Global-norm uses one multi-tensor HIP sum-of-squares launch (ops.optim.global_sq_norm) and one
multi-tensor scale, so the clip costs two launches regardless of parameter count."""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor, _wrap
from ..ops.optim import global_sq_norm


class ClipGradBase:
    def __call__(self, params_grads):
        return self._dygraph_clip(params_grads)

    def _clip_inplace(self, params):
        """Clip .grad of params in place (fast path used by our optimizers)."""
        pg = [(p, p.grad) for p in params if p.grad is not None]
        out = self._dygraph_clip(pg)
        for (p, g), (_, ng) in zip(pg, out):
            if ng is not g:
                p._t.grad.copy_(ng._t)


class ClipGradByValue(ClipGradBase):
    def __init__(self, max, min=None):  # noqa: A002
        self.max = float(max)
        self.min = -self.max if min is None else float(min)

    def _dygraph_clip(self, params_grads):
        out = []
        for p, g in params_grads:
            if g is None or not getattr(p, "need_clip", True):
                out.append((p, g))
                continue
            out.append((p, _wrap(g._t.clamp(self.min, self.max))))
        return out


class ClipGradByNorm(ClipGradBase):
    def __init__(self, clip_norm):
        self.clip_norm = float(clip_norm)

    def _dygraph_clip(self, params_grads):
        out = []
        for p, g in params_grads:
            if g is None or not getattr(p, "need_clip", True):
                out.append((p, g))
                continue
            n = g._t.float().norm()
            s = torch.clamp(self.clip_norm / torch.clamp(n, min=1e-6), max=1.0)
            out.append((p, _wrap((g._t.float() * s).to(g._t.dtype))))
        return out


class ClipGradByGlobalNorm(ClipGradBase):
    def __init__(self, clip_norm, group_name="default_group", auto_skip_clip=False):
        self.clip_norm = float(clip_norm)
        self.group_name = group_name
        self._extra_sq_norm_fn = None  # hook for distributed (TP/sharding) reduction of the partial norm

    def _global_norm(self, grads):
        sq = global_sq_norm(grads)
        if self._extra_sq_norm_fn is not None:
            sq = self._extra_sq_norm_fn(sq)
        return torch.sqrt(sq)

    def _dygraph_clip(self, params_grads):
        grads = [g._t for p, g in params_grads if g is not None and getattr(p, "need_clip", True)]
        if not grads:
            return params_grads
        gn = self._global_norm(grads)
        scale = self.clip_norm / torch.clamp(gn, min=self.clip_norm)
        out = []
        for p, g in params_grads:
            if g is None or not getattr(p, "need_clip", True):
                out.append((p, g))
            else:
                out.append((p, _wrap((g._t * scale.to(g._t.dtype)))))
        return out

    def _coef(self, ps):
        """Device fp32 scalar clip_norm / max(global_norm, clip_norm) over the grads of ``ps``."""
        grads = [p._t.grad for p in ps]
        fn = getattr(self, "_param_sq_fn", None)
        gn = torch.sqrt(fn(ps)) if fn is not None else self._global_norm(grads)
        return (self.clip_norm / torch.clamp(gn.float(), min=self.clip_norm)).reshape(())

    def _clip_inplace(self, params):
        ps = [p for p in params if p._t.grad is not None and getattr(p, "need_clip", True)]
        grads = [p._t.grad for p in ps]
        if not grads:
            return
        torch._foreach_mul_(grads, self._coef(ps))


def clip_grad_norm_(parameters, max_norm, norm_type=2.0, error_if_nonfinite=False):
    if isinstance(parameters, Tensor):
        parameters = [parameters]
    grads = [p._t.grad for p in parameters if p._t.grad is not None]
    if not grads:
        return _wrap(torch.tensor(0.0))
    if norm_type == float("inf"):
        total = torch.stack([g.abs().max().float() for g in grads]).max()
    elif norm_type == 2.0:
        total = torch.sqrt(global_sq_norm(grads))
    else:
        total = torch.stack([g.float().norm(norm_type) for g in grads]).norm(norm_type)
    if error_if_nonfinite and not torch.isfinite(total):
        raise RuntimeError("non-finite gradient norm")
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    torch._foreach_mul_(grads, coef)
    return _wrap(total)


def clip_grad_value_(parameters, clip_value):
    if isinstance(parameters, Tensor):
        parameters = [parameters]
    for p in parameters:
        if p._t.grad is not None:
            p._t.grad.clamp_(-clip_value, clip_value)
