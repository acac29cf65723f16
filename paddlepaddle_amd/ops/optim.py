"""Multi-tensor optimizer kernels (HIP).

Reference: paddle/phi/kernels/gpu/fused_adam_kernel.cu (multi-tensor Adam/AdamW with master
weights), adamw_kernel.cu.
Kernel: csrc/kernels/adamw.hip — one launch updates every tensor of a parameter group:
a device-side table of {param_fp32, grad, m, v, param_lowp, numel} entries, workgroups walk
fixed 64 KiB chunks (persistent-style work list computed on the host once and cached), fp32
math, optional bf16/fp16 shadow copy written in the same pass, grads unscaled by 1/loss_scale.
"""
from __future__ import annotations

import ctypes

import torch

from . import _loader as L

_CHUNK = 16384  # elements per work item


def device_table(rows, dev):
    """int64 pointer / work-item table on ``dev`` (and the host buffer it came from). Eager: a pinned
    non-blocking copy. Inside a hipGraph capture (a captured optimizer step) the values are written by kernels
    that carry them as launch arguments (pa_write_i64), so the graph holds no reference to host memory."""
    host = torch.tensor(rows, dtype=torch.int64)
    if dev.type == "cuda":
        if torch.cuda.is_current_stream_capturing() and L.has("pa_write_i64"):
            out = torch.empty(host.shape, dtype=torch.int64, device=dev)
            L.call("pa_write_i64", L.ptr(out), ctypes.c_void_p(host.data_ptr()), host.numel(), L.stream_ptr())
            return out, host
        host = host.pin_memory()
    return host.to(dev, non_blocking=True), host


class AdamWTable:
    """Device-resident pointer table for one parameter group (rebuilt when buffers change)."""

    def __init__(self, params, grads, ms, vs, lowps):
        self.key = tuple(t.data_ptr() for t in params) + tuple(g.data_ptr() for g in grads)
        rows = []
        items = []
        for i, (p, g, m, v, lp) in enumerate(zip(params, grads, ms, vs, lowps)):
            n = p.numel()
            gdt = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}[g.dtype]
            ldt = 3 if lp is None else {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}[lp.dtype]
            rows.append([p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(),
                         0 if lp is None else lp.data_ptr(), n, gdt | (ldt << 8)])
            for s in range(0, n, _CHUNK):
                items.append([i, s])
        dev = params[0].device
        self.table = torch.tensor(rows, dtype=torch.int64).to(dev)
        self.items = torch.tensor(items, dtype=torch.int64).to(dev)
        self.n_items = len(items)


def adamw_step_hip(table, lr, beta1, beta2, eps, weight_decay, bc1, bc2, grad_scale_inv_ptr=None):
    L.call("pa_adamw_multi", L.ptr(table.table), L.ptr(table.items), table.n_items,
           ctypes.c_void_p(0) if grad_scale_inv_ptr is None else L.ptr(grad_scale_inv_ptr),
           float(lr), float(beta1), float(beta2), float(eps), float(weight_decay), float(bc1), float(bc2),
           ctypes.c_void_p(0), L.stream_ptr())


def adamw_step_ref(params, grads, ms, vs, lowps, lr, beta1, beta2, eps, weight_decay, bc1, bc2, inv_scale=1.0):
    for p, g, m, v, lp in zip(params, grads, ms, vs, lowps):
        gf = g.float()
        if inv_scale != 1.0:
            gf = gf * inv_scale
        if weight_decay:
            p.mul_(1 - lr * weight_decay)
        m.mul_(beta1).add_(gf, alpha=1 - beta1)
        v.mul_(beta2).addcmul_(gf, gf, value=1 - beta2)
        denom = (v / bc2).sqrt_().add_(eps)
        p.addcdiv_(m, denom, value=-lr / bc1)
        if lp is not None:
            lp.copy_(p)


_SQ_CACHE = {}


def global_sq_norm(tensors):
    """Sum of squares over a list of tensors (fp32 0-d tensor): one multi-tensor HIP launch."""
    if not tensors:
        return None
    t0 = tensors[0]
    if L.hip_enabled_for(t0) and L.has("pa_sq_norm_multi") and all(t.is_contiguous() for t in tensors):
        key = tuple(t.data_ptr() for t in tensors)
        ent = _SQ_CACHE.get(key)
        if ent is None:
            rows, items = [], []
            for i, t in enumerate(tensors):
                rows.append([t.data_ptr(), t.numel(), L._DT[t.dtype]])
                for s in range(0, t.numel(), _CHUNK):
                    items.append([i, s])
            ent = (torch.tensor(rows, dtype=torch.int64).to(t0.device), torch.tensor(items, dtype=torch.int64).to(t0.device),
                   len(items), torch.empty(1024, dtype=torch.float32, device=t0.device))
            if len(_SQ_CACHE) > 64:
                _SQ_CACHE.clear()
            _SQ_CACHE[key] = ent
        table, items, n, partial = ent
        L.call("pa_sq_norm_multi", L.ptr(table), L.ptr(items), n, L.ptr(partial), L.stream_ptr())
        return partial.sum()
    return torch.stack([t.float().pow(2).sum() for t in tensors]).sum()
