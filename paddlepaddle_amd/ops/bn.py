"""Channels-last batch norm with fused activation / residual add (csrc/kernels/bn.hip).

Reference: paddle/phi/kernels/gpu/batch_norm_kernel.cu (+ _grad) and the fused_bn_add_activation op
(python/paddle/incubate/layers/nn.py:1092 ``fused_bn_add_act``). Semantics follow the reference:
training uses the biased batch variance both for normalisation and for the running average
``running = momentum * running + (1 - momentum) * batch``.

The HIP path takes a bf16 [..., C] tensor that is contiguous in channels-last order (NHWC storage),
fp32 affine parameters and running statistics. Everything else runs the fp32 torch reference below.
"""
from __future__ import annotations

import torch

from . import _loader as L
from ..framework.trace_hook import static_op


def batch_norm_act_reference(x2, weight, bias, running_mean, running_var, training, momentum, eps, act=None,
                             residual=None):
    """fp32 math on a [R, C] view; updates running stats in place like the kernel."""
    xf = x2.float()
    if training:
        mean = xf.mean(0)
        var = xf.var(0, unbiased=False)
        if running_mean is not None:
            with torch.no_grad():
                running_mean.mul_(momentum).add_((1 - momentum) * mean.detach())
                running_var.mul_(momentum).add_((1 - momentum) * var.detach())
    else:
        mean, var = running_mean.float(), running_var.float()
    y = (xf - mean) * torch.rsqrt(var + eps)
    if weight is not None:
        y = y * weight.float()
    if bias is not None:
        y = y + bias.float()
    if residual is not None:
        y = y + residual.float()
    if act == "relu":
        y = torch.relu(y)
    elif act is not None:
        raise ValueError(f"unsupported fused activation {act}")
    return y.to(x2.dtype)


def _chunks(R, C):
    return int(L.lib().pa_bn_chunks(R, C))


class _BNActHIP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2, weight, bias, residual, running_mean, running_var, training, momentum, eps, relu):
        R, C = x2.shape
        dev = x2.device
        y = torch.empty_like(x2)
        ss = torch.empty(2, C, dtype=torch.float32, device=dev)
        if training:
            mean = torch.empty(C, dtype=torch.float32, device=dev)
            rstd = torch.empty(C, dtype=torch.float32, device=dev)
            partial = torch.empty(2 * _chunks(R, C) * C, dtype=torch.float32, device=dev)
        else:
            mean = running_mean.float().contiguous()
            rstd = torch.rsqrt(running_var.float() + eps)
            w = weight.float() if weight is not None else torch.ones_like(mean)
            b = bias.float() if bias is not None else torch.zeros_like(mean)
            ss[0].copy_(w * rstd)
            ss[1].copy_(b - mean * w * rstd)
            partial = None
        L.call("pa_bn_fwd_nhwc", L.ptr(x2), L.ptr(residual), L.ptr(y), L.ptr(weight), L.ptr(bias),
               L.ptr(running_mean if training else None), L.ptr(running_var if training else None), L.ptr(mean),
               L.ptr(rstd), L.ptr(partial), L.ptr(ss), R, C, float(momentum), float(eps), int(relu), int(training),
               L.stream_ptr())
        # relu without residual: the backward recomputes the mask from x with scale / shift (ss) instead of
        # reading y; with a residual the mask needs y
        mask_x = bool(relu) and residual is None
        ctx.save_for_backward(x2, y if relu and not mask_x else None, weight, mean, rstd, ss if mask_x else None)
        ctx.flags = (bool(relu), bool(training), residual is not None, weight is not None, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, y, weight, mean, rstd, ss = ctx.saved_tensors
        relu, training, has_res, has_w, has_b = ctx.flags
        R, C = x2.shape
        dev = x2.device
        dy = dy.contiguous()
        dx = torch.empty_like(x2)
        dres = torch.empty_like(x2) if has_res and ctx.needs_input_grad[3] else None
        dw = torch.empty(C, dtype=torch.float32, device=dev) if has_w else None
        db = torch.empty(C, dtype=torch.float32, device=dev) if has_b else None
        partial = torch.empty(2 * _chunks(R, C) * C, dtype=torch.float32, device=dev)
        coef = torch.empty(3, C, dtype=torch.float32, device=dev)
        L.call("pa_bn_bwd_nhwc", L.ptr(dy), L.ptr(x2), L.ptr(y), L.ptr(dx), L.ptr(dres), L.ptr(weight), L.ptr(mean),
               L.ptr(rstd), L.ptr(dw), L.ptr(db), L.ptr(partial), L.ptr(coef), R, C, int(relu), int(not training),
               L.ptr(ss), L.stream_ptr())
        if dw is not None and dw.dtype != weight.dtype:
            dw = dw.to(weight.dtype)
        return dx, dw, db, dres, None, None, None, None, None, None


def _hip_ok(x, weight, bias, residual, running_mean, running_var):
    if not L.hip_enabled_for(x) or not L.has("pa_bn_fwd_nhwc"):
        return False
    if x.dtype != torch.bfloat16 or x.dim() < 2:
        return False
    C = x.shape[-1]
    if C % 8 != 0 or not x.is_contiguous():
        return False
    for t in (weight, bias, running_mean, running_var):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != C):
            return False
    if running_mean is None or running_var is None:
        return False
    if residual is not None and (residual.shape != x.shape or residual.dtype != x.dtype or
                                 not residual.is_contiguous()):
        return False
    return True


@static_op
def batch_norm_act_nhwc(x, weight, bias, running_mean, running_var, training=True, momentum=0.9, eps=1e-5,
                        act=None, residual=None):
    """y = act(batch_norm(x) [+ residual]) over the last (channel) dim of a channels-last tensor."""
    if act not in (None, "relu"):
        raise ValueError(f"unsupported fused activation {act}")
    C = x.shape[-1]
    if _hip_ok(x, weight, bias, residual, running_mean, running_var):
        x2 = x.view(-1, C)
        r2 = residual.view(-1, C) if residual is not None else None
        y = _BNActHIP.apply(x2, weight, bias, r2, running_mean, running_var, bool(training), float(momentum),
                            float(eps), act == "relu")
        return y.view(x.shape)
    x2 = x.reshape(-1, C)
    r2 = residual.reshape(-1, C) if residual is not None else None
    return batch_norm_act_reference(x2, weight, bias, running_mean, running_var, training, momentum, eps, act,
                                    r2).view(x.shape)
