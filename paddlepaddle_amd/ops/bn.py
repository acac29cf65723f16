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
from . import _conv_bn as _CB
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
    def forward(ctx, x2, weight, bias, residual, running_mean, running_var, training, momentum, eps, relu,
                sink=None, pre=None):
        ctx.sink = sink
        R, C = x2.shape
        dev = x2.device
        y = torch.empty_like(x2)
        ss = torch.empty(2, C, dtype=torch.float32, device=dev)
        if training:
            mean = torch.empty(C, dtype=torch.float32, device=dev)
            rstd = torch.empty(C, dtype=torch.float32, device=dev)
            partial = torch.empty(2 * _chunks(R, C) * C, dtype=torch.float32, device=dev) if pre is None else None
        else:
            mean = running_mean.float().contiguous()
            rstd = torch.rsqrt(running_var.float() + eps)
            w = weight.float() if weight is not None else torch.ones_like(mean)
            b = bias.float() if bias is not None else torch.zeros_like(mean)
            ss[0].copy_(w * rstd)
            ss[1].copy_(b - mean * w * rstd)
            partial = None
        # relu without residual: the backward recomputes the mask from x with scale / shift (ss) instead of
        # reading y; relu with a residual: the forward writes a bit mask of the relu (R * C / 8 bytes) that the
        # backward reads instead of y
        mask_x = bool(relu) and residual is None
        mbits = None
        if training and pre is not None:
            # conv -> BN fusion: the producing convolution wrote the partial sums (ops/_conv_bn.py)
            stats, chunks = pre
            if relu and residual is not None:
                mbits = torch.empty(R * C // 8, dtype=torch.uint8, device=dev)
            nws = int(L.lib().pa_bn_pre_ws(chunks, C))
            ws = torch.empty(nws, dtype=torch.float32, device=dev) if nws else None
            L.call("pa_bn_fwd_nhwc_pre", L.ptr(x2), L.ptr(residual), L.ptr(y), L.ptr(weight), L.ptr(bias),
                   L.ptr(running_mean), L.ptr(running_var), L.ptr(mean), L.ptr(rstd), L.ptr(stats), chunks, L.ptr(ws),
                   L.ptr(ss), L.ptr(mbits), R, C, float(momentum), float(eps), int(bool(relu)), L.stream_ptr())
        elif relu and residual is not None and L.has("pa_bn_fwd_nhwc_mask"):
            mbits = torch.empty(R * C // 8, dtype=torch.uint8, device=dev)
            L.call("pa_bn_fwd_nhwc_mask", L.ptr(x2), L.ptr(residual), L.ptr(y), L.ptr(weight), L.ptr(bias),
                   L.ptr(running_mean if training else None), L.ptr(running_var if training else None), L.ptr(mean),
                   L.ptr(rstd), L.ptr(partial), L.ptr(ss), L.ptr(mbits), R, C, float(momentum), float(eps),
                   int(training), L.stream_ptr())
        else:
            L.call("pa_bn_fwd_nhwc", L.ptr(x2), L.ptr(residual), L.ptr(y), L.ptr(weight), L.ptr(bias),
                   L.ptr(running_mean if training else None), L.ptr(running_var if training else None), L.ptr(mean),
                   L.ptr(rstd), L.ptr(partial), L.ptr(ss), R, C, float(momentum), float(eps), int(relu),
                   int(training), L.stream_ptr())
        keep = mbits if mbits is not None else (y if relu and not mask_x else None)
        ctx.save_for_backward(x2, keep, weight, mean, rstd, ss if mask_x else None)
        if mask_x and training:
            _CB._PENDING_BN[0] = (x2, mean, ss)  # the consuming convolution may fuse this BN's backward reduction
        ctx.bitmask = mbits is not None
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
        sink = ctx.sink
        to_sink = sink is not None and has_res
        dres = torch.empty_like(x2) if has_res and (ctx.needs_input_grad[3] or to_sink) else None
        dw = torch.empty(C, dtype=torch.float32, device=dev) if has_w else None
        db = torch.empty(C, dtype=torch.float32, device=dev) if has_b else None
        partial = torch.empty(2 * _chunks(R, C) * C, dtype=torch.float32, device=dev)
        coef = torch.empty(3, C, dtype=torch.float32, device=dev)
        if ctx.bitmask:  # `y` holds the relu bit mask
            L.call("pa_bn_bwd_nhwc_mask", L.ptr(dy), L.ptr(x2), L.ptr(y), L.ptr(dx), L.ptr(dres), L.ptr(weight),
                   L.ptr(mean), L.ptr(rstd), L.ptr(dw), L.ptr(db), L.ptr(partial), L.ptr(coef), R, C,
                   int(not training), L.stream_ptr())
        else:
            pre = _CB.take_bwd(dy, x2) if (ss is not None and training and dres is None) else None
            if pre is not None:  # the data-gradient convolution wrote [sum dyp, sum dyp * (x - mean)]
                stats, chunks = pre
                nws = int(L.lib().pa_bn_pre_ws(chunks, C))
                ws = torch.empty(nws, dtype=torch.float32, device=dev) if nws else None
                L.call("pa_bn_bwd_nhwc_pre", L.ptr(dy), L.ptr(x2), L.ptr(dx), L.ptr(weight), L.ptr(mean), L.ptr(rstd),
                       L.ptr(dw), L.ptr(db), L.ptr(stats), chunks, L.ptr(ws), L.ptr(coef), R, C, 0, L.ptr(ss),
                       L.stream_ptr())
            else:
                L.call("pa_bn_bwd_nhwc", L.ptr(dy), L.ptr(x2), L.ptr(y), L.ptr(dx), L.ptr(dres), L.ptr(weight),
                       L.ptr(mean), L.ptr(rstd), L.ptr(dw), L.ptr(db), L.ptr(partial), L.ptr(coef), R, C, int(relu),
                       int(not training), L.ptr(ss), L.stream_ptr())
        if dw is not None and dw.dtype != weight.dtype:
            dw = dw.to(weight.dtype)
        if to_sink:  # the block's first conv adds it to its data gradient (ops/conv.py ResidualGradSink)
            sink.dres = dres
            dres = None
        return dx, dw, db, dres, None, None, None, None, None, None, None, None


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
                        act=None, residual=None, grad_sink=None):
    """y = act(batch_norm(x) [+ residual]) over the last (channel) dim of a channels-last tensor."""
    if act not in (None, "relu"):
        raise ValueError(f"unsupported fused activation {act}")
    C = x.shape[-1]
    if _hip_ok(x, weight, bias, residual, running_mean, running_var):
        x2 = x.view(-1, C)
        r2 = residual.view(-1, C) if residual is not None else None
        sink = grad_sink if (grad_sink is not None and grad_sink.armed and r2 is not None) else None
        if sink is not None:
            r2 = r2.detach()  # its gradient travels through the sink, not autograd
        pre = _CB.take(x) if training else None
        _CB._PENDING_BN[0] = None
        y = _BNActHIP.apply(x2, weight, bias, r2, running_mean, running_var, bool(training), float(momentum),
                            float(eps), act == "relu", sink, pre)
        src, _CB._PENDING_BN[0] = _CB._PENDING_BN[0], None
        if src is not None and torch.is_grad_enabled():
            _CB.tag_bn_output(y, src)
        return y.view(x.shape)
    x2 = x.reshape(-1, C)
    r2 = residual.reshape(-1, C) if residual is not None else None
    return batch_norm_act_reference(x2, weight, bias, running_mean, running_var, training, momentum, eps, act,
                                    r2).view(x.shape)


# ------------------------------------------------------------------ cross-rank (sync) batch norm
def _sync_hip_ok(x2, weight, bias):
    if not L.hip_enabled_for(x2) or not L.has("pa_bn_reduce_nhwc"):
        return False
    if x2.dtype != torch.bfloat16 or x2.shape[-1] % 8 != 0 or not x2.is_contiguous():
        return False
    return all(t is None or (t.dtype == torch.float32 and t.is_contiguous()) for t in (weight, bias))


def _channel_sums(mode, x2, dy=None, mean=None):
    """[2, C] fp32: mode 0 -> (sum x, sum x^2); mode 1 -> (sum dy, sum dy * (x - mean))."""
    R, C = x2.shape
    if _sync_hip_ok(x2, None, None) and (dy is None or (dy.dtype == x2.dtype and dy.is_contiguous())):
        sums = torch.empty(2, C, dtype=torch.float32, device=x2.device)
        partial = torch.empty(2 * _chunks(R, C) * C, dtype=torch.float32, device=x2.device)
        L.call("pa_bn_reduce_nhwc", int(mode), L.ptr(x2), L.ptr(dy), L.ptr(None), L.ptr(mean), L.ptr(None),
               L.ptr(partial), L.ptr(sums), R, C, 0, L.stream_ptr())
        return sums
    xf = x2.float()
    if mode == 0:
        return torch.stack([xf.sum(0), (xf * xf).sum(0)])
    gf = dy.float()
    return torch.stack([gf.sum(0), (gf * (xf - mean)).sum(0)])


class _SyncBN(torch.autograd.Function):
    """Batch statistics over every rank of ``group`` (reference: sync_batch_norm_kernel.cu +
    sync_batch_norm_utils.h:575). Forward all-reduces (sum x, sum x^2, count); backward all-reduces
    (sum dy, sum dy * (x - mean)) so dx carries the cross-rank terms. dweight / dbias stay local (the
    data-parallel gradient all-reduce sums them, as in the reference's KeBNBackwardScaleBias)."""

    @staticmethod
    def forward(ctx, x2, weight, bias, running_mean, running_var, momentum, eps, pg):
        import torch.distributed as dist
        R, C = x2.shape
        sums = _channel_sums(0, x2)
        buf = torch.cat([sums.reshape(-1), torch.full((1,), float(R), device=x2.device)])
        dist.all_reduce(buf, group=pg)
        N = buf[-1]
        mean = buf[:C] / N
        var = (buf[C:2 * C] / N - mean * mean).clamp_min(0.0)
        rstd = torch.rsqrt(var + eps)
        with torch.no_grad():
            if running_mean is not None:
                running_mean.mul_(momentum).add_((1 - momentum) * mean.to(running_mean.dtype))
                running_var.mul_(momentum).add_((1 - momentum) * var.to(running_var.dtype))
        w = weight.float() if weight is not None else torch.ones_like(mean)
        b = bias.float() if bias is not None else torch.zeros_like(mean)
        sc = w * rstd
        ss = torch.stack([sc, b - mean * sc]).contiguous()
        if _sync_hip_ok(x2, weight, bias):
            y = torch.empty_like(x2)
            L.call("pa_bn_fwd_nhwc", L.ptr(x2), L.ptr(None), L.ptr(y), L.ptr(None), L.ptr(None), L.ptr(None),
                   L.ptr(None), L.ptr(mean), L.ptr(rstd), L.ptr(None), L.ptr(ss), R, C, 0.0, float(eps), 0, 0,
                   L.stream_ptr())
        else:
            y = (x2.float() * ss[0] + ss[1]).to(x2.dtype)
        ctx.save_for_backward(x2, weight, mean, rstd)
        ctx.pg, ctx.N = pg, N
        ctx.has = (weight is not None, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        import torch.distributed as dist
        x2, weight, mean, rstd = ctx.saved_tensors
        has_w, has_b = ctx.has
        R, C = x2.shape
        dy = dy.contiguous()
        local = _channel_sums(1, x2, dy, mean)  # [sum dy, sum dy * (x - mean)] on this rank
        dw = (local[1] * rstd).to(weight.dtype) if has_w else None
        db = local[0].to(weight.dtype if has_w else torch.float32) if has_b else None
        glob = local.clone()
        dist.all_reduce(glob, group=ctx.pg)
        N = ctx.N
        a = (weight.float() if has_w else torch.ones_like(mean)) * rstd
        bc = a * rstd * rstd * glob[1] / N
        d0 = bc * mean - a * glob[0] / N
        coef = torch.stack([a, bc, d0]).contiguous()
        if _sync_hip_ok(x2, weight, None) and dy.dtype == x2.dtype:
            dx = torch.empty_like(x2)
            L.call("pa_bn_bwd_apply_nhwc", L.ptr(dy), L.ptr(x2), L.ptr(None), L.ptr(coef), L.ptr(dx), L.ptr(None),
                   R, C, 0, L.ptr(None), L.stream_ptr())
        else:
            dx = (coef[0] * dy.float() - coef[1] * x2.float() + coef[2]).to(x2.dtype)
        return dx, dw, db, None, None, None, None, None


def sync_batch_norm(x, weight, bias, running_mean, running_var, momentum=0.9, eps=1e-5, channel_last=True, pg=None):
    """Training-mode batch norm whose statistics span every rank of the process group ``pg``."""
    t = x if channel_last else x.movedim(1, -1)
    C = t.shape[-1]
    x2 = t.contiguous().view(-1, C)
    y = _SyncBN.apply(x2, weight, bias, running_mean, running_var, float(momentum), float(eps), pg).view(t.shape)
    return y if channel_last else y.movedim(-1, 1)
