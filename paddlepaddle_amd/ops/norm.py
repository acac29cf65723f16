"""RMSNorm / LayerNorm with HIP forward+backward kernels.

Reference: paddle/phi/kernels/gpu/rms_norm_kernel.cu, layer_norm_kernel.cu,
python/paddle/incubate/nn/functional/fused_rms_norm.py.
Kernels: csrc/kernels/norm.hip — one 64-lane wave per row for hidden ≤ 8192 (vectorised
16-byte loads, fp32 statistics kept in registers), block-per-row above that.
"""
from __future__ import annotations

import torch

from . import _loader as L
from ..framework.trace_hook import static_op


def _finalize_parts(pa, pb, dta, dtb, nparts, cols, params=(None, None)):
    """Sum the [nparts, cols] fp32 partials of the weight (and bias) gradient into the parameters' dtypes:
    one HIP launch for both instead of a reduction + a cast each. A parameter whose gradient buffer is
    registered for in-place accumulation (ops.linear.register_main_grad) gets the sum added straight into
    that buffer (no separate autograd accumulation pass); None is returned for it."""
    if pa is None and pb is None:  # a norm without affine weight and bias
        return None, None
    dev = (pa if pa is not None else pb).device
    if L.has("pa_reduce_parts") and all(d in L._DT for d in (dta, dtb) if d is not None):
        from .linear import _vector_main_grad
        mga = _vector_main_grad(params[0], dta) if pa is not None else None
        mgb = _vector_main_grad(params[1], dtb) if pb is not None else None
        oa = (mga[0] if mga else torch.empty(cols, dtype=dta, device=dev)) if pa is not None else None
        ob = (mgb[0] if mgb else torch.empty(cols, dtype=dtb, device=dev)) if pb is not None else None
        L.call("pa_reduce_parts", L.ptr(pa), L.ptr(pb), L.ptr(oa), L.ptr(ob), nparts, cols,
               (L._DT[dta] | (bool(mga) << 8)) if dta is not None else 0,
               (L._DT[dtb] | (bool(mgb) << 8)) if dtb is not None else 0, L.stream_ptr())
        for mg, prm in ((mga, params[0]), (mgb, params[1])):
            if mg:
                mg[1](prm)
        return (None if mga else oa), (None if mgb else ob)
    return (pa.sum(0).to(dta) if pa is not None else None), (pb.sum(0).to(dtb) if pb is not None else None)


def _acc(t):
    """Accumulation dtype of the reference paths: fp32 for 16-bit inputs, the input's own dtype otherwise (a
    float64 norm stays float64)."""
    return t.float() if t.dtype in (torch.float16, torch.bfloat16) else t


def _rms_ref(x, w, eps):
    xf = _acc(x)
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    y = xf * r
    if w is not None:
        y = y * w.to(y.dtype)
    return y.to(x.dtype)


def _ln_ref(x, w, b, eps):
    xf = _acc(x)
    return torch.nn.functional.layer_norm(xf, (x.shape[-1],), None if w is None else w.to(xf.dtype),
                                          None if b is None else b.to(xf.dtype), eps).to(x.dtype)


class _RMSNormHIP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        cols = x.shape[-1]
        x2 = x.contiguous().view(-1, cols)
        rows = x2.shape[0]
        y = torch.empty_like(x2)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        wc = w.contiguous() if w is not None else None
        if wc is not None and wc.dtype != x.dtype:
            wc = wc.to(x.dtype)
        L.call("pa_rms_norm_fwd", L.ptr(x2), L.ptr(wc), L.ptr(y), L.ptr(rstd), rows, cols, float(eps),
               L.dcode(x2), L.stream_ptr())
        ctx.save_for_backward(x2, wc, rstd)
        ctx.w_dtype = None if w is None else w.dtype
        ctx.params = (w, None)
        ctx.shape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, wc, rstd = ctx.saved_tensors
        rows, cols = x2.shape
        dy2 = dy.contiguous().view(rows, cols)
        if dy2.dtype != x2.dtype:
            dy2 = dy2.to(x2.dtype)
        dx = torch.empty_like(x2)
        nparts = min(max((rows + 15) // 16, 1), 512)  # >= ~3 workgroups per CU in the weight-gradient pass
        dw_part = torch.empty(nparts, cols, dtype=torch.float32, device=x2.device) if wc is not None else None
        L.call("pa_rms_norm_bwd", L.ptr(dy2), L.ptr(x2), L.ptr(wc), L.ptr(rstd), L.ptr(dx), L.ptr(dw_part),
               rows, cols, L.dcode(x2) | (nparts << 8), L.stream_ptr())
        dw, _ = _finalize_parts(dw_part, None, ctx.w_dtype, None, nparts, cols, ctx.params) if wc is not None \
            else (None, None)
        return dx.view(ctx.shape), dw, None


class _LayerNormHIP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        cols = x.shape[-1]
        x2 = x.contiguous().view(-1, cols)
        rows = x2.shape[0]
        y = torch.empty_like(x2)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        wc = w.contiguous().to(x.dtype) if w is not None else None
        bc = b.contiguous().to(x.dtype) if b is not None else None
        L.call("pa_layer_norm_fwd", L.ptr(x2), L.ptr(wc), L.ptr(bc), L.ptr(y), L.ptr(mean), L.ptr(rstd),
               rows, cols, float(eps), L.dcode(x2), L.stream_ptr())
        ctx.save_for_backward(x2, wc, mean, rstd)
        ctx.has_b = b is not None
        ctx.w_dtype = None if w is None else w.dtype
        ctx.b_dtype = None if b is None else b.dtype
        ctx.params = (w, b)
        ctx.shape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, wc, mean, rstd = ctx.saved_tensors
        rows, cols = x2.shape
        dy2 = dy.contiguous().view(rows, cols).to(x2.dtype)
        dx = torch.empty_like(x2)
        nparts = min(max((rows + 15) // 16, 1), 512)  # >= ~3 workgroups per CU in the weight-gradient pass
        dw_part = torch.empty(nparts, cols, dtype=torch.float32, device=x2.device)
        db_part = torch.empty(nparts, cols, dtype=torch.float32, device=x2.device)
        L.call("pa_layer_norm_bwd", L.ptr(dy2), L.ptr(x2), L.ptr(wc), L.ptr(mean), L.ptr(rstd), L.ptr(dx),
               L.ptr(dw_part), L.ptr(db_part), L.ptr(None), rows, cols, L.dcode(x2) | (nparts << 8), L.stream_ptr())
        dw, db = _finalize_parts(dw_part if wc is not None else None, db_part if ctx.has_b else None, ctx.w_dtype,
                                 ctx.b_dtype, nparts, cols, getattr(ctx, "params", (None, None)))
        return dx.view(ctx.shape), dw, db, None


@static_op
def rms_norm(x, w, eps=1e-6):
    if L.hip_enabled_for(x) and x.dtype in L._DT and x.shape[-1] % 8 == 0:
        return _RMSNormHIP.apply(x, w, eps)
    return _rms_ref(x, w, eps)


class _LayerNormResidualHIP(torch.autograd.Function):
    """(x, layer_norm(x)) where the first output is the residual branch's use of x: its gradient is added into
    dx inside the LN backward kernel (pa_layer_norm_bwd `res`), replacing the separate residual-gradient add
    of a pre-LN transformer block (x feeds both the LN and the residual)."""

    @staticmethod
    def forward(ctx, x, w, b, eps):
        y = _LayerNormHIP.forward(ctx, x, w, b, eps)
        return x.view_as(x), y

    @staticmethod
    def backward(ctx, g_res, dy):
        x2, wc, mean, rstd = ctx.saved_tensors
        rows, cols = x2.shape
        res = None if g_res is None else g_res.contiguous().view(rows, cols).to(x2.dtype)
        if dy is None:
            return (None if res is None else res.view(ctx.shape)), None, None, None
        dy2 = dy.contiguous().view(rows, cols).to(x2.dtype)
        dx = torch.empty_like(x2)
        nparts = min(max((rows + 15) // 16, 1), 512)
        dw_part = torch.empty(nparts, cols, dtype=torch.float32, device=x2.device)
        db_part = torch.empty(nparts, cols, dtype=torch.float32, device=x2.device)
        L.call("pa_layer_norm_bwd", L.ptr(dy2), L.ptr(x2), L.ptr(wc), L.ptr(mean), L.ptr(rstd), L.ptr(dx),
               L.ptr(dw_part), L.ptr(db_part), L.ptr(res), rows, cols, L.dcode(x2) | (nparts << 8), L.stream_ptr())
        dw, db = _finalize_parts(dw_part if wc is not None else None, db_part if ctx.has_b else None, ctx.w_dtype,
                                 ctx.b_dtype, nparts, cols, getattr(ctx, "params", (None, None)))
        return dx.view(ctx.shape), dw, db, None


class _RMSNormResidualHIP(torch.autograd.Function):
    """(x, rms_norm(x)) with the residual branch's gradient summed into dx by the RMSNorm backward kernel
    (pa_rms_norm_bwd_res), the RMSNorm twin of _LayerNormResidualHIP for pre-norm LLaMA blocks."""

    @staticmethod
    def forward(ctx, x, w, eps):
        y = _RMSNormHIP.forward(ctx, x, w, eps)
        return x.view_as(x), y

    @staticmethod
    def backward(ctx, g_res, dy):
        x2, wc, rstd = ctx.saved_tensors
        rows, cols = x2.shape
        res = None if g_res is None else g_res.contiguous().view(rows, cols).to(x2.dtype)
        if dy is None:
            return (None if res is None else res.view(ctx.shape)), None, None
        dy2 = dy.contiguous().view(rows, cols).to(x2.dtype)
        dx = torch.empty_like(x2)
        nparts = min(max((rows + 15) // 16, 1), 512)
        dw_part = torch.empty(nparts, cols, dtype=torch.float32, device=x2.device) if wc is not None else None
        L.call("pa_rms_norm_bwd_res", L.ptr(dy2), L.ptr(x2), L.ptr(wc), L.ptr(rstd), L.ptr(dx), L.ptr(dw_part),
               L.ptr(res), rows, cols, L.dcode(x2) | (nparts << 8), L.stream_ptr())
        dw, _ = _finalize_parts(dw_part, None, ctx.w_dtype, None, nparts, cols, ctx.params) if wc is not None \
            else (None, None)
        return dx.view(ctx.shape), dw, None


@static_op
def rms_norm_residual(x, w, eps=1e-6):
    """(x_residual, rms_norm(x)): on the HIP path the residual branch's gradient is summed into the norm's input
    gradient inside the backward kernel (no separate add)."""
    if (L.hip_enabled_for(x) and x.dtype in L._DT and x.shape[-1] % 8 == 0 and torch.is_grad_enabled()
            and L.has("pa_rms_norm_bwd_res")):
        return _RMSNormResidualHIP.apply(x, w, eps)
    return x, rms_norm(x, w, eps)


def layer_norm_residual(x, w, b, eps=1e-5):
    """(x_residual, layer_norm(x)): use x_residual for the block's residual connection; on the HIP path its
    gradient is summed into the LN input gradient by the LN backward kernel (no separate add)."""
    if L.hip_enabled_for(x) and x.dtype in L._DT and x.shape[-1] % 8 == 0 and torch.is_grad_enabled():
        return _LayerNormResidualHIP.apply(x, w, b, eps)
    return x, layer_norm(x, w, b, eps)


@static_op
def layer_norm(x, w, b, eps=1e-5):
    if L.hip_enabled_for(x) and x.dtype in L._DT and x.shape[-1] % 8 == 0:
        return _LayerNormHIP.apply(x, w, b, eps)
    return _ln_ref(x, w, b, eps)


def add_rms_norm(x, r, w, eps=1e-6, inplace=False):
    """(s, y) with s = x + r and y = rms_norm(s) * w, in one HIP pass (inference: no autograd). With
    ``inplace`` the sum is written into ``x``. Reference: incubate.nn.functional.fused_rms_norm(residual=...)."""
    if (L.hip_enabled_for(x) and x.dtype in L._DT and x.shape[-1] % 8 == 0 and x.shape[-1] <= 8192
            and r.shape == x.shape and x.is_contiguous() and r.is_contiguous() and w.dtype == x.dtype
            and L.has("pa_add_rms_norm_fwd") and not (torch.is_grad_enabled() and
                                                      (x.requires_grad or r.requires_grad or w.requires_grad))):
        s = x if inplace else torch.empty_like(x)
        y = torch.empty_like(x)
        cols = x.shape[-1]
        L.call("pa_add_rms_norm_fwd", L.ptr(x), L.ptr(r), L.ptr(w), L.ptr(s), L.ptr(y), x.numel() // cols, cols,
               float(eps), L.dcode(x), L.stream_ptr())
        return s, y
    s = x + r
    return s, rms_norm(s, w, eps)
