"""Elementwise math, reductions and products. Reference: python/paddle/tensor/math.py,
python/paddle/tensor/linalg.py (matmul/bmm/dot …), paddle/phi/kernels/*.

Hot ops (matmul) go through the AMP cast policy; on HIP devices torch.matmul dispatches to
hipBLASLt. Fused GEMM epilogues live in ``paddlepaddle_amd.ops``.
"""
from __future__ import annotations

import builtins
import math as _math

import numpy as _np
np = _np

import torch

from ..amp.state import maybe_cast
from ..framework import dtype as _dt
from ..framework.tensor import Tensor, _wrap
from ._helpers import T, TT, axis_arg, dtype_arg, scalar

_g = globals()


# ----------------------------------------------------------------------------- unary
def _make_unary(name, fn, inplace_fn=None):
    def op(x, name=None):
        return _wrap(fn(T(x)))
    op.__name__ = name
    op.__doc__ = f"paddle.{name} (elementwise). Reference: python/paddle/tensor/math.py"
    _g[name] = op

    def op_(x, name=None):
        t = x._t
        if inplace_fn is not None:
            inplace_fn(t)
        else:
            t.copy_(fn(t))
        return x
    op_.__name__ = name + "_"
    _g[name + "_"] = op_


_UNARY = {
    "abs": (torch.abs, torch.Tensor.abs_), "acos": (torch.acos, torch.Tensor.acos_),
    "acosh": (torch.acosh, torch.Tensor.acosh_), "asin": (torch.asin, torch.Tensor.asin_),
    "asinh": (torch.asinh, torch.Tensor.asinh_), "atan": (torch.atan, torch.Tensor.atan_),
    "atanh": (torch.atanh, torch.Tensor.atanh_), "ceil": (torch.ceil, torch.Tensor.ceil_),
    "cos": (torch.cos, torch.Tensor.cos_), "cosh": (torch.cosh, torch.Tensor.cosh_),
    "digamma": (torch.digamma, torch.Tensor.digamma_), "erf": (torch.erf, torch.Tensor.erf_),
    "erfinv": (torch.erfinv, torch.Tensor.erfinv_), "exp": (torch.exp, torch.Tensor.exp_),
    "expm1": (torch.expm1, torch.Tensor.expm1_), "floor": (torch.floor, torch.Tensor.floor_),
    "frac": (torch.frac, torch.Tensor.frac_), "lgamma": (torch.lgamma, torch.Tensor.lgamma_),
    "log": (torch.log, torch.Tensor.log_), "log10": (torch.log10, torch.Tensor.log10_),
    "log1p": (torch.log1p, torch.Tensor.log1p_), "log2": (torch.log2, torch.Tensor.log2_),
    "neg": (torch.neg, torch.Tensor.neg_), "reciprocal": (torch.reciprocal, torch.Tensor.reciprocal_),
    "round": (torch.round, torch.Tensor.round_), "rsqrt": (torch.rsqrt, torch.Tensor.rsqrt_),
    "sigmoid": (torch.sigmoid, torch.Tensor.sigmoid_), "sign": (torch.sign, torch.Tensor.sign_),
    "sin": (torch.sin, torch.Tensor.sin_), "sinh": (torch.sinh, torch.Tensor.sinh_),
    "sqrt": (torch.sqrt, torch.Tensor.sqrt_), "square": (torch.square, torch.Tensor.square_),
    "tan": (torch.tan, torch.Tensor.tan_), "tanh": (torch.tanh, torch.Tensor.tanh_),
    "trunc": (torch.trunc, torch.Tensor.trunc_), "i0": (torch.i0, torch.Tensor.i0_),
    "sinc": (torch.sinc, torch.Tensor.sinc_), "exp2": (torch.exp2, torch.Tensor.exp2_),
    "logit_plain": (torch.logit, None), "conj": (torch.conj_physical, None),
    "angle": (torch.angle, None), "signbit": (torch.signbit, None), "positive": (torch.positive, None),
    "sgn": (torch.sgn, None), "deg2rad": (torch.deg2rad, None), "rad2deg": (torch.rad2deg, None),
    "i0e": (torch.special.i0e, None), "i1": (torch.special.i1, None), "i1e": (torch.special.i1e, None),
    "gammaln": (torch.lgamma, None), "bitwise_not": (torch.bitwise_not, torch.Tensor.bitwise_not_),
    "logical_not": (torch.logical_not, torch.Tensor.logical_not_), "isnan": (torch.isnan, None),
    "isinf": (torch.isinf, None), "isfinite": (torch.isfinite, None), "isneginf": (torch.isneginf, None),
    "isposinf": (torch.isposinf, None), "isreal": (torch.isreal, None),
    "real": (torch.real, None), "imag": (torch.imag, None), "erfc": (torch.erfc, None),
}
for _n, (_f, _fi) in _UNARY.items():
    _make_unary(_n, _f, _fi)
bitwise_invert = _g["bitwise_not"]
bitwise_invert_ = _g["bitwise_not_"]


def _round_half_away(t, decimals=0):
    if not t.is_floating_point():
        return t
    if decimals:
        s = 10.0 ** decimals
        return torch.sign(t) * torch.floor(torch.abs(t) * s + 0.5) / s
    return torch.sign(t) * torch.floor(torch.abs(t) + 0.5)


def round(x, decimals=0, name=None):  # noqa: A001
    """paddle.round: halves round AWAY from zero (phi RoundFunctor uses std::round), not to even as
    torch.round does: round(-0.5) = -1. Reference: python/paddle/tensor/ops.py round."""
    return _wrap(_round_half_away(T(x), decimals))


def round_(x, decimals=0, name=None):
    x._t.copy_(_round_half_away(x._t, decimals))
    return x


def _digamma_paddle(t):
    # phi's digamma (Eigen) is NaN at the poles (0, -1, -2, ...); torch returns -inf at 0
    r = torch.digamma(t)
    return torch.where((t <= 0) & (t == torch.floor(t)), torch.full_like(r, float("nan")), r)


def digamma(x, name=None):
    """paddle.digamma. Reference: python/paddle/tensor/math.py digamma (NaN at non-positive integers)."""
    return _wrap(_digamma_paddle(T(x)))


def digamma_(x, name=None):
    x._t.copy_(_digamma_paddle(x._t))
    return x


def logit(x, eps=None, name=None):
    return _wrap(torch.logit(T(x), eps))


def logit_(x, eps=None, name=None):
    x._t.logit_(eps)
    return x


def stanh(x, scale_a=0.67, scale_b=1.7159, name=None):
    return _wrap(scale_b * torch.tanh(scale_a * T(x)))


def polygamma(x, n, name=None):
    return _wrap(torch.polygamma(n, T(x)))


def polygamma_(x, n, name=None):
    x._t.polygamma_(n)
    return x


def multigammaln(x, p, name=None):
    return _wrap(torch.mvlgamma(T(x), p))


def multigammaln_(x, p, name=None):
    x._t.mvlgamma_(p)
    return x


def gammainc(x, y, name=None):
    return _wrap(torch.special.gammainc(T(x), T(y)))


def gammaincc(x, y, name=None):
    return _wrap(torch.special.gammaincc(T(x), T(y)))


def gammainc_(x, y, name=None):
    x._t.copy_(torch.special.gammainc(x._t, T(y)))
    return x


def gammaincc_(x, y, name=None):
    x._t.copy_(torch.special.gammaincc(x._t, T(y)))
    return x


gammaln_ = _g["lgamma_"]


# ----------------------------------------------------------------------------- binary
def _bin_args(x, y):
    tx, ty = T(x), T(y)
    return tx, ty


def _make_binary(name, fn, inplace_name=None):
    def op(x, y, name=None):
        tx, ty = T(x), T(y)
        return _wrap(fn(tx, ty))
    op.__name__ = name
    op.__doc__ = f"paddle.{name} (broadcasting elementwise). Reference: python/paddle/tensor/math.py"
    _g[name] = op

    def op_(x, y, name=None):
        t = x._t
        r = fn(t, T(y))
        if r.dtype != t.dtype:
            r = r.to(t.dtype)
        if inplace_name is not None:
            getattr(t, inplace_name)(T(y))
        else:
            t.copy_(r)
        return x
    op_.__name__ = name + "_"
    _g[name + "_"] = op_


_BINARY = {
    "add": (torch.add, "add_"), "subtract": (torch.sub, "sub_"), "multiply": (torch.mul, "mul_"),
    "divide": (torch.true_divide, "div_"), "floor_divide": (lambda a, b: torch.div(a, b, rounding_mode="floor"), None),
    "remainder": (torch.remainder, "remainder_"), "pow": (torch.pow, "pow_"),
    "maximum": (torch.maximum, None), "minimum": (torch.minimum, None), "fmax": (torch.fmax, None),
    "fmin": (torch.fmin, None), "atan2": (torch.atan2, None), "hypot": (torch.hypot, None),
    "logaddexp": (torch.logaddexp, None), "heaviside": (torch.heaviside, None), "gcd": (torch.gcd, None),
    "lcm": (torch.lcm, None), "copysign": (torch.copysign, None), "nextafter": (torch.nextafter, None),
    "bitwise_and": (torch.bitwise_and, None), "bitwise_or": (torch.bitwise_or, None),
    "bitwise_xor": (torch.bitwise_xor, None),
    "logical_and": (torch.logical_and, None), "logical_or": (torch.logical_or, None),
    "logical_xor": (torch.logical_xor, None), "xlogy": (torch.xlogy, None),
    "ldexp": (lambda a, b: a * torch.pow(2.0, b), None),
}
for _n, (_f, _fi) in _BINARY.items():
    _make_binary(_n, _f, _fi)

mod = _g["remainder"]
mod_ = _g["remainder_"]


def _with_out(base, arity):
    """Reference signature of the logic / bitwise ops (tensor/logic.py): an optional ``out`` tensor that receives
    the result (and is returned)."""
    def put(r, out):
        if out is None:
            return r
        out._t.resize_(r._t.shape).copy_(r._t)
        return out
    if arity == 2:
        def op(x, y, out=None, name=None):
            return put(base(x, y), out)
    else:
        def op(x, out=None, name=None):
            return put(base(x), out)
    op.__name__, op.__qualname__, op.__doc__ = base.__name__, base.__name__, base.__doc__
    return op


for _n in ("bitwise_and", "bitwise_or", "bitwise_xor", "logical_and", "logical_or", "logical_xor"):
    _g[_n] = _with_out(_g[_n], 2)
for _n in ("bitwise_not", "logical_not"):
    _g[_n] = _with_out(_g[_n], 1)
bitwise_invert = _g["bitwise_not"]


def trunc(input, name=None):
    return _wrap(torch.trunc(T(input)))


def trunc_(input, name=None):
    input._t.trunc_()
    return input


def _unsigned_of(dt):
    return {torch.int8: torch.uint8, torch.int16: torch.int16, torch.int32: torch.int32,
            torch.int64: torch.int64, torch.uint8: torch.uint8}[dt]


def bitwise_left_shift(x, y, is_arithmetic=True, out=None, name=None):
    """paddle.bitwise_left_shift. Reference: python/paddle/tensor/math.py bitwise_left_shift (the arithmetic
    and logical left shifts are the same operation on two's-complement integers)."""
    return _wrap(torch.bitwise_left_shift(T(x), T(y)))


def bitwise_right_shift(x, y, is_arithmetic=True, out=None, name=None):
    """paddle.bitwise_right_shift: arithmetic (sign-extending) by default; ``is_arithmetic=False`` is the
    logical shift (zero fill), computed on the unsigned reinterpretation of the bits.
    Reference: python/paddle/tensor/math.py bitwise_right_shift."""
    tx, ty = T(x), T(y)
    if is_arithmetic or tx.dtype == torch.uint8:
        return _wrap(torch.bitwise_right_shift(tx, ty))
    if tx.dtype == torch.int8:
        return _wrap(torch.bitwise_right_shift(tx.view(torch.uint8), ty.to(torch.uint8)).view(torch.int8))
    bits = torch.iinfo(tx.dtype).bits
    ty = ty.to(tx.dtype)
    # logical shift of a signed value: arithmetic shift, then clear the sign-extended high bits
    sh = torch.bitwise_right_shift(tx, ty)
    mask = torch.where(ty > 0, torch.bitwise_left_shift(torch.ones_like(tx), (bits - ty).clamp(min=0, max=bits - 1)) - 1,
                       torch.full_like(tx, -1))
    mask = torch.where(ty >= bits, torch.zeros_like(tx), mask)
    return _wrap(torch.bitwise_and(sh, mask))


def bitwise_left_shift_(x, y, is_arithmetic=True, out=None, name=None):
    x._t.copy_(bitwise_left_shift(x, y, is_arithmetic)._t)
    return x


def bitwise_right_shift_(x, y, is_arithmetic=True, out=None, name=None):
    x._t.copy_(bitwise_right_shift(x, y, is_arithmetic)._t)
    return x
floor_mod = _g["remainder"]
floor_mod_ = _g["remainder_"]


def pow(x, y, name=None):  # noqa: A001
    tx = T(x)
    if isinstance(y, (int, float)) and not isinstance(y, bool):
        if y == 2:
            return _wrap(tx * tx)
        return _wrap(torch.pow(tx, y))
    return _wrap(torch.pow(tx, T(y)))


def float_power(x, y, name=None):
    return _wrap(torch.float_power(T(x), T(y)))


def scale(x, scale=1.0, bias=0.0, bias_after_scale=True, act=None, name=None):
    t = T(x)
    s = scalar(scale)
    if bias_after_scale:
        out = t * s + bias if bias != 0 else t * s
    else:
        out = (t + bias) * s
    if act is not None:
        out = getattr(torch, act)(out) if hasattr(torch, act) else getattr(torch.nn.functional, act)(out)
    return _wrap(out)


def scale_(x, scale=1.0, bias=0.0, bias_after_scale=True, act=None, name=None):
    x._t.copy_(_g["scale"](x, scale, bias, bias_after_scale, act)._t)
    return x


def clip(x, min=None, max=None, name=None):  # noqa: A002
    lo = scalar(min) if not isinstance(min, Tensor) or min._t.numel() == 1 else T(min)
    hi = scalar(max) if not isinstance(max, Tensor) or max._t.numel() == 1 else T(max)
    return _wrap(torch.clamp(T(x), lo, hi))


def clip_(x, min=None, max=None, name=None):  # noqa: A002
    x._t.clamp_(scalar(min), scalar(max))
    return x


def lerp(x, y, weight, name=None):
    w = T(weight)
    return _wrap(torch.lerp(T(x), T(y), w))


def lerp_(x, y, weight, name=None):
    x._t.lerp_(T(y), T(weight))
    return x


def add_n(inputs, name=None):
    if isinstance(inputs, Tensor):
        return inputs
    ts = [T(v) for v in inputs]
    out = ts[0]
    for t in ts[1:]:
        out = out + t
    return _wrap(out)


def increment(x, value=1.0, name=None):
    x._t.add_(value)
    return x


def addmm(input, x, y, beta=1.0, alpha=1.0, name=None):
    i, a, b = maybe_cast("addmm", T(input), T(x), T(y))
    return _wrap(torch.addmm(i, a, b, beta=beta, alpha=alpha))


def addmm_(input, x, y, beta=1.0, alpha=1.0, name=None):
    input._t.addmm_(T(x), T(y), beta=beta, alpha=alpha)
    return input


def baddbmm(input, x, y, beta=1.0, alpha=1.0, name=None):
    return _wrap(torch.baddbmm(T(input), T(x), T(y), beta=beta, alpha=alpha))


# ----------------------------------------------------------------------------- products
def matmul(x, y, transpose_x=False, transpose_y=False, name=None):
    """paddle.matmul. Reference: python/paddle/tensor/linalg.py matmul; phi matmul_kernel.
    On HIP devices: hipBLASLt (plain library GEMM)."""
    a, b = T(x), T(y)
    a, b = maybe_cast("matmul", a, b)
    if transpose_x:
        a = a.transpose(-1, -2) if a.dim() > 1 else a
    if transpose_y:
        b = b.transpose(-1, -2) if b.dim() > 1 else b
    if a.dtype != b.dtype:
        d = torch.promote_types(a.dtype, b.dtype)
        a, b = a.to(d), b.to(d)
    return _wrap(torch.matmul(a, b))


def mm(input, mat2, name=None):
    return matmul(input, mat2)


def bmm(x, y, name=None):
    a, b = maybe_cast("bmm", T(x), T(y))
    return _wrap(torch.bmm(a, b))


def mv(x, vec, name=None):
    a, b = maybe_cast("mv", T(x), T(vec))
    return _wrap(torch.mv(a, b))


def dot(x, y, name=None):
    a, b = T(x), T(y)
    if a.dim() == 2:
        return _wrap((a * b).sum(-1))
    return _wrap(torch.dot(a, b))


def vecdot(x, y, axis=-1, name=None):
    return _wrap(torch.linalg.vecdot(T(x), T(y), dim=axis))


def inner(x, y, name=None):
    return _wrap(torch.inner(T(x), T(y)))


def outer(x, y, name=None):
    return _wrap(torch.outer(T(x).flatten(), T(y).flatten()))


def kron(x, y, name=None):
    return _wrap(torch.kron(T(x), T(y)))


def cross(x, y, axis=9, name=None):
    tx, ty = T(x), T(y)
    if axis == 9:
        axis = next(i for i, s in enumerate(tx.shape) if s == 3)
    return _wrap(torch.linalg.cross(tx, ty, dim=axis))


def tensordot(x, y, axes=2, name=None):
    """paddle.tensordot. Reference: python/paddle/tensor/manipulation.py tensordot: ``axes`` is an int n (last n
    of x with first n of y), a flat list (the same axes of x and y), or [axes_x, axes_y] where the shorter list is
    extended with the longer one's tail; contracted axes broadcast (size 1 against size n)."""
    tx, ty = T(x), T(y)
    if isinstance(axes, Tensor):
        axes = axes._t.tolist()
    if isinstance(axes, int):
        ax_x, ax_y = list(range(tx.dim() - axes, tx.dim())), list(range(axes))
    else:
        axes = list(axes)
        if len(axes) == 0:
            ax_x, ax_y = [], []
        elif builtins.all(isinstance(a, int) for a in axes):
            ax_x, ax_y = list(axes), list(axes)
        else:
            seqs = [list(a._t.tolist() if isinstance(a, Tensor) else a) for a in axes[:2]]
            ax_x = seqs[0]
            ax_y = seqs[1] if len(seqs) > 1 else list(seqs[0])
            if len(ax_x) < len(ax_y):
                ax_x = ax_x + ax_y[len(ax_x):]
            elif len(ax_y) < len(ax_x):
                ax_y = ax_y + ax_x[len(ax_y):]
    ax_x = [a % tx.dim() for a in ax_x]
    ax_y = [a % ty.dim() for a in ax_y]
    for a, b in zip(ax_x, ax_y):
        if tx.shape[a] != ty.shape[b]:
            if tx.shape[a] == 1:
                ty = ty.sum(b, keepdim=True)
            elif ty.shape[b] == 1:
                tx = tx.sum(a, keepdim=True)
    return _wrap(torch.tensordot(tx, ty, dims=(ax_x, ax_y)))


def multiplex(inputs, index, name=None):
    idx = T(index).flatten().long()
    stacked = torch.stack([T(v) for v in inputs], 0)
    rows = torch.arange(stacked.shape[1], device=idx.device)
    return _wrap(stacked[idx, rows])


def trace(x, offset=0, axis1=0, axis2=1, name=None):
    return _wrap(torch.diagonal(T(x), offset, axis1, axis2).sum(-1))


def diagonal(x, offset=0, axis1=0, axis2=1, name=None):
    return _wrap(torch.diagonal(T(x), offset, axis1, axis2))


# ----------------------------------------------------------------------------- reductions
def _red_dtype(t, dtype):
    if dtype is not None:
        return dtype_arg(dtype)
    if t.dtype in (torch.bool, torch.int32, torch.int16, torch.int8, torch.uint8):
        return torch.int64
    return None


def sum(x, axis=None, dtype=None, keepdim=False, name=None):  # noqa: A001
    t = T(x)
    ax = axis_arg(axis)
    d = _red_dtype(t, dtype)
    if ax is None:
        r = t.sum(dtype=d)
        if keepdim:
            r = r.reshape([1] * t.dim())
        return _wrap(r)
    return _wrap(t.sum(ax, keepdim=keepdim, dtype=d))


def nansum(x, axis=None, dtype=None, keepdim=False, name=None):
    t = T(x)
    ax = axis_arg(axis)
    if ax is None:
        return _wrap(torch.nansum(t, dtype=dtype_arg(dtype)))
    return _wrap(torch.nansum(t, ax, keepdim=keepdim, dtype=dtype_arg(dtype)))


def mean(x, axis=None, keepdim=False, name=None):
    t = T(x)
    ax = axis_arg(axis)
    if ax is None:
        r = t.mean()
        if keepdim:
            r = r.reshape([1] * t.dim())
        return _wrap(r)
    return _wrap(t.mean(ax, keepdim=keepdim))


def nanmean(x, axis=None, keepdim=False, name=None):
    ax = axis_arg(axis)
    return _wrap(torch.nanmean(T(x), ax, keepdim=keepdim) if ax is not None else torch.nanmean(T(x)))


def prod(x, axis=None, keepdim=False, dtype=None, name=None):
    t = T(x)
    ax = axis_arg(axis)
    d = dtype_arg(dtype)
    if ax is None:
        return _wrap(t.prod(dtype=d))
    if isinstance(ax, tuple):
        for a in sorted([a % t.dim() for a in ax], reverse=True):
            t = t.prod(a, keepdim=keepdim, dtype=d)
        return _wrap(t)
    return _wrap(t.prod(ax, keepdim=keepdim, dtype=d))


def _minmax(fn):
    def op(x, axis=None, keepdim=False, name=None):
        t = T(x)
        ax = axis_arg(axis)
        if ax is None:
            r = fn(t)
            if keepdim:
                r = r.reshape([1] * t.dim())
            return _wrap(r)
        return _wrap(fn(t, dim=ax, keepdim=keepdim))
    return op


class _MaxAllTies(torch.autograd.Function):
    """paddle.max / paddle.min gradient: EVERY element equal to the extreme receives the full upstream gradient
    (paddle/phi/kernels/funcs/reduce_grad_functions.h MaxOrMinGrad: dx = dy * (x == y)); amax / amin instead
    split it evenly between ties (torch.amax's rule). Reference: python/paddle/tensor/math.py max (docstring
    example: 5 tied maxima each get 1.0 from max and 0.2 from amax)."""

    @staticmethod
    def forward(ctx, t, dims, keepdim, is_max):
        r = (torch.amax if is_max else torch.amin)(t, dim=dims, keepdim=True)
        ctx.save_for_backward(t, r)
        return r if keepdim else r.reshape([d for i, d in enumerate(t.shape) if i not in dims])

    @staticmethod
    def backward(ctx, g):
        t, r = ctx.saved_tensors
        return (t == r).to(g.dtype) * g.reshape(r.shape), None, None, None


def _minmax_ties(is_max):
    def op(x, axis=None, keepdim=False, name=None):
        t = T(x)
        ax = axis_arg(axis)
        if not t.requires_grad or not torch.is_grad_enabled():
            fn = torch.amax if is_max else torch.amin
            if ax is None:
                r = fn(t)
                return _wrap(r.reshape([1] * t.dim()) if keepdim else r)
            return _wrap(fn(t, dim=ax, keepdim=keepdim))
        dims = tuple(range(t.dim())) if ax is None else tuple(a % builtins.max(t.dim(), 1) for a in
                                                               (ax if isinstance(ax, tuple) else (ax,)))
        return _wrap(_MaxAllTies.apply(t, dims, keepdim, is_max))
    return op


max = _minmax_ties(True)  # noqa: A001
min = _minmax_ties(False)  # noqa: A001
amax = _minmax(torch.amax)
amin = _minmax(torch.amin)


def all(x, axis=None, keepdim=False, name=None):  # noqa: A001
    t = T(x)
    ax = axis_arg(axis)
    if ax is None:
        return _wrap(t.all())
    return _wrap(t.all(dim=ax, keepdim=keepdim))


def any(x, axis=None, keepdim=False, name=None):  # noqa: A001
    t = T(x)
    ax = axis_arg(axis)
    if ax is None:
        return _wrap(t.any())
    return _wrap(t.any(dim=ax, keepdim=keepdim))


def logsumexp(x, axis=None, keepdim=False, name=None):
    t = T(x)
    ax = axis_arg(axis)
    if ax is None:
        ax = tuple(range(t.dim()))
    return _wrap(torch.logsumexp(t, ax, keepdim=keepdim))


def count_nonzero(x, axis=None, keepdim=False, name=None):
    t = T(x)
    ax = axis_arg(axis)
    r = (t != 0).sum(ax, keepdim=keepdim) if ax is not None else (t != 0).sum()
    return _wrap(r.to(torch.int64))


def reduce_as(x, target, name=None):
    t, tg = T(x), T(target)
    nd = t.dim() - tg.dim()
    if nd > 0:
        t = t.sum(tuple(range(nd)))
    dims = tuple(i for i, (a, b) in enumerate(zip(t.shape, tg.shape)) if a != b and b == 1)
    if dims:
        t = t.sum(dims, keepdim=True)
    return _wrap(t)


# ----------------------------------------------------------------------------- cumulative
def cumsum(x, axis=None, dtype=None, name=None):
    t = T(x)
    if axis is None:
        t = t.flatten()
        axis = 0
    return _wrap(torch.cumsum(t, int(axis), dtype=dtype_arg(dtype)))


def cumsum_(x, axis=None, dtype=None, name=None):
    x._t.copy_(cumsum(x, axis, dtype)._t.reshape(x._t.shape))
    return x


def cumprod(x, dim=None, dtype=None, name=None):
    t = T(x)
    if dim is None:
        t = t.flatten()
        dim = 0
    return _wrap(torch.cumprod(t, dim, dtype=dtype_arg(dtype)))


def cumprod_(x, dim=None, dtype=None, name=None):
    x._t.copy_(cumprod(x, dim, dtype)._t.reshape(x._t.shape))
    return x


def cummax(x, axis=None, dtype="int64", name=None):
    t = T(x)
    if axis is None:
        t, axis = t.flatten(), 0
    v, i = torch.cummax(t, axis)
    return _wrap(v), _wrap(i.to(dtype_arg(dtype)))


def cummin(x, axis=None, dtype="int64", name=None):
    t = T(x)
    if axis is None:
        t, axis = t.flatten(), 0
    v, i = torch.cummin(t, axis)
    return _wrap(v), _wrap(i.to(dtype_arg(dtype)))


def logcumsumexp(x, axis=None, dtype=None, name=None):
    t = T(x)
    if axis is None:
        t, axis = t.flatten(), 0
    if dtype is not None:
        t = t.to(dtype_arg(dtype))
    return _wrap(torch.logcumsumexp(t, axis))


def diff(x, n=1, axis=-1, prepend=None, append=None, name=None):
    return _wrap(torch.diff(T(x), n, axis, prepend=T(prepend), append=T(append)))


def trapezoid(y, x=None, dx=None, axis=-1, name=None):
    if x is not None:
        return _wrap(torch.trapezoid(T(y), T(x), dim=axis))
    return _wrap(torch.trapezoid(T(y), dx=1.0 if dx is None else dx, dim=axis))


def cumulative_trapezoid(y, x=None, dx=None, axis=-1, name=None):
    if x is not None:
        return _wrap(torch.cumulative_trapezoid(T(y), T(x), dim=axis))
    return _wrap(torch.cumulative_trapezoid(T(y), dx=1.0 if dx is None else dx, dim=axis))


def renorm(x, p, axis, max_norm, name=None):
    return _wrap(torch.renorm(T(x), p, axis, max_norm))


def renorm_(x, p, axis, max_norm, name=None):
    x._t.renorm_(p, axis, max_norm)
    return x


def nan_to_num(x, nan=0.0, posinf=None, neginf=None, name=None):
    return _wrap(torch.nan_to_num(T(x), nan, posinf, neginf))


def nan_to_num_(x, nan=0.0, posinf=None, neginf=None, name=None):
    x._t.nan_to_num_(nan, posinf, neginf)
    return x


def frexp(x, name=None):
    m, e = torch.frexp(T(x))
    return _wrap(m), _wrap(e.to(T(x).dtype))


def broadcast_shape(x_shape, y_shape):
    return list(torch.broadcast_shapes(tuple(x_shape), tuple(y_shape)))


def inverse(x, name=None):
    from .linalg import _inv  # LU factor + pivot gather + two triangular solves
    return _wrap(_inv(T(x)))


def isclose(x, y, rtol=1e-05, atol=1e-08, equal_nan=False, name=None):
    return _wrap(torch.isclose(T(x), T(y), rtol, atol, equal_nan))


def allclose(x, y, rtol=1e-05, atol=1e-08, equal_nan=False, name=None):
    return _wrap(torch.tensor(torch.allclose(T(x), T(y), rtol, atol, equal_nan)))


def histogram(input, bins=100, min=0, max=0, weight=None, density=False, name=None):  # noqa: A002
    t = T(input).float()
    lo, hi = float(min), float(max)
    if lo == 0 and hi == 0:
        lo, hi = t.min().item(), t.max().item()
    h = torch.histc(t.flatten().cpu(), bins, lo, hi) if weight is None else \
        torch.histogram(t.flatten().cpu(), bins, range=(lo, hi), weight=T(weight).flatten().float().cpu(), density=density)[0]
    if density and weight is None:
        h = h / (h.sum() * (hi - lo) / bins)
    return _wrap(h.to(t.device) if density or weight is not None else h.to(torch.int64).to(t.device))


def histogram_bin_edges(input, bins=100, min=0, max=0, name=None):  # noqa: A002
    t = T(input).float()
    lo, hi = float(min), float(max)
    if lo == 0 and hi == 0:
        lo, hi = t.min().item(), t.max().item()
    return _wrap(torch.linspace(lo, hi, bins + 1, device=t.device))


def histogramdd(x, bins=10, ranges=None, density=False, weights=None, name=None):
    h, edges = torch.histogramdd(T(x).cpu().float(), bins, range=ranges, density=density,
                                 weight=None if weights is None else T(weights).cpu().float())
    return _wrap(h), [_wrap(e) for e in edges]


def bincount(x, weights=None, minlength=0, name=None):
    return _wrap(torch.bincount(T(x), None if weights is None else T(weights), minlength))


def combinations(x, r=2, with_replacement=False, name=None):
    return _wrap(torch.combinations(T(x), r, with_replacement))


def take(x, index, mode="raise", name=None):
    t = T(x).flatten()
    i = T(index).long()
    n = t.numel()
    if mode == "wrap":
        i = torch.remainder(i, n)
    elif mode == "clip":
        i = i.clamp(0, n - 1)
    else:
        i = torch.where(i < 0, i + n, i)
    return _wrap(t[i])


def sinc_(x, name=None):
    x._t.sinc_()
    return x


def atleast_1d(*inputs, name=None):
    r = [_wrap(torch.atleast_1d(T(v))) for v in inputs]
    return r[0] if len(r) == 1 else r


def atleast_2d(*inputs, name=None):
    r = [_wrap(torch.atleast_2d(T(v))) for v in inputs]
    return r[0] if len(r) == 1 else r


def atleast_3d(*inputs, name=None):
    r = [_wrap(torch.atleast_3d(T(v))) for v in inputs]
    return r[0] if len(r) == 1 else r


def cdist(x, y, p=2.0, compute_mode="use_mm_for_euclid_dist_if_necessary", name=None):
    return _wrap(torch.cdist(T(x), T(y), p, compute_mode=compute_mode))


def pdist(x, p=2.0, name=None):
    return _wrap(torch.pdist(T(x), p))


def dist(x, y, p=2, name=None):
    return _wrap(torch.dist(T(x), T(y), p))


def neg_(x, name=None):
    x._t.neg_()
    return x
