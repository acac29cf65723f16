"""Conv -> BN fusion bookkeeping (reference: paddle/phi/kernels/fusion/gpu/fused_scale_bias_relu_conv_bn_kernel.cu,
which computes the batch-norm sums of the convolution output inside the convolution).

Here the producing kernel writes the BN partials in its epilogue (csrc/kernels/gemm.hip ``kEpiStats``) and the
BN forward (ops/bn.py) skips its statistics pass over the activation. No model change is needed: every
convolution output carries its shape key; a training BN that consumes it records the key, and from then on the
convolution of that key produces the statistics as well (the first step runs unfused). The partials are used
only while the tensor is unmodified (same storage and version counter).
"""
from __future__ import annotations

import weakref

import torch

from . import _loader as L

_FEEDS_BN: set = set()   # conv keys whose output a training BN consumed
_PENDING = [None]        # (stats, chunks) of the last _ConvNHWC forward, attached by conv2d_nhwc
_PENDING_BN = [None]     # (x2, mean, ss) of the last relu BN forward without residual, attached to its output
_BWD: dict = {}          # data_ptr of a conv data gradient -> (stats, chunks, numel, version, BN input data_ptr)


def enabled() -> bool:
    return bool(L.flag("FLAGS_conv_bn_fusion", True))


def wanted(key) -> bool:
    return key in _FEEDS_BN and torch.is_grad_enabled() and enabled()


def tag(y, key, pre):
    y._pa_conv_key = key
    y._pa_bn_pre = (pre[0], pre[1], y._version) if pre is not None else None


def _producer(x):
    t = x
    for _ in range(2):
        if t is None:
            return None
        if getattr(t, "_pa_conv_key", None) is not None:
            return t
        t = t._base
    return None


def take(x):
    """(stats, chunks) the convolution that produced ``x`` wrote for it, or None; records the producer key."""
    t = _producer(x)
    if t is None:
        return None
    _FEEDS_BN.add(t._pa_conv_key)
    pre = getattr(t, "_pa_bn_pre", None)
    if pre is None or pre[2] != t._version:
        return None
    if t.data_ptr() != x.data_ptr() or t.numel() != x.numel() or t.shape[-1] != x.shape[-1]:
        return None
    t._pa_bn_pre = None  # consumed once; the partials are not kept alive with the activation
    return pre[0], pre[1]


# ---------------------------------------------------------------- backward: dconv -> drelu -> dBN statistics
# (reference fusion/gpu/fused_dconv_drelu_dbn_kernel.cu). A relu BN without residual tags its output with its
# input, mean and scale / shift; the convolution consuming that output computes its data gradient (the BN's
# output gradient) with an epilogue that also writes [sum dyp, sum dyp * (x - mean)], and the BN backward
# starts from them instead of its reduction pass over dy and x.
def tag_bn_output(y, src):
    y._pa_bn_src = src


def bn_source(x):
    """(bn_input, mean, ss) when ``x`` is (a view of) an untouched relu BN output, else None."""
    if not enabled():
        return None
    t = x
    for _ in range(2):
        if t is None:
            return None
        src = getattr(t, "_pa_bn_src", None)
        if src is not None:
            if t.data_ptr() != x.data_ptr() or t.numel() != x.numel():
                return None
            return src
        t = t._base
    return None


def put_bwd(dx, stats, chunks, bn_x):
    # a weak reference to the gradient tensor itself: an entry whose gradient died (or a later tensor reusing
    # its address) can never match
    _BWD[dx.data_ptr()] = (stats, chunks, weakref.ref(dx), dx._version, bn_x.data_ptr())
    for k in [k for k, v in _BWD.items() if v[2]() is None]:
        del _BWD[k]


def take_bwd(dy, bn_x):
    rec = _BWD.pop(dy.data_ptr(), None)
    if rec is None:
        return None
    stats, chunks, ref, version, xp = rec
    g = ref()
    if g is None or not (dy is g or dy._base is g or (g._base is not None and dy._base is g._base)):
        return None
    if g.numel() != dy.numel() or xp != bn_x.data_ptr() or g._version != version:
        return None
    return stats, chunks


def reduce_cost(y):
    """The BN statistics pass a producer without the fused epilogue leaves to the BN (timed with the
    candidates that lack it, so the per-shape choice compares equal work)."""
    C = y.shape[-1]
    R = y.numel() // C
    from .bn import _chunks
    partial = torch.empty(2 * _chunks(R, C) * C, dtype=torch.float32, device=y.device)
    sums = torch.empty(2, C, dtype=torch.float32, device=y.device)
    L.call("pa_bn_reduce_nhwc", 0, L.ptr(y), L.ptr(None), L.ptr(None), L.ptr(None), L.ptr(None), L.ptr(partial),
           L.ptr(sums), R, C, 0, L.stream_ptr())
    return y


def reduce_cost_bwd(dx, src):
    """The BN-backward reduction (relu mask from x * scale + shift) a data gradient without the fused epilogue
    leaves to the BN."""
    bx, mean, ss = src
    C = dx.shape[-1]
    R = dx.numel() // C
    from .bn import _chunks
    partial = torch.empty(2 * _chunks(R, C) * C, dtype=torch.float32, device=dx.device)
    sums = torch.empty(2, C, dtype=torch.float32, device=dx.device)
    L.call("pa_bn_reduce_nhwc", 1, L.ptr(bx), L.ptr(dx), L.ptr(None), L.ptr(mean), L.ptr(ss), L.ptr(partial),
           L.ptr(sums), R, C, 1, L.stream_ptr())
    return dx
