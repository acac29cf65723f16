"""Convolutions. Reference: python/paddle/nn/functional/conv.py, phi/kernels/gpu/conv_kernel.cu (cuDNN).

MI355X path: MIOpen through ATen with NHWC (channels_last) bf16 tensors — NHWC data_format is a
zero-copy view here (logical NCHW with channels-last strides), which is what MIOpen's fast
implicit-GEMM/Winograd solvers want on CDNA.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ...amp.state import maybe_cast
from ...framework import layout_autotune as _lat
from ...framework.tensor import Tensor, _wrap
from ...tensor._helpers import T


def _tuple(v, n):
    if isinstance(v, (list, tuple)):
        return tuple(int(x) for x in v)
    return (int(v),) * n


def _padding(padding, n, x_spatial, k_spatial, stride, dilation):
    """Return (torch_padding, pre_pad) where pre_pad is an explicit asymmetric F.pad list or None."""
    if isinstance(padding, str):
        p = padding.upper()
        if p == "VALID":
            return 0, None
        if p == "SAME":
            pads = []
            for xs, ks, st, dl in zip(x_spatial, k_spatial, stride, dilation):
                out = (xs + st - 1) // st
                total = max((out - 1) * st + (ks - 1) * dl + 1 - xs, 0)
                pads.append((total // 2, total - total // 2))
            if all(a == b for a, b in pads):
                return tuple(a for a, _ in pads), None
            flat = []
            for a, b in reversed(pads):
                flat += [a, b]
            return 0, flat
    if isinstance(padding, (list, tuple)):
        if len(padding) and isinstance(padding[0], (list, tuple)):
            sp = [tuple(p) for p in padding]
            sp = [p for p in sp if True]
            # [[0,0],[0,0],[t,b],[l,r]] (NCHW) or [[0,0],[t,b],[l,r],[0,0]] (NHWC)
            sp = [p for p in sp][-n - 1:-1] if len(sp) == n + 2 and tuple(sp[-1]) == (0, 0) and tuple(sp[1]) != (0, 0) else sp[-n:]
            if all(a == b for a, b in sp):
                return tuple(a for a, _ in sp), None
            flat = []
            for a, b in reversed(sp):
                flat += [a, b]
            return 0, flat
        if len(padding) == 2 * n:
            pairs = [(padding[2 * i], padding[2 * i + 1]) for i in range(n)]
            if all(a == b for a, b in pairs):
                return tuple(a for a, _ in pairs), None
            flat = []
            for a, b in reversed(pairs):
                flat += [a, b]
            return 0, flat
        return tuple(int(p) for p in padding), None
    return int(padding), None


def _to_cf(t, data_format, n):
    """channel-last logical -> channel-first logical (zero-copy view)."""
    if data_format in ("NHWC", "NLC", "NDHWC"):
        return t.permute(0, n + 1, *range(1, n + 1)), True
    return t, False


def _from_cf(t, cl, n):
    if cl:
        return t.permute(0, *range(2, n + 2), 1)
    return t


def _convnd(n, x, weight, bias, stride, padding, dilation, groups, data_format):
    if n == 2 and data_format == "NCHW" and _lat.applies(T(x)):
        # layout autotune: the NHWC kernels on the channels-last view, result handed back as logical NCHW
        y = _convnd(2, _wrap(_lat.to_nhwc_view(T(x))), weight, bias, stride, padding, dilation, groups, "NHWC")
        return _wrap(_lat.to_nchw_view(T(y)))
    t = T(x)
    w = T(weight)
    t, w = maybe_cast("conv2d", t, w)
    b = T(bias)
    if b is not None and b.dtype != w.dtype:
        b = b.to(w.dtype)
    x_raw = t
    t, cl = _to_cf(t, data_format, n)
    stride = _tuple(stride, n)
    dilation = _tuple(dilation, n)
    pad, pre = _padding(padding, n, t.shape[2:], w.shape[2:], stride, dilation)
    fn = {1: F.conv1d, 2: F.conv2d, 3: F.conv3d}[n]

    def miopen(tt, ww):
        if pre is not None:
            tt = F.pad(tt, pre)
        if cl and n == 2 and not ww.is_contiguous(memory_format=torch.channels_last):
            ww = ww.contiguous(memory_format=torch.channels_last)
        return fn(tt, ww, b, stride, pad, dilation, groups)

    # NHWC depthwise convolutions: direct HIP kernels (ops/dwconv.py) when they measured faster than MIOpen
    if cl and n == 2 and pre is None and groups > 1:
        from ... import ops as _ops
        if _ops.dwconv.eligible(x_raw, w, groups):
            pd = (pad, pad) if isinstance(pad, int) else tuple(pad)
            y = _ops.dwconv.depthwise_conv2d_nhwc(
                x_raw, w, b, stride, pd, dilation,
                lambda xx, ww: _from_cf(miopen(_to_cf(xx, data_format, n)[0], ww), cl, n))
            if y is not None:
                return _wrap(y)
    # NHWC 1x1 convolutions: hand-written MFMA GEMM (ops/conv.py) when it measured faster than MIOpen
    if cl and n == 2 and pre is None and stride[0] == stride[1]:
        from ... import ops as _ops
        pd = pad if isinstance(pad, int) else (pad[0] if pad[0] == pad[1] else None)
        one = tuple(w.shape[2:]) == (1, 1)
        if (_ops._loader.flag("FLAGS_conv_per_direction", True) and pd is not None
                and dilation[0] == dilation[1] and (not one or (pd == 0 and dilation[0] == 1))
                and _ops.conv.eligible_nhwc(x_raw, w, groups)):
            # each of forward / data gradient / weight gradient on the faster of ours and MIOpen (ops/conv.py)
            return _wrap(_ops.conv.conv2d_nhwc(x_raw, w, b, stride[0], pd, dilation[0]))
        if (pad == 0 or pad == (0, 0)) and _ops.conv.eligible(x_raw, w, groups, True):
            y = _ops.conv.conv1x1_nhwc(x_raw, w, b, stride[0],
                                       lambda xx, ww: _from_cf(miopen(_to_cf(xx, data_format, n)[0], ww), cl, n))
            if y is not None:
                return _wrap(y)
        elif (w.shape[2] > 1 or w.shape[3] > 1) and dilation[0] == dilation[1] and \
                (isinstance(pad, int) or pad[0] == pad[1]) and _ops.conv.eligible_implicit(x_raw, w, groups):
            pd = pad if isinstance(pad, int) else pad[0]
            y = _ops.conv.conv_implicit_nhwc(x_raw, w, b, stride[0], pd, dilation[0],
                                             lambda xx, ww: _from_cf(miopen(_to_cf(xx, data_format, n)[0], ww), cl, n))
            if y is not None:
                return _wrap(y)
    # NDHWC 3-D convolutions: forward on the 3-D implicit GEMM when it measured faster than MIOpen
    if cl and n == 3 and pre is None and groups == 1 and t.is_cuda and len(set(stride)) == 1 and \
            len(set(dilation)) == 1:
        from ... import ops as _ops
        pads = (pad,) * 3 if isinstance(pad, int) else tuple(pad)
        if len(pads) == 3 and _ops.conv.conv3d_ndhwc_ok(x_raw, w, groups, stride[0], pads, dilation[0]):
            return _wrap(_ops.conv.conv3d_ndhwc(x_raw, w, b, stride[0], pads, dilation[0]))
    # NLC 1-D convolutions: the NHWC kernels on a 1 x L image with a 1 x K filter (padding (0, p)); each of the
    # three products again on the faster of ours and MIOpen (the data gradient of a 1 x K filter: MIOpen)
    if cl and n == 1 and pre is None and groups == 1 and t.is_cuda:
        from ... import ops as _ops
        pd = pad if isinstance(pad, int) else (pad[0] if len(pad) == 1 else None)
        if pd is not None and _ops._loader.flag("FLAGS_conv_per_direction", True):
            x4, w4 = x_raw.unsqueeze(1), w.unsqueeze(2)
            one = w4.shape[3] == 1
            if (not one or (pd == 0 and dilation[0] == 1)) and _ops.conv.eligible_nhwc(x4, w4, 1):
                y = _ops.conv.conv2d_nhwc(x4, w4, b, stride[0], 0 if one else (0, pd), dilation[0])
                return _wrap(y.squeeze(1))
    out = miopen(t, w)
    return _wrap(_from_cf(out, cl, n))


def conv1d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NCL", name=None):
    return _convnd(1, x, weight, bias, stride, padding, dilation, groups, data_format)


def conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NCHW", name=None):
    return _convnd(2, x, weight, bias, stride, padding, dilation, groups, data_format)


def conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NCDHW", name=None):
    return _convnd(3, x, weight, bias, stride, padding, dilation, groups, data_format)


def _conv_transpose_nd(n, x, weight, bias, stride, padding, output_padding, dilation, groups, output_size,
                       data_format):
    t = T(x)
    w = T(weight)
    t, w = maybe_cast("conv2d_transpose", t, w)
    b = T(bias)
    if b is not None and b.dtype != w.dtype:
        b = b.to(w.dtype)
    t, cl = _to_cf(t, data_format, n)
    stride = _tuple(stride, n)
    dilation = _tuple(dilation, n)
    if isinstance(padding, str):
        padding = 0 if padding.upper() == "VALID" else tuple((k - 1) * d // 2 for k, d in zip(w.shape[2:], dilation))
    pad = _tuple(padding, n) if not (isinstance(padding, (list, tuple)) and len(padding) == 2 * n) else \
        tuple(padding[2 * i] for i in range(n))
    op = _tuple(output_padding, n)
    if output_size is not None:
        osz = _tuple(output_size, n) if not isinstance(output_size, Tensor) else tuple(output_size._t.tolist())
        op = tuple(o - ((i - 1) * s - 2 * p + d * (k - 1) + 1) for o, i, s, p, d, k in
                   zip(osz, t.shape[2:], stride, pad, dilation, w.shape[2:]))
    if (cl and n == 2 and groups == 1 and stride == (1, 1) and dilation == (1, 1) and op == (0, 0)
            and all(k - 1 - q >= 0 for k, q in zip(w.shape[2:], pad)) and w.shape[2] == w.shape[3]
            and pad[0] == pad[1] and t.is_cuda):
        # stride-1 transposed convolution == convolution with the flipped, in/out-swapped filter and padding
        # K-1-p: the NHWC convolution path (hand-written implicit GEMM / 1x1 GEMM kernels when they measured
        # faster than MIOpen); the filter transform is part of the autograd graph, so dW flows back to `weight`
        w2 = w.flip(2, 3).transpose(0, 1)
        return _convnd(2, _wrap(_from_cf(t, cl, n)), _wrap(w2), None if b is None else _wrap(b), 1,
                       w.shape[2] - 1 - pad[0], 1, 1, data_format)
    fn = {1: F.conv_transpose1d, 2: F.conv_transpose2d, 3: F.conv_transpose3d}[n]
    out = fn(t, w, b, stride, pad, op, groups, dilation)
    return _wrap(_from_cf(out, cl, n))


def conv1d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1,
                     output_size=None, data_format="NCL", name=None):
    return _conv_transpose_nd(1, x, weight, bias, stride, padding, output_padding, dilation, groups,
                              output_size, data_format)


def conv2d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, dilation=1, groups=1,
                     output_size=None, data_format="NCHW", name=None):
    return _conv_transpose_nd(2, x, weight, bias, stride, padding, output_padding, dilation, groups,
                              output_size, data_format)


def conv3d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1,
                     output_size=None, data_format="NCDHW", name=None):
    return _conv_transpose_nd(3, x, weight, bias, stride, padding, output_padding, dilation, groups,
                              output_size, data_format)
