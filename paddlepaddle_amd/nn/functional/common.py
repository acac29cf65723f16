"""Common functional ops: linear, dropout, pad, interpolate, embedding, one_hot …
Reference: python/paddle/nn/functional/{common,input}.py."""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from ...amp.state import maybe_cast
from ...framework.tensor import Tensor, _wrap
from ...tensor._helpers import T, shape_arg
from ... import ops as _ops


def linear(x, weight, bias=None, name=None):
    """y = x @ W + b with W [in, out] (paddle layout). hipBLASLt GEMM with the bias in the epilogue."""
    a, w = maybe_cast("linear", T(x), T(weight))
    b = T(bias)
    if b is not None and b.dtype != w.dtype:
        b = b.to(w.dtype)
    if w.dim() == 1:  # a vector weight (e.g. set by the Assign initializer): matmul semantics
        y = torch.matmul(a, w)
        return _wrap(y + b if b is not None else y)
    return _wrap(_ops.fused_linear(a, w, b))


def dropout(x, p=0.5, axis=None, training=True, mode="upscale_in_train", name=None):
    t = T(x)
    if not training or p == 0:
        if mode == "downscale_in_infer" and not training:
            return _wrap(t * (1 - p))
        return x if isinstance(x, Tensor) else _wrap(t)
    if p == 1:
        return _wrap(torch.zeros_like(t))
    if axis is not None:
        ax = [axis] if isinstance(axis, int) else list(axis)
        shape = [t.shape[i] if i in [a % t.dim() for a in ax] else 1 for i in range(t.dim())]
        mask = (torch.rand(shape, device=t.device) >= p).to(t.dtype)
        out = t * mask
        return _wrap(out / (1 - p) if mode == "upscale_in_train" else out)
    if mode == "upscale_in_train":
        return _wrap(_ops.dropout_add(t, None, p, True))
    mask = (torch.rand_like(t, dtype=torch.float32) >= p).to(t.dtype)
    return _wrap(t * mask)


def dropout2d(x, p=0.5, training=True, data_format="NCHW", name=None):
    t = T(x)
    if data_format == "NHWC":
        t = t.permute(0, 3, 1, 2)
        return _wrap(F.dropout2d(t, p, training).permute(0, 2, 3, 1))
    return _wrap(F.dropout2d(t, p, training))


def dropout3d(x, p=0.5, training=True, data_format="NCDHW", name=None):
    return _wrap(F.dropout3d(T(x), p, training))


def alpha_dropout(x, p=0.5, training=True, name=None):
    return _wrap(F.alpha_dropout(T(x), p, training))


def feature_alpha_dropout(x, p=0.5, training=True, name=None):
    return _wrap(F.feature_alpha_dropout(T(x), p, training))


def pad(x, pad, mode="constant", value=0.0, data_format=None, pad_from_left_axis=True, name=None):
    """paddle.nn.functional.pad. Reference: python/paddle/nn/functional/common.py pad (Note 1-3):
    constant mode with a list whose length is not 2*(N-2) pads whole axes — a 2N list from the first axis
    forward (``pad_from_left_axis``) or from the last axis backward, a shorter list from the last axis;
    every other case pads the spatial axes of ``data_format`` ([left, right, top, bottom, front, back])."""
    t = T(x)
    pad_is_tensor = isinstance(pad, Tensor)
    if pad_is_tensor:
        pad = pad._t.tolist()
    pad = [int(p) for p in pad]
    nd = t.dim()
    if mode == "constant" and not pad_is_tensor and len(pad) != 2 * (nd - 2):
        pairs = [(pad[2 * i], pad[2 * i + 1]) for i in range(len(pad) // 2)]
        if len(pad) == 2 * nd and pad_from_left_axis:
            pairs = pairs[::-1]  # pairs[0] belongs to axis 0; torch's list starts at the last axis
        tp = [v for pr in pairs for v in pr]
        return _wrap(F.pad(t, tp, "constant", value))
    channel_last = data_format in ("NHWC", "NLC", "NDHWC", "NWC")
    if channel_last:
        perm = [0, nd - 1] + list(range(1, nd - 1))
        t = t.permute(*perm)
    tm = {"constant": "constant", "reflect": "reflect", "replicate": "replicate", "circular": "circular"}[mode]
    out = F.pad(t, pad, tm, value) if tm == "constant" else F.pad(t, pad, tm)
    if channel_last:
        inv = [0] + list(range(2, nd)) + [1]
        out = out.permute(*inv)
    return _wrap(out)


def zeropad2d(x, padding, data_format="NCHW", name=None):
    return pad(x, padding, "constant", 0.0, data_format)


def interpolate(x, size=None, scale_factor=None, mode="nearest", align_corners=False, align_mode=0,
                data_format=None, name=None, recompute_scale_factor=None):
    t = T(x)
    nd = t.dim()
    if data_format is None:
        data_format = {3: "NCW", 4: "NCHW", 5: "NCDHW"}[nd]
    channel_last = data_format in ("NWC", "NHWC", "NDHWC")
    if channel_last:
        t = t.permute(0, nd - 1, *range(1, nd - 1))
    if isinstance(size, Tensor):
        size = size._t.tolist()
    if size is not None:
        size = [int(s._t.item()) if isinstance(s, Tensor) else int(s) for s in (size if isinstance(size, (list, tuple)) else [size])]
    if isinstance(scale_factor, Tensor):
        scale_factor = scale_factor._t.tolist()
    m = mode.lower()
    tm = {"nearest": "nearest", "bilinear": "bilinear", "trilinear": "trilinear", "bicubic": "bicubic",
          "linear": "linear", "area": "area"}[m]
    kw = {}
    if tm in ("bilinear", "trilinear", "bicubic", "linear"):
        kw["align_corners"] = align_corners
    out = F.interpolate(t, size=size, scale_factor=scale_factor, mode=tm, **kw)
    if channel_last:
        out = out.permute(0, *range(2, nd), 1)
    return _wrap(out)


upsample = interpolate


def embedding(x, weight, padding_idx=None, max_norm=None, norm_type=2.0, sparse=False, name=None):
    w = T(weight)
    idx = T(x)
    if padding_idx is not None and padding_idx < 0:
        padding_idx = w.shape[0] + padding_idx
    return _wrap(F.embedding(idx.long() if idx.dtype not in (torch.int64, torch.int32) else idx, w, padding_idx,
                             max_norm, norm_type, False, sparse))


def one_hot(x, num_classes, name=None):
    return _wrap(F.one_hot(T(x).long(), num_classes).float())


def label_smooth(label, prior_dist=None, epsilon=0.1, name=None):
    t = T(label)
    k = t.shape[-1]
    if prior_dist is not None:
        return _wrap((1 - epsilon) * t + epsilon * T(prior_dist))
    return _wrap((1 - epsilon) * t + epsilon / k)


def cosine_similarity(x1, x2, axis=1, eps=1e-8):
    return _wrap(F.cosine_similarity(T(x1), T(x2), axis, eps))


def bilinear(x1, x2, weight, bias=None, name=None):
    return _wrap(F.bilinear(T(x1), T(x2), T(weight), None if bias is None else T(bias).reshape(-1)))


def unfold(x, kernel_sizes, strides=1, paddings=0, dilations=1, name=None):
    if isinstance(paddings, (list, tuple)) and len(paddings) == 4:
        t = F.pad(T(x), [paddings[1], paddings[3], paddings[0], paddings[2]])
        return _wrap(F.unfold(t, kernel_sizes, dilations, 0, strides))
    return _wrap(F.unfold(T(x), kernel_sizes, dilations, paddings, strides))


def fold(x, output_sizes, kernel_sizes, strides=1, paddings=0, dilations=1, name=None):
    return _wrap(F.fold(T(x), output_sizes, kernel_sizes, dilations, paddings, strides))


def class_center_sample(label, num_classes, num_samples, group=None):
    t = T(label)
    pos = torch.unique(t)
    n_neg = max(num_samples - pos.numel(), 0)
    mask = torch.ones(num_classes, dtype=torch.bool, device=t.device)
    mask[pos] = False
    neg = torch.nonzero(mask).flatten()
    neg = neg[torch.randperm(neg.numel(), device=t.device)[:n_neg]]
    sampled = torch.sort(torch.cat([pos, neg])).values
    remap = torch.full((num_classes,), -1, dtype=torch.long, device=t.device)
    remap[sampled] = torch.arange(sampled.numel(), device=t.device)
    return _wrap(remap[t]), _wrap(sampled)


def sequence_mask(x, maxlen=None, dtype="int64", name=None):
    from ...framework import dtype as _dt
    t = T(x)
    ml = int(t.max().item()) if maxlen is None else int(maxlen)
    r = torch.arange(ml, device=t.device)
    return _wrap((r < t.unsqueeze(-1)).to(_dt.to_torch_dtype(dtype)))


def pixel_shuffle(x, upscale_factor, data_format="NCHW", name=None):
    t = T(x)
    if data_format == "NHWC":
        return _wrap(F.pixel_shuffle(t.permute(0, 3, 1, 2), upscale_factor).permute(0, 2, 3, 1))
    return _wrap(F.pixel_shuffle(t, upscale_factor))


def pixel_unshuffle(x, downscale_factor, data_format="NCHW", name=None):
    t = T(x)
    if data_format == "NHWC":
        return _wrap(F.pixel_unshuffle(t.permute(0, 3, 1, 2), downscale_factor).permute(0, 2, 3, 1))
    return _wrap(F.pixel_unshuffle(t, downscale_factor))


def channel_shuffle(x, groups, data_format="NCHW", name=None):
    t = T(x)
    if data_format == "NHWC":
        return _wrap(F.channel_shuffle(t.permute(0, 3, 1, 2), groups).permute(0, 2, 3, 1))
    return _wrap(F.channel_shuffle(t, groups))


def gather_tree(ids, parents):
    i, p = T(ids), T(parents)
    T_, B, W = i.shape
    out = torch.empty_like(i)
    out[-1] = i[-1]
    cur = torch.arange(W, device=i.device).expand(B, W).clone()
    cur = p[-1].gather(1, torch.arange(W, device=i.device).expand(B, W))
    for t in range(T_ - 2, -1, -1):
        out[t] = i[t].gather(1, cur)
        cur = p[t].gather(1, cur)
    return _wrap(out)


def temporal_shift(x, seg_num, shift_ratio=0.25, name=None, data_format="NCHW"):
    t = T(x)
    nt, c, h, w = t.shape
    n = nt // seg_num
    t = t.reshape(n, seg_num, c, h, w)
    fold_ = int(c * shift_ratio)
    out = torch.zeros_like(t)
    out[:, :-1, :fold_] = t[:, 1:, :fold_]
    out[:, 1:, fold_:2 * fold_] = t[:, :-1, fold_:2 * fold_]
    out[:, :, 2 * fold_:] = t[:, :, 2 * fold_:]
    return _wrap(out.reshape(nt, c, h, w))
