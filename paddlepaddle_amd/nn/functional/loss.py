"""Loss functions. Reference: python/paddle/nn/functional/loss.py (cross_entropy at :2673).
Hard-label softmax cross-entropy runs on the fused HIP kernel (csrc/kernels/softmax.hip)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ...framework.tensor import Tensor, _wrap
from ...tensor._helpers import T
from ... import ops as _ops


def _reduce(l, reduction):
    if reduction == "mean":
        return l.mean()
    if reduction == "sum":
        return l.sum()
    return l


def _acc_dt(x):
    """Loss accumulation dtype: fp32 for 16-bit logits, float64 kept."""
    return torch.float64 if x.dtype == torch.float64 else torch.float32


def cross_entropy(input, label, weight=None, ignore_index=-100, reduction="mean", soft_label=False, axis=-1,
                  use_softmax=True, label_smoothing=0.0, name=None):
    x = T(input)
    y = T(label)
    nd = x.dim()
    ax = axis % nd
    if ax != nd - 1:
        x = x.movedim(ax, -1)
        if soft_label or y.dim() == nd:
            y = y.movedim(ax, -1)
    C = x.shape[-1]
    w = T(weight)
    if soft_label or (y.is_floating_point() and y.shape == x.shape):
        logp = F.log_softmax(x.to(_acc_dt(x)), -1) if use_softmax else torch.log(x.to(_acc_dt(x)))
        yt = y.to(_acc_dt(x))
        if label_smoothing:
            yt = yt * (1 - label_smoothing) + label_smoothing / C
        if w is not None:
            logp = logp * w.to(_acc_dt(x))
        l = -(yt * logp).sum(-1, keepdim=True)
        if reduction == "none":
            return _wrap(l)
        return _wrap(_reduce(l, reduction))
    squeeze_back = y.dim() == nd
    if squeeze_back:
        y = y.squeeze(-1)
    y = y.long()
    if use_softmax and w is None and label_smoothing == 0.0:
        l = _ops.softmax_cross_entropy(x, y, ignore_index)
        if reduction == "none":
            return _wrap(l.unsqueeze(-1) if squeeze_back else l)
        if reduction == "sum":
            return _wrap(l.sum())
        valid = (y != ignore_index).sum()
        return _wrap(l.sum() / valid.clamp_min(1).to(l.dtype))
    logp = F.log_softmax(x.to(_acc_dt(x)), -1) if use_softmax else torch.log(x.to(_acc_dt(x)))
    flat = logp.reshape(-1, C)
    yl = y.reshape(-1)
    l = F.nll_loss(flat, yl, weight=None if w is None else w.to(_acc_dt(x)), ignore_index=ignore_index,
                   reduction="none")
    if label_smoothing:
        smooth = -flat.mean(-1) if w is None else -(flat * w.to(_acc_dt(x))).sum(-1) / C
        l = (1 - label_smoothing) * l + label_smoothing * smooth * (yl != ignore_index)
    l = l.reshape(y.shape)
    if reduction == "none":
        return _wrap(l.unsqueeze(-1) if squeeze_back else l)
    if reduction == "sum":
        return _wrap(l.sum())
    if w is not None:
        wsum = (w.to(_acc_dt(x))[yl.clamp_min(0)] * (yl != ignore_index)).sum()
        return _wrap(l.sum() / wsum)
    return _wrap(l.sum() / (yl != ignore_index).sum().clamp_min(1))


def softmax_with_cross_entropy(logits, label, soft_label=False, ignore_index=-100, numeric_stable_mode=True,
                               return_softmax=False, axis=-1):
    loss = cross_entropy(logits, label, soft_label=soft_label, ignore_index=ignore_index, reduction="none",
                         axis=axis)
    lt = T(label)
    if not soft_label and lt.dim() < T(logits).dim():
        loss = _wrap(loss._t.unsqueeze(axis))
    if return_softmax:
        return loss, _wrap(F.softmax(T(logits).float(), axis).to(T(logits).dtype))
    return loss


def mse_loss(input, label, reduction="mean", name=None):
    return _wrap(F.mse_loss(T(input), T(label), reduction=reduction))


def square_error_cost(input, label):
    return _wrap((T(input) - T(label)) ** 2)


def l1_loss(input, label, reduction="mean", name=None):
    return _wrap(F.l1_loss(T(input), T(label), reduction=reduction))


def nll_loss(input, label, weight=None, ignore_index=-100, reduction="mean", name=None):
    return _wrap(F.nll_loss(T(input), T(label).long(), T(weight), ignore_index=ignore_index, reduction=reduction))


def binary_cross_entropy(input, label, weight=None, reduction="mean", name=None):
    return _wrap(F.binary_cross_entropy(T(input), T(label), T(weight), reduction=reduction))


def binary_cross_entropy_with_logits(logit, label, weight=None, reduction="mean", pos_weight=None, name=None):
    return _wrap(F.binary_cross_entropy_with_logits(T(logit), T(label), T(weight), reduction=reduction,
                                                    pos_weight=T(pos_weight)))


def kl_div(input, label, reduction="mean", log_target=False, name=None):
    r = "batchmean" if reduction == "batchmean" else reduction
    return _wrap(F.kl_div(T(input), T(label), reduction=r, log_target=log_target))


def smooth_l1_loss(input, label, reduction="mean", delta=1.0, name=None):
    return _wrap(F.huber_loss(T(input), T(label), reduction=reduction, delta=delta))


def huber_loss(input, label, reduction="mean", delta=1.0, name=None):
    return _wrap(F.huber_loss(T(input), T(label), reduction=reduction, delta=delta))


def margin_ranking_loss(input, other, label, margin=0.0, reduction="mean", name=None):
    return _wrap(F.margin_ranking_loss(T(input), T(other), T(label), margin, reduction=reduction))


def hinge_embedding_loss(input, label, margin=1.0, reduction="mean", name=None):
    return _wrap(F.hinge_embedding_loss(T(input), T(label), margin, reduction=reduction))


def cosine_embedding_loss(input1, input2, label, margin=0, reduction="mean", name=None):
    return _wrap(F.cosine_embedding_loss(T(input1), T(input2), T(label), margin, reduction=reduction))


def triplet_margin_loss(input, positive, negative, margin=1.0, p=2.0, epsilon=1e-6, swap=False,
                        reduction="mean", name=None):
    return _wrap(F.triplet_margin_loss(T(input), T(positive), T(negative), margin, p, epsilon, swap,
                                       reduction=reduction))


def triplet_margin_with_distance_loss(input, positive, negative, distance_function=None, margin=1.0, swap=False,
                                      reduction="mean", name=None):
    df = None
    if distance_function is not None:
        def df(a, b):
            return T(distance_function(_wrap(a), _wrap(b)))
    return _wrap(F.triplet_margin_with_distance_loss(T(input), T(positive), T(negative), distance_function=df,
                                                     margin=margin, swap=swap, reduction=reduction))


def multi_label_soft_margin_loss(input, label, weight=None, reduction="mean", name=None):
    return _wrap(F.multilabel_soft_margin_loss(T(input), T(label), T(weight), reduction=reduction))


def multi_margin_loss(input, label, p=1, margin=1.0, weight=None, reduction="mean", name=None):
    return _wrap(F.multi_margin_loss(T(input), T(label).long(), p, margin, T(weight), reduction=reduction))


def soft_margin_loss(input, label, reduction="mean", name=None):
    return _wrap(F.soft_margin_loss(T(input), T(label), reduction=reduction))


def poisson_nll_loss(input, label, log_input=True, full=False, epsilon=1e-8, reduction="mean", name=None):
    return _wrap(F.poisson_nll_loss(T(input), T(label), log_input, full, eps=epsilon, reduction=reduction))


def gaussian_nll_loss(input, label, variance, full=False, epsilon=1e-6, reduction="mean", name=None):
    return _wrap(F.gaussian_nll_loss(T(input), T(label), T(variance), full, epsilon, reduction))


def sigmoid_focal_loss(logit, label, normalizer=None, alpha=0.25, gamma=2.0, reduction="sum", name=None):
    x, y = T(logit), T(label)
    p = torch.sigmoid(x)
    ce = F.binary_cross_entropy_with_logits(x, y, reduction="none")
    pt = p * y + (1 - p) * (1 - y)
    l = ce * (1 - pt) ** gamma
    if alpha >= 0:
        l = (alpha * y + (1 - alpha) * (1 - y)) * l
    if normalizer is not None:
        l = l / T(normalizer)
    return _wrap(_reduce(l, reduction))


def dice_loss(input, label, epsilon=0.00001, name=None):
    x, y = T(input), T(label)
    y1 = F.one_hot(y.squeeze(-1).long(), x.shape[-1]).to(x.dtype)
    red = tuple(range(1, x.dim()))
    inter = (x * y1).sum(red)
    union = x.sum(red) + y1.sum(red)
    return _wrap((1 - (2 * inter) / (union + epsilon)).mean())


def log_loss(input, label, epsilon=1e-4, name=None):
    x, y = T(input), T(label)
    return _wrap(-y * torch.log(x + epsilon) - (1 - y) * torch.log(1 - x + epsilon))


def npair_loss(anchor, positive, labels, l2_reg=0.002):
    a, p, lb = T(anchor), T(positive), T(labels).reshape(-1, 1).float()
    reg = l2_reg * ((a ** 2).sum(1).mean() + (p ** 2).sum(1).mean()) * 0.25
    sim = a @ p.T
    tgt = (lb == lb.T).float()
    tgt = tgt / tgt.sum(1, keepdim=True)
    ce = (-tgt * F.log_softmax(sim, 1)).sum(1).mean()
    return _wrap(ce + reg)


def ctc_loss(log_probs, labels, input_lengths, label_lengths, blank=0, reduction="mean", norm_by_times=False):
    lp = T(log_probs)
    l = F.ctc_loss(F.log_softmax(lp.float(), -1), T(labels).long(), T(input_lengths).long(),
                   T(label_lengths).long(), blank, reduction="none", zero_infinity=False)
    if reduction == "mean":
        return _wrap((l / T(label_lengths).float().clamp_min(1)).mean())
    return _wrap(_reduce(l, reduction))


def margin_cross_entropy(logits, label, margin1=1.0, margin2=0.5, margin3=0.0, scale=64.0, group=None,
                         return_softmax=False, reduction="mean"):
    x = T(logits).float()
    y = T(label).reshape(-1).long()
    theta = torch.acos(x.clamp(-1 + 1e-7, 1 - 1e-7))
    tgt = torch.cos(margin1 * theta + margin2) - margin3
    onehot = F.one_hot(y, x.shape[-1]).bool()
    x2 = torch.where(onehot, tgt, x) * scale
    l = F.cross_entropy(x2, y, reduction="none").unsqueeze(-1)
    out = _wrap(_reduce(l, reduction))
    if return_softmax:
        return out, _wrap(F.softmax(x2, -1))
    return out


def rnnt_loss(input, label, input_lengths, label_lengths, blank=0, fastemit_lambda=0.001, reduction="mean",
              name=None):
    from .extension import rnnt_loss as _rnnt
    return _rnnt(input, label, input_lengths, label_lengths, blank, fastemit_lambda, reduction, name)


def edit_distance(input, label, normalized=True, ignored_tokens=None, input_length=None, label_length=None,
                  name=None):
    """Levenshtein distance between each pair of int64 sequences. Returns (sequence_num [1] int64,
    distances [B, 1] float32) in the order phi's edit_distance kernel writes them (the reference docstring
    prints them under swapped names). ``normalized`` divides by the label length.
    Reference: python/paddle/nn/functional/loss.py edit_distance, phi/kernels/cpu/edit_distance_kernel.cc."""
    import numpy as _np
    if ignored_tokens:
        raise ValueError(f"Expected ignored_tokens is None (got {ignored_tokens})")
    a = T(input).detach().cpu().numpy()
    b = T(label).detach().cpu().numpy()
    B = a.shape[0]
    la = T(input_length).cpu().numpy().reshape(-1) if input_length is not None else _np.full(B, a.shape[1])
    lb = T(label_length).cpu().numpy().reshape(-1) if label_length is not None else _np.full(B, b.shape[1])
    out = _np.zeros((B, 1), dtype=_np.float32)
    for i in range(B):
        x, y = a[i, :int(la[i])], b[i, :int(lb[i])]
        m, n = len(x), len(y)
        prev = _np.arange(n + 1, dtype=_np.int64)
        for r in range(1, m + 1):
            cur = _np.empty(n + 1, dtype=_np.int64)
            cur[0] = r
            for c in range(1, n + 1):
                cur[c] = min(prev[c] + 1, cur[c - 1] + 1, prev[c - 1] + (x[r - 1] != y[c - 1]))
            prev = cur
        d = float(prev[n])
        out[i, 0] = d / n if normalized and n > 0 else d
    dev = T(input).device
    return (_wrap(torch.tensor([B], dtype=torch.int64, device=dev)), _wrap(torch.from_numpy(out).to(dev)))


def adaptive_log_softmax_with_loss(input, label, head_weight, tail_weights, cutoffs, head_bias=None, name=None):
    """Adaptive softmax (Grave et al.; reference nn/functional/loss.py:4461): the head scores the shortlist
    [0, cutoffs[0]) plus one logit per tail cluster; a target in cluster i ([cutoffs[i-1], cutoffs[i])) scores
    head_logprob[shortlist + i - 1] + log_softmax((x @ proj_i) @ out_i)[target - cutoffs[i-1]].
    ``cutoffs`` ends with the class count. Returns (per-sample target log-probabilities, mean NLL)."""
    x, y = T(input), T(label)
    if y.dim() > 1:
        raise ValueError("0D or 1D label tensor expected, multi-label not supported")
    batched = y.dim() == 1
    if batched and (x.dim() != 2 or x.shape[0] != y.shape[0]):
        raise ValueError("1D label tensor expects 2D input tensors with the same batch size")
    if not batched:
        if x.dim() != 1:
            raise ValueError("0D label tensor expects 1D input tensors")
        x, y = x.unsqueeze(0), y.unsqueeze(0)
    y = y.long()
    cut = [int(T(c).item()) if isinstance(c, (Tensor, torch.Tensor)) else int(c) for c in cutoffs]
    short = cut[0]
    head = x @ T(head_weight)
    if head_bias is not None:
        head = head + T(head_bias)
    head_lp = head.float().log_softmax(-1).to(x.dtype)
    out = torch.zeros(y.shape[0], dtype=x.dtype, device=x.device)
    m0 = y < short
    if bool(m0.any()):
        rows = m0.nonzero().squeeze(1)
        out = out.index_put((rows,), head_lp[rows].gather(1, y[rows].unsqueeze(1)).squeeze(1))
    for i in range(1, len(cut)):
        lo, hi = cut[i - 1], cut[i]
        m = (y >= lo) & (y < hi)
        if not bool(m.any()):
            continue
        rows = m.nonzero().squeeze(1)
        proj, o = tail_weights[i - 1]
        tail = ((x[rows] @ T(proj)) @ T(o)).float().log_softmax(-1).to(x.dtype)
        val = head_lp[rows, short + i - 1] + tail.gather(1, (y[rows] - lo).unsqueeze(1)).squeeze(1)
        out = out.index_put((rows,), val)
    if bool(((y < 0) | (y >= cut[-1])).any()):
        raise ValueError(f"target values should be in [0, {cut[-1] - 1}]")
    loss = (-out).mean()
    return _wrap(out if batched else out.squeeze(0)), _wrap(loss)
