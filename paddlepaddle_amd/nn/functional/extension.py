"""Less common nn.functional ops: fractional max pooling, hierarchical sigmoid, RNN-T loss, adaptive
log-softmax, block-sparse / flashmask attention, packed varlen attention.

References: python/paddle/nn/functional/pooling.py (fractional_max_pool2d/3d; index math in
paddle/phi/kernels/funcs/pooling.h FractionalStartIndex/EndIndex/RationalU), loss.py (hsigmoid_loss,
rnnt_loss, adaptive_log_softmax_with_loss; tree code in phi/kernels/funcs/matrix_bit_code.h),
sparse_attention.py, flash_attention.py (flashmask_attention, flash_attn_varlen_qkvpacked).
These run as ATen compositions on the HIP device (not hot paths of the benchmarked models); the
attention variants build their mask once and go through the same SDPA/flash entry point.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ...framework.tensor import _wrap
from ...tensor._helpers import T
from ... import ops as _ops

__all__ = ["fractional_max_pool2d", "fractional_max_pool3d", "hsigmoid_loss", "rnnt_loss",
           "adaptive_log_softmax_with_loss", "sparse_attention", "flashmask_attention",
           "flash_attn_varlen_qkvpacked"]


# ----------------------------------------------------------------------------------- fractional pool
def _frac_u(u, alpha, n_in, n_out, pool):
    if pool > 0:
        return u
    base = n_in // n_out
    u_max1 = (base + 2) / alpha - 1
    u_max2 = (n_in + 1 - base) / alpha - (n_out - 1)
    return u * min(u_max1, u_max2)


def _frac_windows(n_in, n_out, pool, u, device):
    alpha = (n_in - pool) / (n_out - (1 if pool > 0 else 0))
    uu = _frac_u(u, alpha, n_in, n_out, pool)
    starts, ends = [], []
    for i in range(n_out):
        s = int((i + uu) * alpha) - int(uu * alpha)
        e = (s + pool) if pool > 0 else int((i + 1 + uu) * alpha) - int(uu * alpha)
        starts.append(max(s, 0))
        ends.append(min(e, n_in))
    L = max(e - s for s, e in zip(starts, ends))
    idx = torch.tensor([[min(s + j, e - 1) for j in range(L)] for s, e in zip(starts, ends)], device=device)
    return idx  # [n_out, L] (windows padded by repeating their last element)


def _fractional(x, output_size, kernel_size, random_u, return_mask, nd):
    t = T(x)
    sp = list(t.shape[2:])
    if isinstance(output_size, int):
        output_size = [output_size] * nd
    output_size = [sp[i] if o is None else int(o) for i, o in enumerate(output_size)]
    if kernel_size is None:
        ks = [0] * nd
    else:
        ks = [kernel_size] * nd if isinstance(kernel_size, int) else list(kernel_size)
    u = float(random_u) if random_u is not None else float(torch.rand(()).item())
    idxs = [_frac_windows(sp[i], output_size[i], ks[i], u, t.device) for i in range(nd)]
    # gather each spatial dim's windows: [..., O_i, L_i] per dim, then reduce over all L_i jointly
    g = t
    for d in range(nd):
        ax = 2 + 2 * d
        o, L = idxs[d].shape
        g = g.index_select(ax, idxs[d].reshape(-1))
        g = g.reshape(*g.shape[:ax], o, L, *g.shape[ax + 1:])
    # g: [N, C, O0, L0, O1, L1, (O2, L2)]
    perm = [0, 1] + [2 + 2 * d for d in range(nd)] + [3 + 2 * d for d in range(nd)]
    g = g.permute(*perm)
    flat = g.reshape(*g.shape[:2 + nd], -1)
    val, arg = flat.max(-1)
    if not return_mask:
        return _wrap(val)
    # flat input index of the argmax
    Ls = [i.shape[1] for i in idxs]
    rem = arg
    coords = []
    for d in reversed(range(nd)):
        coords.append(rem % Ls[d])
        rem = rem // Ls[d]
    coords = coords[::-1]
    flat_idx = torch.zeros_like(arg)
    for d in range(nd):
        shape = [1] * (2 + nd)
        shape[2 + d] = output_size[d]
        win = idxs[d]  # [O_d, L_d]
        o_idx = torch.arange(output_size[d], device=t.device).view(*shape).expand_as(arg)
        pos = win[o_idx, coords[d]]
        flat_idx = flat_idx * sp[d] + pos
    return _wrap(val), _wrap(flat_idx.to(torch.int64))


def fractional_max_pool2d(x, output_size, kernel_size=None, random_u=None, return_mask=False, name=None):
    return _fractional(x, output_size, kernel_size, random_u, return_mask, 2)


def fractional_max_pool3d(x, output_size, kernel_size=None, random_u=None, return_mask=False, name=None):
    return _fractional(x, output_size, kernel_size, random_u, return_mask, 3)


# ----------------------------------------------------------------------------------- hsigmoid
def _default_codes(label, num_classes):
    """(node index [B, L], bit [B, L], valid [B, L]) of the default complete-binary-tree code."""
    c = label.to(torch.int64).reshape(-1) + num_classes
    L = int(num_classes - 1).bit_length()
    j = torch.arange(L, device=c.device)
    length = torch.floor(torch.log2(c.double())).to(torch.int64)  # FindLastSet(c) - 1
    idx = (c.unsqueeze(1) >> (j + 1)) - 1
    bit = ((c.unsqueeze(1) >> j) & 1).bool()
    valid = j.unsqueeze(0) < length.unsqueeze(1)
    return idx.clamp_min(0), bit, valid


def hsigmoid_loss(input, label, num_classes, weight, bias=None, path_table=None, path_code=None, is_sparse=False,
                  name=None):
    """Hierarchical sigmoid loss [B, 1]; same padding convention as the reference kernel (positions past a
    code's length contribute log 2)."""
    x, w = T(input), T(weight)
    b = T(bias)
    if path_table is None:
        idx, bit, valid = _default_codes(T(label), num_classes)
    else:
        pt, pc = T(path_table).to(torch.int64), T(path_code).to(torch.int64)
        valid = torch.cumprod((pt >= 0).to(torch.int64), 1).bool()
        idx, bit = pt.clamp_min(0), pc.bool()
    pre = torch.einsum("bd,bld->bl", x, w[idx])
    if b is not None:
        pre = pre + b.reshape(-1)[idx]
    pre = torch.where(valid, pre, torch.zeros_like(pre)).clamp(-40.0, 40.0)
    loss = F.softplus(pre).sum(1) - (pre * (bit & valid)).sum(1)
    return _wrap(loss.unsqueeze(1))


# ----------------------------------------------------------------------------------- RNN-T
def rnnt_loss(input, label, input_lengths, label_lengths, blank=0, fastemit_lambda=0.001, reduction="mean",
              name=None):
    """RNN transducer loss. Reference: python/paddle/nn/functional/loss.py rnnt_loss: ``input`` [B, T, U+1, V]
    holds LOG-PROBABILITIES (the docstring's contract; its example, -2.85042444, is computed on them as given).
    The forward variable alpha[t, u] is a log-space recursion; FastEmit scales the gradient of the
    label-emission terms by (1 + lambda) and leaves the loss value unchanged. Output dtype = input dtype."""
    logits = T(input)
    if not logits.is_floating_point():
        logits = logits.float()
    lab = T(label).to(torch.int64)
    tl = T(input_lengths).to(torch.int64)
    ul = T(label_lengths).to(torch.int64)
    B, Tm, U1, V = logits.shape
    lp = logits
    blank_lp = lp[..., blank]                                        # [B, T, U+1]
    lab_pad = torch.cat([lab, torch.zeros(B, 1, dtype=torch.int64, device=lab.device)], 1)[:, :U1]
    emit_lp = lp.gather(3, lab_pad.view(B, 1, U1, 1).expand(B, Tm, U1, 1)).squeeze(3)  # [B, T, U+1]
    if fastemit_lambda:
        emit_lp = emit_lp * (1.0 + fastemit_lambda) - fastemit_lambda * emit_lp.detach()
    alpha = [[None] * U1 for _ in range(Tm)]
    for t in range(Tm):
        for u in range(U1):
            if t == 0 and u == 0:
                alpha[t][u] = torch.zeros(B, device=lp.device, dtype=lp.dtype)
                continue
            cands = []
            if t > 0:
                cands.append(alpha[t - 1][u] + blank_lp[:, t - 1, u])
            if u > 0:
                cands.append(alpha[t][u - 1] + emit_lp[:, t, u - 1])
            alpha[t][u] = torch.logsumexp(torch.stack(cands), 0) if len(cands) > 1 else cands[0]
    A = torch.stack([torch.stack(r, 1) for r in alpha], 1)           # [B, T, U+1]
    bi = torch.arange(B, device=lp.device)
    tt, uu = (tl - 1).clamp_min(0), ul
    ll = A[bi, tt, uu] + blank_lp[bi, tt, uu]
    loss = -ll
    loss = torch.where(tl > 0, loss, torch.zeros_like(loss))
    if reduction == "mean":
        loss = loss.sum() / B
    elif reduction == "sum":
        loss = loss.sum()
    return _wrap(loss)


# ----------------------------------------------------------------------------------- adaptive softmax
def adaptive_log_softmax_with_loss(input, label, head_weight, tail_weights, cutoffs, head_bias=None, name=None):
    """(output, loss): log-probability of the target class per row and the mean NLL (nn/functional/loss.py)."""
    from .loss import adaptive_log_softmax_with_loss as _alsm
    return _alsm(input, label, head_weight, tail_weights, cutoffs, head_bias, name)


# ----------------------------------------------------------------------------------- attention variants
def sparse_attention(query, key, value, sparse_csr_offset, sparse_csr_columns, key_padding_mask=None,
                     attn_mask=None, name=None):
    """Attention restricted to a per-(batch, head) CSR pattern. q/k/v: [B, H, S, D]; offsets [B, H, S+1],
    columns [B, H, nnz]. key_padding_mask [B, S] / attn_mask [S, S]: 0 = masked (reference semantics)."""
    q, k, v = T(query), T(key), T(value)
    off, col = T(sparse_csr_offset).to(torch.int64), T(sparse_csr_columns).to(torch.int64)
    B, H, S, D = q.shape
    allowed = torch.zeros(B, H, S, S, dtype=torch.bool, device=q.device)
    nnz = col.shape[-1]
    pos = torch.arange(nnz, device=q.device).view(1, 1, 1, nnz)
    row = (pos >= off[..., :-1].unsqueeze(-1)) & (pos < off[..., 1:].unsqueeze(-1))     # [B, H, S, nnz]
    rows_of = row.float().argmax(2)                                                      # [B, H, nnz]
    valid = row.any(2)
    bi = torch.arange(B, device=q.device).view(B, 1, 1).expand(B, H, nnz)
    hi = torch.arange(H, device=q.device).view(1, H, 1).expand(B, H, nnz)
    allowed[bi[valid], hi[valid], rows_of[valid], col[valid]] = True
    if key_padding_mask is not None:
        allowed &= (T(key_padding_mask) != 0).view(B, 1, 1, S)
    if attn_mask is not None:
        allowed &= (T(attn_mask) != 0).view(1, 1, S, S)
    s = (q @ k.transpose(-1, -2)) / math.sqrt(D)
    s = s.masked_fill(~allowed, float("-inf"))
    p = torch.softmax(s.float(), -1).nan_to_num(0.0).to(q.dtype)
    return _wrap(p @ v)


def flashmask_attention(*args, **kwargs):
    """Reference: python/paddle/nn/functional/flash_attention.py:1306; in-kernel row bounds (see
    nn/functional/flash_attention.py)."""
    from .flash_attention import flashmask_attention as _fm
    return _fm(*args, **kwargs)


def flash_attn_varlen_qkvpacked(*args, **kwargs):
    """Reference: python/paddle/nn/functional/flash_attention.py:961 (one varlen launch)."""
    from .flash_attention import flash_attn_varlen_qkvpacked as _f
    return _f(*args, **kwargs)