"""Fused softmax + cross-entropy over large vocabularies (HIP).

Reference: paddle/phi/kernels/gpu/cross_entropy_kernel.cu (softmax_with_cross_entropy),
c_softmax_with_cross_entropy for the vocab-parallel case.
Kernel: csrc/kernels/softmax.hip — one workgroup per row, online max/sum in one pass over the
row (bf16 logits are never up-cast to a materialised fp32 copy), backward writes
softmax - onehot scaled by the incoming per-row gradient.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _loader as L
from ..framework.trace_hook import static_op


class _SoftmaxCEHIP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        V = logits.shape[-1]
        lg = logits.contiguous().view(-1, V)
        lb = labels.contiguous().view(-1).to(torch.int64)
        rows = lg.shape[0]
        loss = torch.empty(rows, dtype=torch.float32, device=lg.device)
        lse = torch.empty(rows, dtype=torch.float32, device=lg.device)
        L.call("pa_softmax_ce_fwd", L.ptr(lg), L.ptr(lb), L.ptr(loss), L.ptr(lse), rows, V, int(ignore_index),
               L.dcode(lg), L.stream_ptr())
        ctx.save_for_backward(lg, lb, lse)
        ctx.ignore_index = ignore_index
        ctx.shape = logits.shape
        return loss.view(logits.shape[:-1])

    @staticmethod
    def backward(ctx, dloss):
        lg, lb, lse = ctx.saved_tensors
        rows, V = lg.shape
        dl = dloss.contiguous().view(-1).float()
        dlogits = torch.empty_like(lg)
        L.call("pa_softmax_ce_bwd", L.ptr(lg), L.ptr(lb), L.ptr(lse), L.ptr(dl), L.ptr(dlogits), rows, V,
               int(ctx.ignore_index), L.dcode(lg), L.stream_ptr())
        return dlogits.view(ctx.shape), None, None


@static_op
def softmax_cross_entropy(logits, labels, ignore_index=-100):
    """Per-row loss (fp32) = logsumexp(logits) - logits[label]; 0 where label == ignore_index."""
    if L.hip_enabled_for(logits) and logits.dtype in L._DT and logits.shape[-1] % 8 == 0:
        return _SoftmaxCEHIP.apply(logits, labels, ignore_index)
    V = logits.shape[-1]
    lf = logits.reshape(-1, V)
    lf = lf.float() if lf.dtype in (torch.float16, torch.bfloat16) else lf  # float64 stays float64
    lb = labels.reshape(-1).long()
    loss = F.cross_entropy(lf, lb, ignore_index=ignore_index, reduction="none")
    return loss.view(logits.shape[:-1])


# ---------------------------------------------------------------------------------------------
# Cross entropy over a vocabulary slice [v0, v0 + V) (vocab-parallel CE, vocab-chunked LM head):
# per-row logsumexp and label logit of the slice; the gradient with the global logsumexp.
def ce_slice_stats(logits2d, labels1d, v0):
    """(lse [rows] fp32, label logit [rows] fp32, 0 when the label is outside the slice)."""
    rows, V = logits2d.shape
    if L.hip_enabled_for(logits2d) and logits2d.dtype in L._DT and V % 8 == 0 and logits2d.is_contiguous():
        lse = torch.empty(rows, dtype=torch.float32, device=logits2d.device)
        tgt = torch.empty(rows, dtype=torch.float32, device=logits2d.device)
        L.call("pa_ce_slice_fwd", L.ptr(logits2d), L.ptr(labels1d), L.ptr(lse), L.ptr(tgt), rows, V, int(v0),
               L.dcode(logits2d), L.stream_ptr())
        return lse, tgt
    lf = logits2d.float()
    local = labels1d - v0
    inr = (local >= 0) & (local < V)
    tgt = torch.where(inr, lf.gather(-1, local.clamp(0, V - 1).unsqueeze(-1)).squeeze(-1), torch.zeros_like(lf[:, 0]))
    return torch.logsumexp(lf, -1), tgt


def ce_slice_grad(logits2d, labels1d, v0, lse, dloss, ignore_index, out=None):
    """(softmax(x; lse) - onehot) * dloss for the slice; ``out`` may alias ``logits2d`` (in place)."""
    rows, V = logits2d.shape
    if out is None:
        out = torch.empty_like(logits2d)
    if L.hip_enabled_for(logits2d) and logits2d.dtype in L._DT and V % 8 == 0 and logits2d.is_contiguous() \
            and out.is_contiguous():
        L.call("pa_ce_slice_bwd", L.ptr(logits2d), L.ptr(labels1d), L.ptr(lse), L.ptr(dloss.float().contiguous()),
               L.ptr(out), rows, V, int(v0), int(ignore_index), L.dcode(logits2d), L.stream_ptr())
        return out
    p = torch.exp(logits2d.float() - lse.unsqueeze(-1))
    local = labels1d - v0
    inr = (local >= 0) & (local < V)
    p.scatter_add_(-1, local.clamp(0, V - 1).unsqueeze(-1), -inr.float().unsqueeze(-1))
    g = dloss.float().masked_fill(labels1d == ignore_index, 0.0)
    out.copy_(p * g.unsqueeze(-1))
    return out
