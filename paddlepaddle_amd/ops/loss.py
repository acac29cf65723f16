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
    lf = logits.reshape(-1, V).float()
    lb = labels.reshape(-1).long()
    loss = F.cross_entropy(lf, lb, ignore_index=ignore_index, reduction="none")
    return loss.view(logits.shape[:-1])
