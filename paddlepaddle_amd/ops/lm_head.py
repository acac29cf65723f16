"""LM head + cross-entropy without materialising the [tokens, vocab] logits.

The vocabulary is cut into a few slices. Forward: per slice, one GEMM gives the slice's logits, the
slice CE kernel (csrc/kernels/softmax.hip ce_slice_fwd) reduces them to a per-token logsumexp and label
logit, and the slice's logits are dropped; the slice statistics merge into the global logsumexp.
Backward recomputes each slice's logits, turns them into dlogits in place (ce_slice_bwd:
softmax - onehot, scaled by the incoming per-token gradient), then dX += dlogits . W_slice and
dW_slice = dlogits^T . X, written straight into the slice's rows of dW. Peak extra memory is one
slice of logits instead of the whole [T, V] logits and their gradient; the price is the recomputed
forward GEMM. All three GEMM kinds go through the per-shape choice of ops/linear.py (hand-written
MFMA GEMM or hipBLASLt).

Reference: the reference materialises logits (python/paddle/nn/functional/loss.py cross_entropy over
the LM head output); the per-slice statistics are the ones its vocab-parallel
c_softmax_with_cross_entropy exchanges between ranks."""
from __future__ import annotations

import torch

from .linear import _nt_fwd, _nt_dgrad, _nt_wgrad
from .loss import ce_slice_stats, ce_slice_grad


def _slices(V, n):
    step = -(-V // n)
    step = -(-step // 256) * 256
    return [(v0, min(V, v0 + step)) for v0 in range(0, V, step)]


class _LMHeadCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, w, labels, ignore_index, n_slices):
        T, V = h.shape[0], w.shape[0]
        lab = labels.reshape(-1).to(torch.int64).contiguous()
        parts = _slices(V, n_slices)
        lses = torch.empty(len(parts), T, dtype=torch.float32, device=h.device)
        tgt = torch.zeros(T, dtype=torch.float32, device=h.device)
        for i, (v0, v1) in enumerate(parts):
            logits = _nt_fwd(h, w[v0:v1])
            lse_s, tgt_s = ce_slice_stats(logits, lab, v0)
            lses[i] = lse_s
            tgt += tgt_s
            del logits
        lse = torch.logsumexp(lses, 0)
        loss = (lse - tgt).masked_fill(lab == ignore_index, 0.0)
        ctx.save_for_backward(h, w, lab, lse)
        ctx.ignore_index, ctx.parts = ignore_index, parts
        return loss

    @staticmethod
    def backward(ctx, dloss):
        h, w, lab, lse = ctx.saved_tensors
        dl = dloss.reshape(-1).float().contiguous()
        dh = None
        dw = torch.empty_like(w) if ctx.needs_input_grad[1] else None
        for v0, v1 in ctx.parts:
            ws = w[v0:v1]
            dlog = _nt_fwd(h, ws)  # recomputed slice logits, turned into their gradient in place
            ce_slice_grad(dlog, lab, v0, lse, dl, ctx.ignore_index, out=dlog)
            if ctx.needs_input_grad[0]:
                part = _nt_dgrad(dlog, ws)
                dh = part if dh is None else dh.add_(part)
            if dw is not None:
                dw[v0:v1] = _nt_wgrad(dlog, h)
            del dlog
        return dh, dw, None, None, None


def lm_head_cross_entropy(h, w, labels, ignore_index=-100, n_slices=4):
    """Per-token loss (fp32) of softmax(h @ w.T) against labels; h [..., H], w [V, H] (tied embedding
    layout), labels [...]. Same values and gradients as cross_entropy(linear_nt(h, w), labels)."""
    shape = h.shape[:-1]
    h2 = h.reshape(-1, h.shape[-1])
    if not h2.is_contiguous():
        h2 = h2.contiguous()
    if h2.dtype != w.dtype:
        h2 = h2.to(w.dtype)
    return _LMHeadCE.apply(h2, w, labels, int(ignore_index), int(n_slices)).view(shape)
