"""AMP global state shared by ops. Reference: paddle/fluid/eager/amp_auto_cast.h,
python/paddle/amp/amp_lists.py (white/black lists)."""
from __future__ import annotations

import torch

# ops that run in low precision under O1 (MFMA-bound ops)
WHITE_LIST = {
    "matmul", "matmul_v2", "mm", "bmm", "linear", "fused_linear", "conv2d", "conv1d", "conv3d",
    "conv2d_transpose", "einsum", "addmm", "flash_attention", "scaled_dot_product_attention",
    "fused_gemm_epilogue", "mv", "baddbmm",
}
# ops kept in fp32 under O1 and O2 (numerically sensitive)
BLACK_LIST = {
    "exp", "square", "log", "mean", "sum", "cos_sim", "softmax", "softmax_with_cross_entropy",
    "sigmoid_cross_entropy_with_logits", "c_softmax_with_cross_entropy", "cross_entropy",
    "cross_entropy2", "log_softmax", "pow", "reduce_sum", "norm", "cumsum", "logsumexp",
    "binary_cross_entropy", "mse_loss", "nll_loss", "kl_div", "smooth_l1_loss",
}


class _AmpState:
    __slots__ = ("enabled", "level", "dtype", "white", "black")

    def __init__(self):
        self.enabled = False
        self.level = "O0"
        self.dtype = torch.float16
        self.white = set(WHITE_LIST)
        self.black = set(BLACK_LIST)


STATE = _AmpState()


def cast_tensor_raw(t, dtype):
    return t.to(dtype)


def amp_dtype_for(op_name):
    """Return the torch dtype inputs of ``op_name`` must be cast to, or None."""
    s = STATE
    if not s.enabled:
        return None
    if op_name in s.black:
        return torch.float32
    if s.level == "O2":
        return s.dtype
    if op_name in s.white:
        return s.dtype
    return None


def maybe_cast(op_name, *ts):
    """Cast floating torch tensors for an AMP-aware op. Returns the (possibly) cast tuple."""
    d = amp_dtype_for(op_name)
    if d is None:
        return ts
    out = []
    for t in ts:
        if isinstance(t, torch.Tensor) and t.is_floating_point() and t.dtype != d:
            t = t.to(d)
        out.append(t)
    return tuple(out)
