"""Linear layers with fused epilogues.

Reference: paddle/phi/kernels/fusion/gpu/fused_gemm_epilogue_kernel.cu,
python/paddle/incubate/nn/functional/fused_matmul_bias.py.
paddle's Linear weight is [in_features, out_features]: y = x @ W + b.
The GEMM itself runs on hipBLASLt (plain library GEMM, bias folded into the GEMM as beta·C);
the activation epilogue (bias+GELU) is a fused HIP pass (csrc/kernels/act.hip). A hand-written
MFMA GEMM (csrc/kernels/gemm.hip) is used when it beats the library on a shape (see ops/gemm.py).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .activation import bias_gelu, gelu


def fused_linear(x, w, b=None, act=None):
    if act is None:
        if b is None:
            return torch.matmul(x, w)
        if x.dim() == 2:
            return torch.addmm(b, x, w)
        return torch.addmm(b, x.reshape(-1, x.shape[-1]), w).view(*x.shape[:-1], w.shape[-1])
    if act in ("gelu", "gelu_tanh", "gelu_approximate"):
        h = torch.matmul(x, w)
        if b is not None:
            return bias_gelu(h, b)
        return gelu(h, approximate=True)
    if act == "gelu_erf":
        h = torch.matmul(x, w) if b is None else fused_linear(x, w, b)
        return gelu(h, approximate=False)
    if act == "relu":
        h = fused_linear(x, w, b)
        return F.relu(h)
    raise ValueError(f"unsupported activation {act}")
