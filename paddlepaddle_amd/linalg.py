"""paddle.linalg. Reference: python/paddle/linalg.py."""
from .tensor.linalg import *  # noqa: F401,F403
from .tensor.linalg import norm, vector_norm, matrix_norm, cond, det, slogdet, matrix_rank, matrix_power, \
    matrix_exp, cholesky, cholesky_solve, cholesky_inverse, qr, lu, lu_unpack, svd, svdvals, svd_lowrank, \
    pca_lowrank, eig, eigvals, eigh, eigvalsh, solve, triangular_solve, lstsq, pinv, multi_dot, \
    householder_product, corrcoef, cov, ormqr, vecdot, inv  # noqa: F401
from .tensor.math import matmul, cross  # noqa: F401
from .tensor.manipulation import matrix_transpose  # noqa: F401


def fp8_fp8_half_gemm_fused(x, y, transpose_x=False, transpose_y=False, bias=None, scale=1.0,
                            output_dtype="float16", act="identity", name=None):
    """out = act(scale * op(x) @ op(y) + bias) for OCP fp8 (e4m3fn / e5m2) x, y and a half-precision
    output (reference: python/paddle/tensor/linalg.py fp8_fp8_half_gemm_fused). On the HIP device the
    product runs as a scaled fp8 GEMM (hipBLASLt fp8 MFMA through torch._scaled_mm) when available, else
    as an fp32-accumulated dequantised GEMM."""
    import torch as _torch
    from .framework.tensor import _wrap as _w
    a, b = x._t, y._t
    if transpose_x:
        a = a.transpose(-1, -2)
    if transpose_y:
        b = b.transpose(-1, -2)
    odt = {"float16": _torch.float16, "bfloat16": _torch.bfloat16}[str(output_dtype)]
    out = None
    if a.is_cuda and a.dim() == 2 and hasattr(_torch, "_scaled_mm"):
        try:
            one = _torch.ones((), device=a.device)
            out = _torch._scaled_mm(a.contiguous(), b.t().contiguous().t(), scale_a=one * float(scale),
                                    scale_b=one, out_dtype=odt)
        except (RuntimeError, TypeError):
            out = None
    if out is None:
        out = (float(scale) * _torch.matmul(a.float(), b.float())).to(odt)
    if bias is not None:
        out = out + bias._t.to(odt)
    if act in ("gelu",):
        out = _torch.nn.functional.gelu(out.float(), approximate="tanh").to(odt)
    elif act == "relu":
        out = _torch.relu(out)
    return _w(out)
