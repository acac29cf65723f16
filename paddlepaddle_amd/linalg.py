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
    """out = act(scale * op(x) @ op(y) + bias) for OCP fp8 (e4m3fn / e5m2) x, y and an fp16 / bf16 output
    (reference: python/paddle/tensor/linalg.py fp8_fp8_half_gemm_fused). On the device it is the
    hand-written block-scaled-MFMA fp8 GEMM of csrc/kernels/gemm_fp8.hip (ops/fp8.py): both operands are
    fed K-major, so transpose_y=True (weight stored [N, K]) needs no copy; leading batch dims of x fold
    into M when y is 2-D, and batched y runs per batch."""
    import torch as _torch
    from .framework.tensor import _wrap as _w
    from .ops.fp8 import gemm_fp8
    odt = {"float16": _torch.float16, "bfloat16": _torch.bfloat16}.get(str(output_dtype))
    if odt is None:
        raise ValueError("The output_dtype must be float16 or bfloat16")
    a, b = x._t, y._t
    if transpose_x:
        a = a.transpose(-1, -2)
    b_nk = b if transpose_y else b.transpose(-1, -2)  # [.., N, K]
    bt = None if bias is None else bias._t
    if b_nk.dim() == 2:
        lead = a.shape[:-1]
        a2 = a.reshape(-1, a.shape[-1])
        out = gemm_fp8(a2, b_nk, bt, float(scale), act, odt)
        return _w(out.view(*lead, out.shape[-1]))
    outs = [gemm_fp8(a[i], b_nk[i], bt, float(scale), act, odt) for i in range(b_nk.shape[0])]
    return _w(_torch.stack(outs))
