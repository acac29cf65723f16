"""paddle.linalg. Reference: python/paddle/linalg.py."""
from .tensor.linalg import *  # noqa: F401,F403
from .tensor.linalg import norm, vector_norm, matrix_norm, cond, det, slogdet, matrix_rank, matrix_power, \
    matrix_exp, cholesky, cholesky_solve, cholesky_inverse, qr, lu, lu_unpack, svd, svdvals, svd_lowrank, \
    pca_lowrank, eig, eigvals, eigh, eigvalsh, solve, triangular_solve, lstsq, pinv, multi_dot, \
    householder_product, corrcoef, cov, ormqr, vecdot, inv  # noqa: F401
from .tensor.math import matmul, cross  # noqa: F401
from .tensor.manipulation import matrix_transpose  # noqa: F401
