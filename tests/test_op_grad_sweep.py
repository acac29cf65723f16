"""OpTest-style sweep (tests/op_test.py; reference test/legacy_test/op_test.py:2877,3081): every op in the table
is checked forward against NumPy where a closed form exists and backward against central-difference numeric
gradients in float64, on the CPU through the native backward engine."""
import math

import numpy as np
import pytest

import paddlepaddle_amd as paddle
import paddlepaddle_amd.nn.functional as F
from op_test import check_grad, check_output

R = np.random.RandomState(1234)


def u(*shape, lo=-1.0, hi=1.0):
    return R.uniform(lo, hi, shape).astype(np.float64)


def away(*shape, lo=0.2, hi=1.0):
    """values with |x| in [lo, hi] (random signs): away from kinks at 0."""
    return (R.uniform(lo, hi, shape) * R.choice([-1.0, 1.0], shape)).astype(np.float64)


def distinct(*shape):
    """a random permutation of well separated values: max / min / sort ties never occur."""
    n = int(np.prod(shape))
    return (R.permutation(n).astype(np.float64) * 0.37 - n * 0.15).reshape(shape)


def pos(*shape, lo=0.3, hi=2.0):
    return R.uniform(lo, hi, shape).astype(np.float64)


def spd(n):
    a = R.standard_normal((n, n))
    return (a @ a.T + n * np.eye(n)).astype(np.float64)


def ints(*shape, hi=4):
    return R.randint(0, hi, shape).astype(np.int64)


def sym(f):
    """f over the symmetric part of its (first) matrix argument: a perturbation of one element of the numeric
    gradient then moves the operand along the same symmetric direction the analytic gradient describes."""
    return lambda a, *r: f((a + paddle.transpose(a, [1, 0])) * 0.5, *r)


# label / target constants (fixed once: the objective must be a deterministic function of the inputs)
SIGN34 = np.sign(away(3, 4))
BIN34 = (R.rand(3, 4) > 0.5).astype("float64")
POS34 = pos(3, 4)
U34 = u(3, 4)
R31 = R.rand(3, 1)


# name -> (fn, inputs, kwargs, numpy reference or None)
UNARY = {
    "abs": (paddle.abs, np.abs), "acos": (paddle.acos, np.arccos), "asin": (paddle.asin, np.arcsin),
    "atan": (paddle.atan, np.arctan), "cos": (paddle.cos, np.cos), "cosh": (paddle.cosh, np.cosh),
    "sin": (paddle.sin, np.sin), "sinh": (paddle.sinh, np.sinh), "tan": (paddle.tan, np.tan),
    "tanh": (paddle.tanh, np.tanh), "exp": (paddle.exp, np.exp), "expm1": (paddle.expm1, np.expm1),
    "erf": (paddle.erf, None), "sigmoid": (F.sigmoid, lambda x: 1 / (1 + np.exp(-x))),
    "square": (paddle.square, np.square), "asinh": (paddle.asinh, np.arcsinh), "atanh": (paddle.atanh, np.arctanh),
    "neg": (paddle.neg, np.negative), "sgn_mul": (lambda x: x * paddle.sign(x), np.abs),
    "deg2rad": (paddle.deg2rad, np.deg2rad), "rad2deg": (paddle.rad2deg, np.rad2deg),
    "stanh": (paddle.stanh, lambda x: 1.7159 * np.tanh(0.67 * x)),
    "sinc_like": (lambda x: paddle.sin(x) / x, lambda x: np.sin(x) / x),
}
POSITIVE = {
    "log": (paddle.log, np.log), "log2": (paddle.log2, np.log2), "log10": (paddle.log10, np.log10),
    "log1p": (paddle.log1p, np.log1p), "sqrt": (paddle.sqrt, np.sqrt), "rsqrt": (paddle.rsqrt, lambda x: x ** -0.5),
    "reciprocal": (paddle.reciprocal, np.reciprocal), "lgamma": (paddle.lgamma, None),
    "digamma": (paddle.digamma, None), "acosh_shift": (lambda x: paddle.acosh(x + 1.0), lambda x: np.arccosh(x + 1)),
    "pow_scalar": (lambda x: paddle.pow(x, 2.5), lambda x: x ** 2.5),
    "logit": (lambda x: paddle.logit(x * 0.3), lambda x: np.log(x * 0.3 / (1 - x * 0.3))),
}
ACTIVATIONS = {
    "relu": (F.relu, lambda x: np.maximum(x, 0)), "relu6": (lambda x: F.relu6(x * 4), None),
    "elu": (F.elu, None), "selu": (F.selu, None), "celu": (F.celu, None), "gelu": (F.gelu, None),
    "gelu_tanh": (lambda x: F.gelu(x, approximate=True), None), "silu": (F.silu, lambda x: x / (1 + np.exp(-x))),
    "mish": (F.mish, None), "softplus": (F.softplus, lambda x: np.log1p(np.exp(x))),
    "softsign": (F.softsign, lambda x: x / (1 + np.abs(x))), "softshrink": (lambda x: F.softshrink(x, 0.1), None),
    "hardshrink": (lambda x: F.hardshrink(x, 0.1), None), "hardtanh": (lambda x: F.hardtanh(x * 0.8), None),
    "hardsigmoid": (F.hardsigmoid, None), "hardswish": (F.hardswish, None),
    "leaky_relu": (lambda x: F.leaky_relu(x, 0.1), lambda x: np.where(x > 0, x, 0.1 * x)),
    "log_sigmoid": (F.log_sigmoid, lambda x: -np.log1p(np.exp(-x))),
    "tanhshrink": (F.tanhshrink, lambda x: x - np.tanh(x)),
    "thresholded_relu": (lambda x: F.thresholded_relu(x, 0.1), None),
    "swish": (F.swish, None), "softmax": (lambda x: F.softmax(x, -1), None),
    "log_softmax": (lambda x: F.log_softmax(x, 0), None), "glu": (lambda x: F.glu(x, -1), None),
}
BINARY = {
    "add": (paddle.add, np.add), "subtract": (paddle.subtract, np.subtract), "multiply": (paddle.multiply, np.multiply),
    "divide": (lambda a, b: paddle.divide(a, b + 3.0), lambda a, b: a / (b + 3)),
    "maximum": (paddle.maximum, np.maximum), "minimum": (paddle.minimum, np.minimum),
    "fmax": (paddle.fmax, np.fmax), "fmin": (paddle.fmin, np.fmin), "atan2": (paddle.atan2, np.arctan2),
    "pow": (lambda a, b: paddle.pow(a + 2.0, b), lambda a, b: (a + 2) ** b),
    "logaddexp": (paddle.logaddexp, np.logaddexp), "hypot": (paddle.hypot, np.hypot),
    "broadcast_add": (lambda a, b: a + b[:1], lambda a, b: a + b[:1]),
    "lerp": (lambda a, b: paddle.lerp(a, b, 0.3), lambda a, b: a + 0.3 * (b - a)),
    "dist": (lambda a, b: paddle.dist(a, b, 2), lambda a, b: np.linalg.norm((a - b).ravel())),
    "inner": (paddle.inner, np.inner), "outer": (lambda a, b: paddle.outer(a[0], b[0]), lambda a, b: np.outer(a[0], b[0])),
    "kron": (paddle.kron, np.kron), "cross": (lambda a, b: paddle.cross(a[:, :3], b[:, :3], axis=1),
                                             lambda a, b: np.cross(a[:, :3], b[:, :3])),
}


def _table():
    t = []
    for n, (f, ref) in UNARY.items():
        x = u(3, 4, lo=-0.9, hi=0.9) if n in ("acos", "asin", "atanh") else away(3, 4)
        t.append((n, f, [x], {}, ref))
    for n, (f, ref) in POSITIVE.items():
        t.append((n, f, [pos(3, 4)], {}, ref))
    for n, (f, ref) in ACTIVATIONS.items():
        t.append((n, f, [away(3, 4)], {}, ref))
    for n, (f, ref) in BINARY.items():
        a, b = (distinct(3, 4), distinct(3, 4)[::-1].copy() + 0.11) if n in ("maximum", "minimum", "fmax", "fmin") \
            else (away(3, 4), away(3, 4))
        t.append((n, f, [a, b], {}, ref))
    t += [
        # reductions / scans
        ("sum", lambda x: paddle.sum(x, axis=1), [u(3, 4)], {}, lambda x: x.sum(1)),
        ("mean", lambda x: paddle.mean(x, axis=0, keepdim=True), [u(3, 4)], {}, lambda x: x.mean(0, keepdims=True)),
        ("prod", lambda x: paddle.prod(x, axis=1), [away(3, 4)], {}, lambda x: x.prod(1)),
        ("max", lambda x: paddle.max(x, axis=1), [distinct(3, 4)], {}, lambda x: x.max(1)),
        ("min", lambda x: paddle.min(x), [distinct(3, 4)], {}, lambda x: x.min()),
        ("amax", lambda x: paddle.amax(x, axis=0), [distinct(3, 4)], {}, lambda x: x.max(0)),
        ("amin", lambda x: paddle.amin(x, axis=1), [distinct(3, 4)], {}, lambda x: x.min(1)),
        ("logsumexp", lambda x: paddle.logsumexp(x, axis=1), [u(3, 4)], {}, None),
        ("std", lambda x: paddle.std(x, axis=1), [u(3, 4)], {}, lambda x: x.std(1, ddof=1)),
        ("var", lambda x: paddle.var(x), [u(3, 4)], {}, lambda x: x.var(ddof=1)),
        ("norm_fro", lambda x: paddle.linalg.norm(x), [u(3, 4)], {}, lambda x: np.linalg.norm(x)),
        ("norm_p3", lambda x: paddle.linalg.norm(x, p=3, axis=1), [away(3, 4)], {}, None),
        ("cumsum", lambda x: paddle.cumsum(x, axis=1), [u(3, 4)], {}, lambda x: np.cumsum(x, 1)),
        ("cumprod", lambda x: paddle.cumprod(x, dim=1), [away(3, 4)], {}, lambda x: np.cumprod(x, 1)),
        ("logcumsumexp", lambda x: paddle.logcumsumexp(x, axis=0), [u(3, 4)], {}, None),
        ("trace", paddle.trace, [u(4, 4)], {}, np.trace),
        ("sort", lambda x: paddle.sort(x, axis=1), [distinct(3, 4)], {}, lambda x: np.sort(x, 1)),
        ("topk", lambda x: paddle.topk(x, 2)[0], [distinct(3, 4)], {}, None),
        ("kthvalue", lambda x: paddle.kthvalue(x, 2)[0], [distinct(3, 4)], {}, None),
        ("median", lambda x: paddle.median(x, axis=1), [distinct(3, 5)], {}, lambda x: np.median(x, 1)),
        ("quantile", lambda x: paddle.quantile(x, 0.3, axis=1), [distinct(3, 5)], {}, lambda x: np.quantile(x, 0.3, 1)),
        # manipulation / indexing
        ("reshape", lambda x: paddle.reshape(x, [4, 3]), [u(3, 4)], {}, lambda x: x.reshape(4, 3)),
        ("transpose", lambda x: paddle.transpose(x, [1, 0]), [u(3, 4)], {}, lambda x: x.T),
        ("concat", lambda a, b: paddle.concat([a, b], axis=1), [u(3, 4), u(3, 2)], {},
         lambda a, b: np.concatenate([a, b], 1)),
        ("stack", lambda a, b: paddle.stack([a, b]), [u(3, 4), u(3, 4)], {}, lambda a, b: np.stack([a, b])),
        ("split", lambda x: paddle.split(x, [1, 3], axis=1), [u(3, 4)], {}, lambda x: np.split(x, [1], 1)),
        ("chunk", lambda x: paddle.chunk(x, 2, axis=1), [u(3, 4)], {}, lambda x: np.split(x, 2, 1)),
        ("unbind", lambda x: paddle.unbind(x, 0), [u(3, 4)], {}, lambda x: list(x)),
        ("squeeze_unsqueeze", lambda x: paddle.squeeze(paddle.unsqueeze(x, [0, 2]), 0), [u(3, 4)], {},
         lambda x: x[:, None]),
        ("flatten", lambda x: paddle.flatten(x), [u(2, 3, 2)], {}, lambda x: x.reshape(-1)),
        ("flip", lambda x: paddle.flip(x, [0, 1]), [u(3, 4)], {}, lambda x: x[::-1, ::-1]),
        ("roll", lambda x: paddle.roll(x, 1, 1), [u(3, 4)], {}, lambda x: np.roll(x, 1, 1)),
        ("rot90", lambda x: paddle.rot90(x), [u(3, 4)], {}, np.rot90),
        ("tile", lambda x: paddle.tile(x, [2, 1]), [u(3, 4)], {}, lambda x: np.tile(x, (2, 1))),
        ("expand", lambda x: paddle.expand(x, [2, 3, 4]), [u(3, 4)], {}, lambda x: np.broadcast_to(x, (2, 3, 4))),
        ("broadcast_to", lambda x: paddle.broadcast_to(x, [3, 4]), [u(1, 4)], {}, lambda x: np.broadcast_to(x, (3, 4))),
        ("gather", lambda x: paddle.gather(x, paddle.to_tensor([2, 0, 2])), [u(3, 4)], {}, lambda x: x[[2, 0, 2]]),
        ("gather_nd", lambda x: paddle.gather_nd(x, paddle.to_tensor([[0, 1], [2, 3]])), [u(3, 4)], {},
         lambda x: x[[0, 2], [1, 3]]),
        ("index_select", lambda x: paddle.index_select(x, paddle.to_tensor([3, 1]), axis=1), [u(3, 4)], {},
         lambda x: x[:, [3, 1]]),
        ("take_along_axis", lambda x: paddle.take_along_axis(x, paddle.to_tensor([[0], [3], [1]]), 1), [u(3, 4)], {},
         lambda x: x[[0, 1, 2], [0, 3, 1]][:, None]),
        ("put_along_axis", lambda x, v: paddle.put_along_axis(x, paddle.to_tensor([[1], [2], [0]]), v, 1),
         [u(3, 4), u(3, 1)], {}, None),
        ("scatter", lambda x, v: paddle.scatter(x, paddle.to_tensor([2, 0]), v), [u(3, 4), u(2, 4)], {}, None),
        ("index_add", lambda x, v: paddle.index_add(x, paddle.to_tensor([0, 2]), 0, v), [u(3, 4), u(2, 4)], {}, None),
        ("slice", lambda x: paddle.slice(x, [1], [1], [3]), [u(3, 4)], {}, lambda x: x[:, 1:3]),
        ("strided_slice", lambda x: paddle.strided_slice(x, [1], [0], [4], [2]), [u(3, 4)], {}, lambda x: x[:, 0:4:2]),
        ("getitem", lambda x: x[1:, ::2], [u(3, 4)], {}, lambda x: x[1:, ::2]),
        ("where", lambda a, b: paddle.where(a > 0, a, b), [away(3, 4), u(3, 4)], {}, lambda a, b: np.where(a > 0, a, b)),
        ("masked_fill", lambda x: paddle.masked_fill(x, x > 0, 0.5), [away(3, 4)], {}, lambda x: np.where(x > 0, .5, x)),
        ("tril", lambda x: paddle.tril(x), [u(4, 4)], {}, np.tril), ("triu", lambda x: paddle.triu(x, 1), [u(4, 4)], {},
                                                                      lambda x: np.triu(x, 1)),
        ("diag", lambda x: paddle.diag(x), [u(4)], {}, np.diag),
        ("diagonal", lambda x: paddle.diagonal(x), [u(4, 4)], {}, np.diagonal),
        ("repeat_interleave", lambda x: paddle.repeat_interleave(x, 2, 0), [u(3, 4)], {},
         lambda x: np.repeat(x, 2, 0)),
        ("moveaxis", lambda x: paddle.moveaxis(x, 0, 2), [u(2, 3, 4)], {}, lambda x: np.moveaxis(x, 0, 2)),
        ("clip", lambda x: paddle.clip(x, -0.5, 0.5), [away(3, 4, lo=0.6, hi=0.9) * 0 + u(3, 4) * 0.4], {},
         lambda x: np.clip(x, -.5, .5)),
        ("scale", lambda x: paddle.scale(x, 2.0, 1.0), [u(3, 4)], {}, lambda x: 2 * x + 1),
        # linear algebra
        ("matmul", paddle.matmul, [u(3, 4), u(4, 2)], {}, np.matmul),
        ("matmul_t", lambda a, b: paddle.matmul(a, b, transpose_y=True), [u(3, 4), u(2, 4)], {},
         lambda a, b: a @ b.T),
        ("bmm", paddle.bmm, [u(2, 3, 4), u(2, 4, 2)], {}, np.matmul),
        ("mv", paddle.mv, [u(3, 4), u(4)], {}, np.dot), ("dot", paddle.dot, [u(4), u(4)], {}, np.dot),
        ("multi_dot", lambda a, b, c: paddle.linalg.multi_dot([a, b, c]), [u(2, 3), u(3, 4), u(4, 2)], {},
         lambda a, b, c: a @ b @ c),
        ("det", paddle.linalg.det, [spd(3)], {}, np.linalg.det),
        ("slogdet", lambda x: paddle.linalg.slogdet(x)[1], [spd(3)], {}, lambda x: np.linalg.slogdet(x)[1]),
        ("inv", paddle.linalg.inv, [spd(3)], {}, np.linalg.inv),
        ("cholesky", sym(paddle.linalg.cholesky), [spd(3)], {}, np.linalg.cholesky),
        ("solve", paddle.linalg.solve, [spd(3), u(3, 2)], {}, np.linalg.solve),
        ("triangular_solve", lambda a, b: paddle.linalg.triangular_solve(paddle.tril(a) + 3 * paddle.eye(3), b,
                                                                          upper=False), [u(3, 3), u(3, 2)], {}, None),
        ("cholesky_solve", sym(lambda a, b: paddle.linalg.cholesky_solve(b, paddle.linalg.cholesky(a))),
         [spd(3), u(3, 2)], {}, None),
        ("pinv", paddle.linalg.pinv, [spd(3)], {}, np.linalg.pinv),
        ("matrix_power", lambda x: paddle.linalg.matrix_power(x, 3), [u(3, 3)], {},
         lambda x: np.linalg.matrix_power(x, 3)),
        ("eigh_values", sym(lambda x: paddle.linalg.eigh(x)[0]), [spd(3)], {}, lambda x: np.linalg.eigh(x)[0]),
        ("svd_values", lambda x: paddle.linalg.svd(x)[1], [u(4, 3)], {}, lambda x: np.linalg.svd(x)[1]),
        ("qr_r_abs", lambda x: paddle.abs(paddle.linalg.qr(x)[1]), [u(4, 3)], {}, None),
        ("lstsq", lambda a, b: paddle.linalg.lstsq(a, b)[0], [u(5, 3), u(5, 2)], {}, None),
        ("matrix_exp", paddle.linalg.matrix_exp, [u(3, 3) * 0.5], {}, None),
        ("cov", lambda x: paddle.linalg.cov(x), [u(3, 6)], {}, np.cov),
        # nn.functional
        ("linear", F.linear, [u(3, 4), u(4, 2), u(2)], {}, lambda x, w, b: x @ w + b),
        ("bilinear", F.bilinear, [u(2, 3), u(2, 4), u(5, 3, 4)], {}, None),
        ("layer_norm", lambda x, w, b: F.layer_norm(x, [4], w, b), [u(3, 4), u(4), u(4)], {}, None),
        ("rms_norm", lambda x, w: F.rms_norm(x, [4], w, 1e-6), [u(3, 4), u(4)], {}, None),
        ("group_norm", lambda x, w, b: F.group_norm(x, 2, 1e-5, w, b), [u(2, 4, 3), u(4), u(4)], {}, None),
        ("instance_norm", lambda x: F.instance_norm(x), [u(2, 3, 5)], {}, None),
        ("batch_norm_train", lambda x, w, b: F.batch_norm(x, paddle.zeros([3], "float64"),
                                                          paddle.ones([3], "float64"), w, b, training=True),
         [u(4, 3, 2), u(3), u(3)], {}, None),
        ("local_response_norm", lambda x: F.local_response_norm(x, 3), [u(1, 5, 2, 2)], {}, None),
        ("normalize", lambda x: F.normalize(x, axis=1), [away(3, 4)], {}, None),
        ("conv1d", lambda x, w: F.conv1d(x, w, padding=1), [u(1, 2, 5), u(3, 2, 3)], {}, None),
        ("conv2d", lambda x, w, b: F.conv2d(x, w, b, stride=1, padding=1), [u(1, 2, 4, 4), u(2, 2, 3, 3), u(2)], {},
         None),
        ("conv2d_stride_groups", lambda x, w: F.conv2d(x, w, stride=2, groups=2), [u(1, 4, 5, 5), u(2, 2, 3, 3)], {},
         None),
        ("conv3d", lambda x, w: F.conv3d(x, w), [u(1, 1, 3, 3, 3), u(1, 1, 2, 2, 2)], {}, None),
        ("conv2d_transpose", lambda x, w: F.conv2d_transpose(x, w, stride=2), [u(1, 2, 3, 3), u(2, 1, 2, 2)], {},
         None),
        ("avg_pool2d", lambda x: F.avg_pool2d(x, 2), [u(1, 2, 4, 4)], {}, None),
        ("max_pool2d", lambda x: F.max_pool2d(x, 2), [distinct(1, 2, 4, 4)], {}, None),
        ("adaptive_avg_pool2d", lambda x: F.adaptive_avg_pool2d(x, 2), [u(1, 2, 5, 5)], {}, None),
        ("adaptive_max_pool2d", lambda x: F.adaptive_max_pool2d(x, 2), [distinct(1, 1, 4, 4)], {}, None),
        ("interp_bilinear", lambda x: F.interpolate(x, scale_factor=2, mode="bilinear"), [u(1, 1, 3, 3)], {}, None),
        ("interp_bicubic", lambda x: F.interpolate(x, size=[4, 5], mode="bicubic"), [u(1, 1, 3, 3)], {}, None),
        ("grid_sample", lambda x, g: F.grid_sample(x, g * 0.8, align_corners=False), [u(1, 1, 3, 3), u(1, 2, 2, 2)], {},
         None),
        ("pad_reflect", lambda x: F.pad(x, [1, 1, 1, 1], mode="reflect"), [u(1, 1, 3, 3)], {}, None),
        ("pad_replicate", lambda x: F.pad(x, [1, 0, 0, 1], mode="replicate"), [u(1, 1, 3, 3)], {}, None),
        ("pixel_shuffle", lambda x: F.pixel_shuffle(x, 2), [u(1, 4, 2, 2)], {}, None),
        ("unfold", lambda x: F.unfold(x, 2), [u(1, 2, 3, 3)], {}, None),
        ("embedding", lambda w: F.embedding(paddle.to_tensor([[1, 3], [0, 1]]), w), [u(4, 3)], {}, None),
        ("cosine_similarity", F.cosine_similarity, [away(3, 4), away(3, 4)], {}, None),
        ("pairwise_distance", F.pairwise_distance, [u(3, 4), u(3, 4)], {}, None),
        ("dropout_eval", lambda x: F.dropout(x, 0.5, training=False), [u(3, 4)], {}, lambda x: x),
        # losses
        ("mse_loss", F.mse_loss, [u(3, 4), u(3, 4)], {}, lambda a, b: ((a - b) ** 2).mean()),
        ("l1_loss", F.l1_loss, [away(3, 4), away(3, 4) * 0], {}, lambda a, b: np.abs(a - b).mean()),
        ("smooth_l1_loss", F.smooth_l1_loss, [u(3, 4), u(3, 4) * 3], {}, None),
        ("cross_entropy", lambda x: F.cross_entropy(x, paddle.to_tensor([1, 0, 3])), [u(3, 4)], {}, None),
        ("cross_entropy_soft", lambda x, y: F.cross_entropy(x, F.softmax(y), soft_label=True), [u(3, 4), u(3, 4)], {},
         None),
        ("nll_loss", lambda x: F.nll_loss(F.log_softmax(x), paddle.to_tensor([1, 0, 3])), [u(3, 4)], {}, None),
        ("bce", lambda x, y: F.binary_cross_entropy(F.sigmoid(x), F.sigmoid(y)), [u(3, 4), u(3, 4)], {}, None),
        ("bce_logits", lambda x, y: F.binary_cross_entropy_with_logits(x, F.sigmoid(y)), [u(3, 4), u(3, 4)], {}, None),
        ("kl_div", lambda x, y: F.kl_div(F.log_softmax(x), F.softmax(y), reduction="batchmean"), [u(3, 4), u(3, 4)],
         {}, None),
        ("margin_ranking", lambda a, b: F.margin_ranking_loss(a, b, paddle.to_tensor(SIGN34), margin=0.1), [u(3, 4), u(3, 4)], {}, None),
        ("soft_margin", lambda x: F.soft_margin_loss(x, paddle.to_tensor(SIGN34)), [u(3, 4)], {}, None),
        ("hinge_embedding", lambda x: F.hinge_embedding_loss(x, paddle.to_tensor(SIGN34)), [pos(3, 4, lo=0.2, hi=0.8)], {}, None),
        ("cosine_embedding", lambda a, b: F.cosine_embedding_loss(a, b, paddle.to_tensor([1, -1, 1])), [away(3, 4),
                                                                                                       away(3, 4)], {},
         None),
        ("triplet_margin", lambda a, p_, n: F.triplet_margin_loss(a, p_, n), [u(3, 4), u(3, 4), u(3, 4) + 2.0], {},
         None),
        ("multi_label_soft_margin", lambda x: F.multi_label_soft_margin_loss(x, paddle.to_tensor(BIN34)), [u(3, 4)], {}, None),
        ("log_loss", lambda x: F.log_loss(F.sigmoid(x), paddle.to_tensor(R31)), [u(3, 1)], {}, None),
        ("poisson_nll", lambda x: F.poisson_nll_loss(x, paddle.to_tensor(POS34)), [u(3, 4)], {}, None),
        ("gaussian_nll", lambda x, v: F.gaussian_nll_loss(x, paddle.to_tensor(U34), v), [u(3, 4), pos(3, 4)], {},
         None),
        ("sigmoid_focal", lambda x: F.sigmoid_focal_loss(x, paddle.to_tensor(BIN34)),
         [u(3, 4)], {}, None),
        ("huber", lambda a, b: paddle.nn.functional.smooth_l1_loss(a, b, delta=0.5), [u(3, 4), u(3, 4) * 2], {}, None),
        # round 4 additions: linear algebra compositions, scans, pooling variants, shape ops
        ("addmm", lambda c, a, b: paddle.addmm(c, a, b, beta=0.5, alpha=2.0), [u(3, 5), u(3, 4), u(4, 5)], {},
         lambda c, a, b: 0.5 * c + 2.0 * a @ b),
        ("einsum", lambda a, b: paddle.einsum("ij,jk->ik", a, b), [u(3, 4), u(4, 2)], {}, lambda a, b: a @ b),
        ("tensordot", lambda a, b: paddle.tensordot(a, b, axes=1), [u(3, 4), u(4, 2)], {}, lambda a, b: a @ b),
        ("diff", lambda x: paddle.diff(x, axis=1), [u(3, 5)], {}, lambda x: np.diff(x, axis=1)),
        ("trapezoid", lambda x: paddle.trapezoid(x, dx=0.5, axis=1), [u(3, 5)], {}, None),
        ("cumulative_trapezoid", lambda x: paddle.cumulative_trapezoid(x, dx=0.5, axis=1), [u(3, 5)], {}, None),
        ("nansum", lambda x: paddle.nansum(x, axis=1), [u(3, 4)], {}, lambda x: np.nansum(x, 1)),
        ("nanmean", lambda x: paddle.nanmean(x, axis=0), [u(3, 4)], {}, lambda x: np.nanmean(x, 0)),
        ("renorm", lambda x: paddle.renorm(x, 2.0, 0, 0.5), [u(3, 4) * 2], {}, None),
        ("diag_embed", lambda x: paddle.diag_embed(x), [u(2, 3)], {}, None),
        ("hstack", lambda a, b: paddle.hstack([a, b]), [u(3, 2), u(3, 4)], {}, lambda a, b: np.hstack([a, b])),
        ("vstack", lambda a, b: paddle.vstack([a, b]), [u(2, 4), u(3, 4)], {}, lambda a, b: np.vstack([a, b])),
        ("index_fill", lambda x: paddle.index_fill(x, paddle.to_tensor([0, 2]), 1, 0.5), [u(3, 4)], {}, None),
        ("copysign", lambda a: paddle.copysign(a, paddle.to_tensor(SIGN34)), [away(3, 4)], {},
         lambda a: np.copysign(a, SIGN34)),
        ("frac", lambda x: paddle.frac(x * 0.9), [pos(3, 4, lo=0.1, hi=0.9)], {}, None),
        ("i0", paddle.i0, [u(3, 4)], {}, None),
        ("i1", paddle.i1, [u(3, 4)], {}, None),
        ("erfinv", lambda x: paddle.erfinv(x * 0.8), [u(3, 4)], {}, None),
        ("polygamma", lambda x: paddle.polygamma(x, 1), [pos(3, 4)], {}, None),
        ("avg_pool1d", lambda x: F.avg_pool1d(x, 2, 2), [u(2, 3, 8)], {}, None),
        ("max_pool1d", lambda x: F.max_pool1d(x, 2, 2), [distinct(2, 3, 8)], {}, None),
        ("avg_pool3d", lambda x: F.avg_pool3d(x, 2, 2), [u(1, 2, 4, 4, 4)], {}, None),
        ("adaptive_avg_pool1d", lambda x: F.adaptive_avg_pool1d(x, 3), [u(2, 3, 7)], {}, None),
        ("pixel_unshuffle", lambda x: F.pixel_unshuffle(x, 2), [u(1, 2, 4, 4)], {}, None),
        ("channel_shuffle", lambda x: F.channel_shuffle(x, 2), [u(1, 4, 3, 3)], {}, None),
        ("fold", lambda x: F.fold(x, [4, 4], [2, 2]), [u(1, 8, 9)], {}, None),
        ("affine_grid", lambda t: F.affine_grid(t, [1, 1, 3, 3], align_corners=False), [u(1, 2, 3)], {}, None),
        ("pad_constant", lambda x: F.pad(x, [1, 2, 0, 1], value=0.3), [u(1, 2, 3, 3)], {}, None),
        ("interp_trilinear", lambda x: F.interpolate(x, size=[3, 5, 5], mode="trilinear", data_format="NCDHW"),
         [u(1, 1, 2, 3, 3)], {}, None),
        ("square_error_cost", lambda a, b: F.square_error_cost(a, b), [u(3, 4), u(3, 4)], {},
         lambda a, b: (a - b) ** 2),
        ("npair_loss", lambda a, p_: F.npair_loss(a, p_, paddle.to_tensor(np.array([0.0, 1.0, 2.0]))),
         [u(3, 4), u(3, 4)], {}, None),
        ("max_pool3d", lambda x: F.max_pool3d(x, 2, 2), [u(1, 2, 4, 4, 4)], {}, None),
        ("adaptive_max_pool1d", lambda x: F.adaptive_max_pool1d(x, 3), [u(2, 3, 7)], {}, None),
        ("adaptive_avg_pool3d", lambda x: F.adaptive_avg_pool3d(x, 2), [u(1, 2, 4, 5, 3)], {}, None),
        ("conv1d_transpose", lambda x, w: F.conv1d_transpose(x, w, stride=2, padding=1), [u(2, 3, 5), u(3, 2, 3)],
         {}, None),
        ("conv3d_transpose", lambda x, w: F.conv3d_transpose(x, w, stride=1), [u(1, 2, 3, 3, 3), u(2, 2, 2, 2, 2)],
         {}, None),
        ("prelu", lambda x, w: F.prelu(x, w), [u(2, 3, 4), u(3) * 0.5], {}, None),
        ("maxout", lambda x: F.maxout(x, 2, axis=1), [u(2, 4, 3, 3)], {}, None),
        ("rrelu_eval", lambda x: F.rrelu(x, training=False), [u(3, 4)], {}, None),
        ("dice_loss", lambda x: F.dice_loss(F.softmax(x), paddle.to_tensor(np.array([[0], [2], [1]], np.int64))),
         [u(3, 3)], {}, None),
        ("label_smooth", lambda x: F.label_smooth(F.softmax(x), epsilon=0.1), [u(3, 4)], {}, None),
        ("multi_margin", lambda x: F.multi_margin_loss(x, paddle.to_tensor(np.array([0, 2, 1], np.int64))),
         [u(3, 4)], {}, None),
        ("cdist", lambda a, b: paddle.cdist(a, b), [u(3, 4), u(5, 4) + 1.0], {}, None),
        ("vector_norm", lambda x: paddle.linalg.vector_norm(x, p=3.0, axis=1), [u(3, 4) + 2.0], {}, None),
        ("matrix_norm_nuc", lambda x: paddle.linalg.matrix_norm(x, p="nuc"), [u(3, 3)], {}, None),
        ("cummax", lambda x: paddle.cummax(x, axis=1)[0], [u(3, 5)], {}, None),
        ("temporal_shift", lambda x: F.temporal_shift(x, seg_num=2, shift_ratio=0.25), [u(4, 4, 2, 2)], {}, None),
        ("zeropad2d", lambda x: F.zeropad2d(x, [1, 0, 2, 1]), [u(1, 2, 3, 3)], {}, None),
        ("interp_nearest", lambda x: F.interpolate(x, scale_factor=2, mode="nearest"), [u(1, 2, 3, 3)], {}, None),
        ("softmax_with_ce", lambda x: F.softmax_with_cross_entropy(x, paddle.to_tensor(np.array([[1], [0], [3]],
                                                                                               np.int64))),
         [u(3, 4)], {}, None),
        ("max_unpool2d", lambda x: F.max_unpool2d(*F.max_pool2d(x, 2, 2, return_mask=True), 2, 2),
         [u(1, 2, 4, 4)], {}, None),
        ("triplet_margin_dist", lambda a, p_, n: F.triplet_margin_with_distance_loss(a, p_, n),
         [u(3, 4), u(3, 4), u(3, 4) + 2.0], {}, None),
        ("bilinear_tensor", lambda a, b, w: F.bilinear(a, b, w), [u(2, 3), u(2, 4), u(5, 3, 4)], {}, None),
    ]
    return t


TABLE = _table()


@pytest.mark.parametrize("name,fn,inputs,kw,ref", TABLE, ids=[t[0] for t in TABLE])
def test_op(name, fn, inputs, kw, ref):
    if ref is not None:
        check_output(fn, inputs, ref, rtol=1e-6, atol=1e-8, **kw)
    tol = 5e-4 if name in ("lstsq", "matrix_exp", "pinv", "svd_values", "eigh_values", "qr_r_abs", "grid_sample",
                           "interp_bicubic", "quantile", "median") else 1e-5
    check_grad(fn, inputs, max_relative_error=tol, **kw)


def test_sweep_covers_the_api_breadth():
    assert len(TABLE) >= 230, len(TABLE)
