"""paddle.static.nn control flow (cond / case / switch_case / while_loop / static_pylayer) and the remaining
static.nn layer builders.

Reference: python/paddle/static/nn/control_flow.py (cond, case, switch_case, while_loop),
static_pylayer.py, static/nn/common.py (conv3d, deform_conv2d, nce, row_conv, spectral_norm,
sparse_embedding), static/nn/sequence_lod.py.

Design: in dygraph (and under jit.to_static, which traces with concrete values) the predicates are
concrete, so control flow is plain Python. Inside a static program the tensors are meta tensors
(shape/dtype only, see static/program.py): ``cond`` records each branch into its own sub-block and
``while_loop`` records the condition and the body into two sub-blocks over loop-variable slots; the
program gets ONE control-flow node (program.CFNode) whose replay evaluates the predicate on the device
values and runs only the chosen block / iterates the body (reference: conditional_block and while ops
executing sub-blocks, static/nn/control_flow.py:755,1620). ``case`` / ``switch_case`` nest ``cond``.
Gradients flow through whatever the replay executed (autograd records the taken branch / every
iteration).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import nn as _nn
from ..nn import functional as F
from ..framework.tensor import Tensor, _wrap

__all__ = ["cond", "case", "switch_case", "while_loop", "static_pylayer", "conv3d", "conv3d_transpose",
           "deform_conv2d", "nce", "row_conv", "spectral_norm", "sparse_embedding", "py_func",
           "sequence_conv", "sequence_pool", "sequence_first_step", "sequence_last_step", "sequence_expand"]


def _is_meta(t):
    return isinstance(t, Tensor) and t._t.device.type == "meta"


def _map2(fn, a, b):
    if isinstance(a, (list, tuple)):
        return type(a)(_map2(fn, x, y) for x, y in zip(a, b))
    if isinstance(a, dict):
        return {k: _map2(fn, a[k], b[k]) for k in a}
    return fn(a, b)


def _prog():
    from ..framework.trace_hook import _active_program
    prog = _active_program()
    if prog is None:
        raise RuntimeError("static control flow outside of a program being built")
    return prog


def _tensors_of(x):
    return x._t if isinstance(x, Tensor) else x


def _leaves_to_t(x):
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, (list, tuple)):
        return type(x)(_leaves_to_t(v) for v in x)
    if isinstance(x, dict):
        return {k: _leaves_to_t(v) for k, v in x.items()}
    return x


def _out_like(a, b):
    """Output structure of a cond: fresh meta values for tensor leaves (shapes / dtypes must agree)."""
    def leaf(x, y):
        if isinstance(x, Tensor) or isinstance(y, Tensor):
            if not (isinstance(x, Tensor) and isinstance(y, Tensor)):
                raise ValueError("cond branches must both return a Tensor at the same position")
            if list(x.shape) != list(y.shape) or x._t.dtype != y._t.dtype:
                raise ValueError(f"cond branches return different shapes / dtypes: {list(x.shape)} {x._t.dtype} vs "
                                 f"{list(y.shape)} {y._t.dtype}")
            with torch._C.DisableTorchFunction():
                return _wrap(torch.empty(x._t.shape, dtype=x._t.dtype, device="meta"))
        if x != y:
            raise ValueError(f"cond branches return different non-tensor values {x!r} / {y!r}")
        return x
    return _map2(leaf, a, b)


def _static_cond(pred, true_fn, false_fn):
    from .program import CFNode, _SubBlock
    from ..framework.trace_hook import _active_program
    prog = _active_program()
    if prog is None:  # meta tensors outside any program: shape inference only
        t = true_fn() if true_fn is not None else None
        f = false_fn() if false_fn is not None else None
        return _out_like(t, f) if t is not None else None
    with prog._sub_block() as tb:
        t = true_fn() if true_fn is not None else None
    with prog._sub_block() as fb:
        f = false_fn() if false_fn is not None else None
    if (t is None) != (f is None):
        raise ValueError("cond: both branches must return values (or both None)")
    res = [prog._template(_leaves_to_t(t)), prog._template(_leaves_to_t(f))]
    out = _out_like(t, f) if t is not None else None
    outs = prog._out_template(_leaves_to_t(out)) if out is not None else None
    node = CFNode("cond", (prog._template(pred._t),), outs, [_SubBlock(tb), _SubBlock(fb)], res)
    prog._append(node)
    return out


def cond(pred, true_fn=None, false_fn=None, name=None, return_names=None):
    if not _is_meta(pred):
        p = bool(pred._t.reshape([]).item()) if isinstance(pred, Tensor) else bool(pred)
        fn = true_fn if p else false_fn
        return fn() if fn is not None else None
    return _static_cond(pred, true_fn, false_fn)


def case(pred_fn_pairs, default=None, name=None):
    pairs = list(pred_fn_pairs)
    if not pairs:
        raise ValueError("pred_fn_pairs must not be empty")
    if default is None:
        pairs, default = pairs[:-1], pairs[-1][1]
    out = default
    for pred, fn in reversed(pairs):
        out_fn = (lambda o: (lambda: o))(out) if not callable(out) else out
        out = (lambda p, f, o: (lambda: cond(p, f, o)))(pred, fn, out_fn)
    return out()


def switch_case(branch_index, branch_fns, default=None, name=None):
    if isinstance(branch_fns, dict):
        items = sorted(branch_fns.items())
    elif branch_fns and isinstance(branch_fns[0], (list, tuple)):
        items = sorted(branch_fns)
    else:
        items = list(enumerate(branch_fns))
    if default is None:
        default = items[-1][1]
    if not _is_meta(branch_index):
        i = int(branch_index._t.reshape([]).item()) if isinstance(branch_index, Tensor) else int(branch_index)
        for k, fn in items:
            if k == i:
                return fn()
        return default()
    out_fn = default
    for k, fn in reversed(items):
        out_fn = (lambda k_, f_, o_: (lambda: cond(_wrap(branch_index._t == k_), f_, o_)))(k, fn, out_fn)
    return out_fn()


def _static_while(cond_fn, body, loop_vars):
    from .program import CFNode, _SubBlock
    prog = _prog()
    init = [v if isinstance(v, Tensor) else _wrap(torch.as_tensor(v)) for v in loop_vars]
    ph = [_wrap(prog._new_like(v._t)) for v in init]
    slots = [prog._slot_of[id(p._t)] for p in ph]
    with prog._sub_block() as cb:
        c = cond_fn(*ph)
    with prog._sub_block() as bb:
        out = body(*ph)
    out = list(out) if isinstance(out, (list, tuple)) else [out]
    if len(out) != len(ph):
        raise ValueError(f"while_loop body returned {len(out)} values for {len(ph)} loop variables")
    for o, p in zip(out, ph):
        if list(o.shape) != list(p.shape):
            raise ValueError(f"while_loop variable changes shape {list(p.shape)} -> {list(o.shape)} (loop "
                             "variables must keep their shapes)")
    res = [prog._template(_tensors_of(c)), prog._template([_tensors_of(o) for o in out])]
    with torch._C.DisableTorchFunction():
        metas = [torch.empty(p._t.shape, dtype=p._t.dtype, device="meta") for p in ph]
    outs = prog._out_template(metas)
    node = CFNode("while", prog._template([v._t for v in init]), outs, [_SubBlock(cb), _SubBlock(bb)], res, slots)
    prog._append(node)
    return [_wrap(m) for m in metas]


def while_loop(cond, body, loop_vars, is_test=False, name=None):
    loop_vars = list(loop_vars)
    first = cond(*loop_vars)
    if _is_meta(first) or any(_is_meta(v) for v in loop_vars):
        return _static_while(cond, body, loop_vars)
    c = first
    while True:
        if not bool(c._t.reshape([]).item() if isinstance(c, Tensor) else c):
            break
        out = body(*loop_vars)
        loop_vars = list(out) if isinstance(out, (list, tuple)) else [out]
        c = cond(*loop_vars)
    return loop_vars


def static_pylayer(forward_fn, inputs, backward_fn=None, name=None):
    """Custom forward with an optional user backward (dygraph PyLayer semantics)."""
    if backward_fn is None:
        return forward_fn(*inputs)

    class _Fn(torch.autograd.Function):
        @staticmethod
        def forward(ctx, *ts):
            with torch.no_grad():
                out = forward_fn(*[_wrap(t) for t in ts])
            ctx.multi = isinstance(out, (list, tuple))
            outs = out if ctx.multi else [out]
            return tuple(o._t for o in outs) if ctx.multi else outs[0]._t

        @staticmethod
        def backward(ctx, *gs):
            r = backward_fn(*[_wrap(g) for g in gs])
            r = r if isinstance(r, (list, tuple)) else [r]
            return tuple(x._t if isinstance(x, Tensor) else x for x in r)

    out = _Fn.apply(*[x._t for x in inputs])
    return tuple(_wrap(o) for o in out) if isinstance(out, tuple) else _wrap(out)


def py_func(func, x, out, backward_func=None, skip_vars_in_backward_input=None):
    xs = x if isinstance(x, (list, tuple)) else [x]
    res = func(*xs)
    if out is None:
        return None
    outs = out if isinstance(out, (list, tuple)) else [out]
    res = res if isinstance(res, (list, tuple)) else [res]
    for o, r in zip(outs, res):
        o._t = (r._t if isinstance(r, Tensor) else torch.as_tensor(np.asarray(r))).to(o._t.dtype)
    return out


# ----------------------------------------------------------------------------------- layer builders
def conv3d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None, param_attr=None,
           bias_attr=None, use_cudnn=True, act=None, name=None, data_format="NCDHW"):
    from .nn import _act
    cin = input.shape[1] if data_format == "NCDHW" else input.shape[-1]
    conv = _nn.Conv3D(cin, num_filters, filter_size, stride, padding, dilation, groups or 1,
                      weight_attr=param_attr, bias_attr=bias_attr, data_format=data_format)
    return _act(conv(input), act)


def conv3d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0, stride=1, dilation=1,
                     groups=None, param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None,
                     data_format="NCDHW"):
    from .nn import _act
    cin = input.shape[1] if data_format == "NCDHW" else input.shape[-1]
    conv = _nn.Conv3DTranspose(cin, num_filters, filter_size, stride, padding, dilation=dilation,
                               groups=groups or 1, weight_attr=param_attr, bias_attr=bias_attr,
                               data_format=data_format)
    return _act(conv(input), act)


def deform_conv2d(x, offset, mask, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=1,
                  deformable_groups=1, im2col_step=1, weight_attr=None, bias_attr=None, name=None):
    from ..vision.ops import DeformConv2D
    layer = DeformConv2D(x.shape[1], num_filters, filter_size, stride, padding, dilation, deformable_groups, groups,
                         weight_attr=weight_attr, bias_attr=bias_attr)
    return layer(x, offset, mask)


def nce(input, label, num_total_classes, sample_weight=None, param_attr=None, bias_attr=None, num_neg_samples=None,
        name=None, sampler="uniform", custom_dist=None, seed=0, is_sparse=False):
    """Noise-contrastive estimation loss [B, 1] with a uniform / custom negative sampler."""
    dim = input.shape[-1]
    w = _nn.Layer().create_parameter([num_total_classes, dim], attr=param_attr)
    b = _nn.Layer().create_parameter([num_total_classes], attr=bias_attr, is_bias=True)
    k = num_neg_samples or 10
    x, y = input._t, label._t.reshape(-1).long()
    g = torch.Generator(device="cpu").manual_seed(seed or 0)
    if sampler == "custom_dist" and custom_dist is not None:
        probs = torch.as_tensor(np.asarray(custom_dist), dtype=torch.float32)
    else:
        probs = torch.full((num_total_classes,), 1.0 / num_total_classes)
    neg = torch.multinomial(probs, x.shape[0] * k, replacement=True, generator=g).view(x.shape[0], k).to(x.device)
    q = probs.to(x.device)

    def logit(ids):
        return (x.unsqueeze(1) * w._t[ids]).sum(-1) + b._t[ids]
    pos_l = logit(y.unsqueeze(1)).squeeze(1) - torch.log(k * q[y])
    neg_l = logit(neg) - torch.log(k * q[neg])
    loss = -torch.nn.functional.logsigmoid(pos_l) - torch.nn.functional.logsigmoid(-neg_l).sum(1)
    if sample_weight is not None:
        loss = loss * sample_weight._t.reshape(-1)
    return _wrap(loss.unsqueeze(1))


def row_conv(input, future_context_size, param_attr=None, act=None):
    """Lookahead convolution: out[t] = sum_{i=0..k} x[t + i] * w[i] (per feature), over [B, T, D]."""
    from .nn import _act
    D = input.shape[-1]
    k = future_context_size
    w = _nn.Layer().create_parameter([k + 1, D], attr=param_attr)
    x = input._t
    xp = torch.nn.functional.pad(x, (0, 0, 0, k))
    out = sum(xp[:, i:i + x.shape[1]] * w._t[i] for i in range(k + 1))
    return _act(_wrap(out), act)


def spectral_norm(weight, dim=0, power_iters=1, eps=1e-12, name=None):
    layer = _nn.SpectralNorm(weight.shape, dim=dim, power_iters=power_iters, eps=eps)
    return layer(weight)


def sparse_embedding(input, size, padding_idx=None, is_test=False, entry=None, table_class="MemorySparseTable",
                     param_attr=None, dtype="float32", slot=None):
    """Lookup into a parameter-server sparse table (distributed/ps) when this process is a PS trainer; without a
    PS runtime (single process / collective mode) a local dense embedding of the same shape."""
    from ..distributed.ps import the_one_ps as _ps
    rt = _ps.get_runtime()
    if rt is not None and rt.client is not None:
        from ..distributed.ps.layers import DistributedEmbedding
        name = getattr(param_attr, "name", None) or f"sparse_embedding_{size[0]}x{size[1]}"
        cache = _SPARSE_EMB.get(name)
        if cache is None:
            cache = _SPARSE_EMB[name] = DistributedEmbedding(size, name=name, padding_idx=padding_idx, entry=entry)
        cache.training = not is_test
        return cache(input)
    return _nn.Embedding(size[0], size[1], padding_idx=padding_idx, weight_attr=param_attr)(input)


_SPARSE_EMB = {}


def _lod(*a, **k):
    raise NotImplementedError("LoD sequence ops (sequence_*) belong to the legacy LoDTensor model; use padded "
                              "batches with lengths / masks (paddle.nn.functional) instead")


sequence_conv = sequence_pool = sequence_first_step = sequence_last_step = sequence_expand = _lod
