"""paddle._C_ops: the generated eager op entry points of the reference (paddle/fluid/pybind/eager_op_function.cc,
generated from paddle/phi/ops/yaml/ops.yaml, fused_ops.yaml and inconsistent/dygraph_ops.yaml).

Every op of those files is callable here with the reference signature — positional arguments in yaml order,
keyword arguments by yaml name, yaml defaults — and returns the yaml outputs the reference's eager API returns
(intermediate outputs dropped, one output unwrapped): ``_C_ops.layer_norm(x, scale, bias, eps, 1)`` -> out,
``_C_ops.flash_attn(q, k, v, None, None, 0.0, True, False, False, "")`` -> (out, softmax, softmax_lse, seed_offset),
``_C_ops.rms_norm(x, None, residual, w, None, eps, 2, -1, 0, 0, 0)`` -> (out, residual_out). ``<op>_`` is the
in-place form for ops with in-place pairs (yaml ``inplace``): the outputs are written into the paired inputs.

The signature table is _c_ops_sigs.SIGS (tools/gen_c_ops_sigs.py). Implementations: _IMPL below for ops whose
reference outputs or argument conventions differ from this framework's public API (multi-output normalisations,
attention with its LSE / seed outputs, optimizer updates, fused epilogues ...); every other op binds its yaml
arguments by name (with a small rename table) onto the public function of the same name (paddle.*,
nn.functional, linalg, fft, incubate functional, nn.quant). ``coverage()`` reports which ops resolve how.
"""
from __future__ import annotations

import inspect
import math

import torch

from ._c_ops_sigs import SIGS

_REQ = "__required__"
_IMPL: dict = {}
_CACHE: dict = {}


def _t(x):
    if x is None:
        return None
    if isinstance(x, torch.Tensor):
        return x
    return getattr(x, "_t", x)


def _w(t):
    from .framework.tensor import _wrap
    return None if t is None else _wrap(t)


def impl(*names):
    def deco(fn):
        for n in names:
            _IMPL[n] = fn
        return fn
    return deco


def _default(v):
    if isinstance(v, tuple) and len(v) == 2 and v[0] == "expr":
        return None  # DataType::UNDEFINED, CPUPlace(), ... -> the framework default
    return v


def _bind(op, args, kwargs):
    sig = SIGS[op][0]
    if len(args) > len(sig):
        raise TypeError(f"_C_ops.{op}() takes {len(sig)} arguments ({len(args)} given)")
    out = {}
    for i, (name, _kind, default) in enumerate(sig):
        if i < len(args):
            out[name] = args[i]
        elif name in kwargs:
            out[name] = kwargs.pop(name)
        elif default != _REQ:
            out[name] = _default(default)
        elif name in SIGS[op][4]:  # optional input
            out[name] = None
        else:
            raise TypeError(f"_C_ops.{op}() missing required argument {name!r}")
    if kwargs:
        raise TypeError(f"_C_ops.{op}() got unexpected arguments {sorted(kwargs)}")
    for name, kind, _d in sig:  # framework.proto VarType codes (what legacy callers pass) -> dtype names
        v = out.get(name)
        if kind == "DataType" and isinstance(v, int) and not isinstance(v, bool):
            out[name] = _VARTYPE.get(v, v)
    return out


_VARTYPE = {0: "bool", 1: "int16", 2: "int32", 3: "int64", 4: "float16", 5: "float32", 6: "float64", 20: "uint8",
            21: "int8", 22: "bfloat16", 23: "complex64", 24: "complex128"}


def _namespaces():
    import paddlepaddle_amd as P
    from .nn import functional as F
    from .incubate.nn import functional as IF
    from .nn import quant as Q
    return (P, F, P.linalg, IF, P.fft, Q, P.geometric, P.signal)


def _public(name):
    for ns in _namespaces():
        fn = getattr(ns, name, None)
        if callable(fn) and not isinstance(fn, type):
            return fn
    return None


# yaml argument name -> public parameter names tried in order (after the same name)
_RENAME = {"x": ("input", "inputs", "tensor"), "axis": ("dim", "axes"), "value": ("fill_value",),
           "sections": ("num_or_sections",), "num": ("num_or_sections",), "keepdim": ("keep_dim",),
           "perm": ("axis",), "out_dtype": ("dtype",), "repeat_times": ("repeat_times",),
           "y": ("other",), "index": ("indices",), "transpose_x": ("trans_x",), "transpose_y": ("trans_y",)}


def _generic(op):
    name = op[:-1] if op.endswith("_") and op[:-1] not in SIGS else op
    fn = _public(name)
    if fn is None:
        return None
    try:
        params = inspect.signature(fn).parameters
    except (TypeError, ValueError):
        params = {}
    pnames = [p for p in params if params[p].kind not in (inspect.Parameter.VAR_POSITIONAL,
                                                          inspect.Parameter.VAR_KEYWORD)]
    has_varkw = any(p.kind is inspect.Parameter.VAR_KEYWORD for p in params.values())

    defaults = {n: _default(d) for n, _k, d in SIGS[op][0] if d != _REQ}

    def call(**a):
        kw, used = {}, set()
        for yname, v in a.items():
            cands = (yname,) + _RENAME.get(yname, ())
            hit = next((c for c in cands if c in pnames and c not in used), None)
            if hit is not None:
                kw[hit] = v
                used.add(hit)
            elif has_varkw:
                kw[yname] = v
            elif v is None or (isinstance(v, (list, tuple)) and not v) or (yname in defaults and v == defaults[yname]):
                continue  # an attribute at its yaml default that the public function has no parameter for
            else:
                raise NotImplementedError(f"_C_ops.{op}: argument {yname}={v!r} has no counterpart in "
                                          f"{getattr(fn, '__module__', '')}.{getattr(fn, '__name__', name)}")
        return fn(**kw)
    return call


def _resolve(op):
    fn = _IMPL.get(op)
    if fn is not None:
        return fn, "explicit"
    g = _generic(op)
    return (g, "generic") if g is not None else (None, "missing")


def _make(op):
    outs, inter, inplace = SIGS[op][1], SIGS[op][2], SIGS[op][3]
    keep = [i for i, o in enumerate(outs) if o not in inter]

    def f(*args, **kwargs):
        a = _bind(op, args, dict(kwargs))
        fn, how = _resolve(op)
        if fn is None:
            raise NotImplementedError(f"_C_ops.{op}: no implementation in paddlepaddle_amd")
        res = fn(**a)
        if how == "explicit" and len(outs) > 1:
            res = tuple(res)
            res = [res[i] for i in keep]
        elif isinstance(res, list) and len(outs) > 1:
            res = list(res)
        if op.endswith("_") and inplace:  # in-place op (adamw_, ...): results written into the paired inputs
            pairs = dict(inplace)
            vals = res if isinstance(res, (list, tuple)) and len(keep) > 1 else [res]
            names = [outs[i] for i in keep]
            inv = {o: i for i, o in pairs.items()}
            ret = []
            for nm, v in zip(names, vals):
                src = a.get(inv.get(nm))
                if src is not None and v is not None and v is not src and hasattr(src, "_t") and hasattr(v, "_t"):
                    src._t.data.copy_(v._t.detach().reshape(src._t.shape).to(src._t.dtype))
                    v = src
                ret.append(v)
            return ret[0] if len(ret) == 1 else tuple(ret)
        if isinstance(res, (list, tuple)) and len(keep) == 1 and len(outs) > 1 and how == "explicit":
            return res[0]
        return res
    f.__name__ = op
    f.__doc__ = f"_C_ops.{op}({', '.join(n for n, _, _ in SIGS[op][0])}) -> {', '.join(outs[i] for i in keep)}"
    return f


def _inplace_of(op):
    """``op_`` for an op with in-place pairs: run ``op`` and write its outputs into the paired inputs."""
    base = _make(op)
    pairs = SIGS[op][3]
    names = [n for n, _, _ in SIGS[op][0]]
    outs = [o for o in SIGS[op][1] if o not in SIGS[op][2]]

    def f(*args, **kwargs):
        a = _bind(op, args, dict(kwargs))
        res = base(**a)
        vals = list(res) if isinstance(res, (list, tuple)) and len(outs) > 1 else [res]
        ret = []
        for o, v in zip(outs, vals):
            src = next((a[i] for i, oo in pairs if oo == o), None)
            if src is not None and hasattr(src, "_t") and hasattr(v, "_t"):
                if tuple(src._t.shape) == tuple(v._t.shape):
                    src._t.data.copy_(v._t.detach().to(src._t.dtype))
                else:
                    src._t.data = v._t.detach().to(src._t.dtype)
                ret.append(src)
            else:
                ret.append(v)
        return ret[0] if len(ret) == 1 else tuple(ret)
    f.__name__ = op + "_"
    del names
    return f


def __getattr__(name):
    if name.startswith("__"):
        raise AttributeError(name)
    if name in _CACHE:
        return _CACHE[name]
    if name in SIGS:
        fn = _make(name)
    elif name.endswith("_") and name[:-1] in SIGS and SIGS[name[:-1]][3]:
        fn = _inplace_of(name[:-1])
    else:
        fn = _public(name)
        if fn is None and name.endswith("_") and _public(name[:-1]) is not None:
            base = _public(name[:-1])

            def fn(x, *a, **k):
                out = base(x, *a, **k)
                if hasattr(out, "_t"):
                    x._t.data.copy_(out._t.detach())
                return x
        if fn is None:
            raise AttributeError(f"paddle._C_ops has no op {name!r}")
    _CACHE[name] = fn
    return fn


def coverage():
    """{"explicit": [...], "generic": [...], "missing": [...]}: how every yaml op resolves."""
    res = {"explicit": [], "generic": [], "missing": []}
    for op in sorted(SIGS):
        res[_resolve(op)[1]].append(op)
    return res


# ----------------------------------------------------------------------------------------------- implementations
def _rows(x, axis):
    shape = x.shape
    return int(math.prod(shape[:axis])), int(math.prod(shape[axis:]))


@impl("layer_norm")
def _layer_norm(x, scale, bias, epsilon=1e-5, begin_norm_axis=1):
    xt = _t(x)
    axis = begin_norm_axis % xt.dim() if xt.dim() else 0
    ns = xt.shape[axis:]
    from .nn import functional as F
    w = None if scale is None else _w(_t(scale).reshape(ns))
    b = None if bias is None else _w(_t(bias).reshape(ns))
    out = F.layer_norm(x if hasattr(x, "_t") else _w(xt), list(ns), w, b, epsilon)
    rows, cols = _rows(xt, axis)
    xf = xt.detach().reshape(rows, cols).float()
    return out, _w(xf.mean(-1)), _w(xf.var(-1, unbiased=False))


@impl("rms_norm")
def _rms_norm(x, bias, residual, norm_weight, norm_bias, epsilon, begin_norm_axis, quant_scale=-1.0,
              quant_round_type=0, quant_max_bound=0.0, quant_min_bound=0.0):
    from .incubate.nn import functional as IF
    r = IF.fused_rms_norm(x, norm_weight, norm_bias, epsilon, begin_norm_axis, bias=bias, residual=residual,
                          quant_scale=quant_scale, quant_round_type=quant_round_type,
                          quant_max_bound=quant_max_bound, quant_min_bound=quant_min_bound)
    out, res_out = (r if isinstance(r, tuple) else (r, None))
    src = _t(res_out) if res_out is not None else _t(x)
    if res_out is None and bias is not None:
        src = src + _t(bias)
    axis = begin_norm_axis % src.dim()
    rows, cols = _rows(src, axis)
    inv = torch.rsqrt(src.detach().reshape(rows, cols).float().pow(2).mean(-1) + epsilon)
    return out, res_out, _w(inv)


def _seed_offset(fixed_seed_offset, device):
    if fixed_seed_offset is not None:
        return fixed_seed_offset
    return _w(torch.zeros(2, dtype=torch.int64))


def _attn_outputs(q, k, o, lse, causal, scale, mask, return_softmax, fixed_seed_offset):
    from .nn.functional.flash_attention import _softmax_of
    sm = _softmax_of(q, k, causal, scale, mask) if return_softmax else torch.empty(0, dtype=q.dtype,
                                                                                    device=q.device)
    return _w(o), _w(sm), _w(lse), _seed_offset(fixed_seed_offset, q.device)


@impl("flash_attn")
def _flash_attn(q, k, v, fixed_seed_offset, attn_mask, dropout=0.0, causal=False, return_softmax=False,
                is_test=False, rng_name=""):
    from .ops import attention as A
    from .nn.functional.flash_attention import _seed_of
    qt, kt, vt = _t(q), _t(k), _t(v)
    scale = 1.0 / math.sqrt(qt.shape[-1])
    mask = _t(attn_mask)
    seed = _seed_of(fixed_seed_offset)
    o, lse = A.attention(qt, kt, vt, causal=causal, scale=scale, mask=mask, dropout=dropout, training=not is_test,
                         seed=seed, return_lse=True)
    return _attn_outputs(qt, kt, o, lse, causal, scale, mask, return_softmax, fixed_seed_offset)


@impl("flash_attn_unpadded")
def _flash_attn_unpadded(q, k, v, cu_seqlens_q, cu_seqlens_k, fixed_seed_offset, attn_mask, max_seqlen_q,
                         max_seqlen_k, scale, dropout=0.0, causal=False, return_softmax=False, is_test=False,
                         rng_name=""):
    from .ops import attention as A
    from .nn.functional.flash_attention import _seed_of
    qt, kt, vt = _t(q), _t(k), _t(v)
    if return_softmax:
        raise NotImplementedError("_C_ops.flash_attn_unpadded(return_softmax=True)")
    o, lse = A.attention(qt, kt, vt, causal=causal, scale=float(scale), dropout=dropout, training=not is_test,
                         seed=_seed_of(fixed_seed_offset), cu_seqlens_q=_t(cu_seqlens_q),
                         cu_seqlens_k=_t(cu_seqlens_k), max_seqlen_q=int(max_seqlen_q),
                         max_seqlen_k=int(max_seqlen_k), return_lse=True)
    return (_w(o), _w(torch.empty(0, dtype=qt.dtype, device=qt.device)), _w(lse),
            _seed_offset(fixed_seed_offset, qt.device))


@impl("flash_attn_qkvpacked")
def _flash_attn_qkvpacked(qkv, fixed_seed_offset, attn_mask, dropout=0.0, causal=False, return_softmax=False,
                          is_test=False, rng_name=""):
    from .nn.functional.flash_attention import _split_packed
    q, k, v = _split_packed(_t(qkv))
    return _flash_attn(_w(q), _w(k), _w(v), fixed_seed_offset, attn_mask, dropout, causal, return_softmax, is_test,
                       rng_name)


@impl("dropout")
def _dropout(x, seed_tensor, p, is_test, mode, seed, fix_seed):
    xt = _t(x)
    p = float(_t(p).item()) if hasattr(p, "_t") else float(p)
    upscale = mode in ("upscale_in_train", "upscale-in-train")
    if is_test or p == 0.0:
        out = xt if upscale else xt * (1.0 - p)
        return _w(out), _w(torch.ones_like(xt, dtype=torch.uint8))
    g = None
    if fix_seed or seed_tensor is not None:
        g = torch.Generator(device=xt.device)
        g.manual_seed(int(_t(seed_tensor).reshape(-1)[0].item()) if seed_tensor is not None else int(seed))
    keep = (torch.rand(xt.shape, device=xt.device, generator=g) >= p)
    out = xt * keep.to(xt.dtype)
    if upscale:
        out = out / (1.0 - p) if p < 1.0 else torch.zeros_like(xt)
    return _w(out), _w(keep.to(torch.uint8))


@impl("cross_entropy_with_softmax")
def _ce_softmax(input, label, soft_label=False, use_softmax=True, numeric_stable_mode=True, ignore_index=-100,
                axis=-1):
    x = _t(input)
    lab = _t(label)
    ax = axis % x.dim()
    sm = torch.softmax(x.float(), ax) if use_softmax else x.float()
    logp = torch.log(sm.clamp_min(1e-38)) if not use_softmax else torch.log_softmax(x.float(), ax)
    if soft_label:
        loss = -(lab.float() * logp).sum(ax, keepdim=True)
    else:
        li = lab.long()
        if li.dim() == x.dim() and li.shape[ax] == 1:
            li = li.squeeze(ax)
        valid = li != ignore_index
        safe = li.masked_fill(~valid, 0)
        loss = -logp.gather(ax, safe.unsqueeze(ax)).squeeze(ax)
        loss = (loss * valid).unsqueeze(ax)
    return _w(sm.to(x.dtype)), _w(loss.to(x.dtype))


@impl("fused_rotary_position_embedding")
def _fused_rope(q, k, v, sin, cos, position_ids, use_neox_rotary_style=True, time_major=False,
                rotary_emb_base=10000.0):
    from .incubate.nn import functional as IF
    r = IF.fused_rotary_position_embedding(q, k, v, sin=sin, cos=cos, position_ids=position_ids,
                                           use_neox_rotary_style=use_neox_rotary_style, time_major=time_major,
                                           rotary_emb_base=rotary_emb_base)
    r = tuple(r) if isinstance(r, (list, tuple)) else (r,)
    return tuple(r) + (None,) * (3 - len(r))


@impl("fused_linear_param_grad_add")
def _fused_linear_param_grad_add(x, dout, dweight, dbias, multi_precision=True, has_bias=True):
    """dweight (+)= x^T . dout over all leading dims, dbias (+)= column sums (reference fusion kernel
    fused_linear_param_grad_add_kernel.cu:146)."""
    xt, dt = _t(x), _t(dout)
    x2 = xt.reshape(-1, xt.shape[-1])
    d2 = dt.reshape(-1, dt.shape[-1])
    acc = torch.float32 if multi_precision else dt.dtype
    dw = (x2.to(acc).t() @ d2.to(acc))
    if dweight is not None:
        dw = _t(dweight).to(acc) + dw
    db = None
    if has_bias:
        db = d2.to(acc).sum(0)
        if dbias is not None:
            db = _t(dbias).to(acc) + db
    return _w(dw), _w(db)


@impl("fused_gemm_epilogue")
def _fused_gemm_epilogue(x, y, bias, trans_x=False, trans_y=False, activation="none"):
    xt, yt = _t(x), _t(y)
    a = xt.transpose(-1, -2) if trans_x else xt
    b = yt.transpose(-1, -2) if trans_y else yt
    pre = torch.matmul(a, b) + _t(bias)
    act = (activation or "none").lower()
    if act == "relu":
        out = torch.relu(pre)
    elif act == "gelu":
        out = torch.nn.functional.gelu(pre, approximate="tanh")
    else:
        out = pre
    return _w(out), (_w(pre) if act != "none" else None)


def _adam_like(param, grad, learning_rate, moment1, moment2, moment2_max, beta1_pow, beta2_pow, master_param,
               skip_update, beta1, beta2, epsilon, multi_precision, use_global_beta_pow, amsgrad, decay=None):
    if skip_update is not None and bool(_t(skip_update).reshape(-1)[0].item()):
        return (param, moment1, moment2, moment2_max, beta1_pow, beta2_pow, master_param)
    b1 = float(_t(beta1).item()) if hasattr(beta1, "_t") else float(beta1)
    b2 = float(_t(beta2).item()) if hasattr(beta2, "_t") else float(beta2)
    eps = float(_t(epsilon).item()) if hasattr(epsilon, "_t") else float(epsilon)
    lr = _t(learning_rate).float().reshape(-1)[0]
    p = _t(master_param) if (multi_precision and master_param is not None) else _t(param)
    g = _t(grad).float()
    m, v = _t(moment1), _t(moment2)
    b1p, b2p = _t(beta1_pow), _t(beta2_pow)
    with torch.no_grad():
        pf = p.float()
        if decay is not None:
            pf = pf * (1.0 - lr * decay)
        mf = m.float() * b1 + (1 - b1) * g
        vf = v.float() * b2 + (1 - b2) * g * g
        vhat = vf
        vmax = None
        if amsgrad and moment2_max is not None:
            vmax = torch.maximum(_t(moment2_max).float(), vf)
            vhat = vmax
        b1pf, b2pf = b1p.float().reshape(-1)[0].to(pf.device), b2p.float().reshape(-1)[0].to(pf.device)
        lr_t = lr * torch.sqrt(1 - b2pf) / (1 - b1pf)
        pf = pf - lr_t * (mf / (torch.sqrt(vhat) + eps * torch.sqrt(1 - b2pf)))
        m.copy_(mf.to(m.dtype))
        v.copy_(vf.to(v.dtype))
        if vmax is not None:
            _t(moment2_max).copy_(vmax.to(_t(moment2_max).dtype))
        p.copy_(pf.to(p.dtype))
        if multi_precision and master_param is not None:
            _t(param).copy_(pf.to(_t(param).dtype))
        if not use_global_beta_pow:
            b1p.mul_(b1)
            b2p.mul_(b2)
    return (param, moment1, moment2, moment2_max, beta1_pow, beta2_pow, master_param)


@impl("adam_")
def _adam_(param, grad, learning_rate, moment1, moment2, moment2_max, beta1_pow, beta2_pow, master_param,
           skip_update, beta1=0.9, beta2=0.999, epsilon=1e-8, lazy_mode=False, min_row_size_to_use_multithread=1000,
           multi_precision=False, use_global_beta_pow=False, amsgrad=False):
    return _adam_like(param, grad, learning_rate, moment1, moment2, moment2_max, beta1_pow, beta2_pow, master_param,
                      skip_update, beta1, beta2, epsilon, multi_precision, use_global_beta_pow, amsgrad)


@impl("adamw_")
def _adamw_(param, grad, learning_rate, moment1, moment2, moment2_max, beta1_pow, beta2_pow, master_param,
            skip_update, beta1=0.9, beta2=0.999, epsilon=1e-8, lr_ratio=1.0, coeff=0.01, with_decay=False,
            lazy_mode=False, min_row_size_to_use_multithread=1000, multi_precision=False, use_global_beta_pow=False,
            amsgrad=False):
    lrt = _t(learning_rate)
    if lr_ratio != 1.0:
        learning_rate = _w(lrt.float() * lr_ratio)
    return _adam_like(param, grad, learning_rate, moment1, moment2, moment2_max, beta1_pow, beta2_pow, master_param,
                      skip_update, beta1, beta2, epsilon, multi_precision, use_global_beta_pow, amsgrad,
                      decay=coeff if with_decay else None)


@impl("sgd_")
def _sgd_(param, learning_rate, grad, master_param, multi_precision=False):
    lr = _t(learning_rate).float().reshape(-1)[0]
    p = _t(master_param) if (multi_precision and master_param is not None) else _t(param)
    with torch.no_grad():
        pf = p.float() - lr * _t(grad).float()
        p.copy_(pf.to(p.dtype))
        if multi_precision and master_param is not None:
            _t(param).copy_(pf.to(_t(param).dtype))
    return param, master_param


@impl("momentum_")
def _momentum_(param, grad, velocity, learning_rate, master_param, mu, use_nesterov=False,
               regularization_method="", regularization_coeff=0.0, multi_precision=False, rescale_grad=1.0):
    lr = _t(learning_rate).float().reshape(-1)[0]
    p = _t(master_param) if (multi_precision and master_param is not None) else _t(param)
    with torch.no_grad():
        g = _t(grad).float() * rescale_grad
        if regularization_method == "l2_decay":
            g = g + regularization_coeff * p.float()
        vel = _t(velocity)
        vf = vel.float() * mu + g
        pf = p.float() - lr * ((g + mu * vf) if use_nesterov else vf)
        vel.copy_(vf.to(vel.dtype))
        p.copy_(pf.to(p.dtype))
        if multi_precision and master_param is not None:
            _t(param).copy_(pf.to(_t(param).dtype))
    return param, velocity, master_param


@impl("check_finite_and_unscale_")
def _check_finite_and_unscale_(x, scale):
    s = _t(scale).float().reshape(-1)[0]
    found = torch.zeros(1, dtype=torch.bool, device=s.device)
    with torch.no_grad():
        for t in x:
            tt = _t(t)
            found |= ~torch.isfinite(tt).all().reshape(1).to(found.device)
            tt.mul_((1.0 / s).to(tt.dtype) if tt.is_floating_point() else 1)
    return list(x), _w(found)


@impl("full")
def _full(shape, value, dtype=None, place=None):
    import paddlepaddle_amd as P
    shp = [int(_t(s).item()) if hasattr(s, "_t") else int(s) for s in (_t(shape).tolist()
                                                                      if hasattr(shape, "_t") else shape)]
    return P.full(shp, value, dtype=dtype or "float32")


@impl("gaussian")
def _gaussian(shape, mean=0.0, std=1.0, seed=0, dtype=None, place=None):
    import paddlepaddle_amd as P
    out = P.normal(mean, std, list(shape))
    return out.astype(dtype) if dtype is not None else out


@impl("embedding")
def _embedding(x, weight, padding_idx=-1, sparse=False):
    from .nn import functional as F
    return F.embedding(x, weight, padding_idx=None if padding_idx in (-1, None) else padding_idx, sparse=sparse)


@impl("matmul")
def _matmul(x, y, transpose_x=False, transpose_y=False):
    import paddlepaddle_amd as P
    return P.matmul(x, y, transpose_x=transpose_x, transpose_y=transpose_y)


@impl("softmax")
def _softmax(x, axis=-1):
    from .nn import functional as F
    return F.softmax(x, axis=axis)


@impl("swiglu")
def _swiglu(x, y=None):
    from .incubate.nn import functional as IF
    return IF.swiglu(x, y)


@impl("top_p_sampling")
def _top_p_sampling(x, ps, threshold, topp_seed, seed=-1, k=0, mode="truncate", return_top=False):
    """Nucleus sampling per row: (out probability, ids, top-k scores, top-k ids); top-k outputs are filled only with
    return_top (reference top_p_sampling_kernel.cu semantics at the API level)."""
    xt = _t(x).float()
    p = _t(ps).float().reshape(-1, 1)
    srt, idx = torch.sort(xt, -1, descending=True)
    cum = srt.cumsum(-1)
    cut = (cum - srt) > p
    if threshold is not None:
        cut |= srt < _t(threshold).float().reshape(-1, 1)
    cut[:, 0] = False
    probs = srt.masked_fill(cut, 0.0)
    g = None
    if seed is not None and seed >= 0:
        g = torch.Generator(device=xt.device)
        g.manual_seed(int(seed))
    pick = torch.multinomial(probs / probs.sum(-1, keepdim=True), 1, generator=g)
    ids = idx.gather(-1, pick)
    out = srt.gather(-1, pick)
    kk = max(int(k), 1)
    tops, topi = (srt[:, :kk], idx[:, :kk]) if return_top else (None, None)
    return _w(out.to(_t(x).dtype)), _w(ids.long()), _w(tops), _w(topi)


# ---- ops whose public counterpart has another name or argument convention
def _pd():
    import paddlepaddle_amd as P
    return P


def _F():
    from .nn import functional as F
    return F


def _VO():
    from .vision import ops as VO
    return VO


@impl("roi_align")
def _roi_align(x, boxes, boxes_num, pooled_height=1, pooled_width=1, spatial_scale=1.0, sampling_ratio=-1,
               aligned=False):
    return _VO().roi_align(x, boxes, boxes_num, (pooled_height, pooled_width), spatial_scale, sampling_ratio, aligned)


@impl("roi_pool")
def _roi_pool(x, boxes, boxes_num, pooled_height=1, pooled_width=1, spatial_scale=1.0):
    return _VO().roi_pool(x, boxes, boxes_num, (pooled_height, pooled_width), spatial_scale), None


@impl("psroi_pool")
def _psroi_pool(x, boxes, boxes_num, pooled_height=1, pooled_width=1, output_channels=1, spatial_scale=1.0):
    return _VO().psroi_pool(x, boxes, boxes_num, (pooled_height, pooled_width), spatial_scale)


@impl("nms")
def _nms(x, threshold=1.0):
    return _VO().nms(x, iou_threshold=threshold)


@impl("bce_loss")
def _bce_loss(input, label):
    return _F().binary_cross_entropy(input, label, reduction="none")


@impl("kldiv_loss")
def _kldiv_loss(x, label, reduction="mean", log_target=False):
    return _F().kl_div(x, label, reduction=reduction, log_target=log_target)


@impl("hinge_loss")
def _hinge_loss(logits, labels):
    lg, lb = _t(logits), _t(labels)
    return _w(torch.clamp(1.0 - lg * (2.0 * lb - 1.0), min=0.0))


def _interp(mode):
    def f(x, out_size=None, size_tensor=None, scale_tensor=None, data_format="NCHW", out_d=0, out_h=0, out_w=0,
          scale=None, interp_method="bilinear", align_corners=True, align_mode=1):
        nsp = _t(x).dim() - 2
        size = None
        if out_size is not None:
            size = [int(v) for v in _t(out_size).reshape(-1).tolist()]
        elif size_tensor:
            size = [int(_t(s).reshape(-1)[0].item()) for s in size_tensor]
        else:
            dims = {1: [out_w], 2: [out_h, out_w], 3: [out_d, out_h, out_w]}[nsp]
            if all(d and d > 0 for d in dims):
                size = dims
        sf = None
        if size is None:
            if scale_tensor is not None:
                sf = [float(v) for v in _t(scale_tensor).reshape(-1).tolist()]
            elif scale:
                sf = list(scale) if isinstance(scale, (list, tuple)) else [scale] * nsp
        m = {"bilinear": "bilinear", "nearest": "nearest", "linear": "linear", "bicubic": "bicubic",
             "trilinear": "trilinear"}[interp_method or mode]
        return _F().interpolate(x, size=size, scale_factor=sf, mode=m, align_corners=align_corners and m != "nearest",
                                align_mode=align_mode, data_format=data_format)
    return f


for _m in ("bilinear", "nearest", "linear", "bicubic", "trilinear"):
    _IMPL[_m + "_interp"] = _interp(_m)


@impl("pool2d")
def _pool2d(x, kernel_size, strides=(1, 1), paddings=(0, 0), ceil_mode=False, exclusive=True, data_format="NCHW",
            pooling_type="max", global_pooling=False, adaptive=False, padding_algorithm="EXPLICIT"):
    F = _F()
    xt = _t(x)
    hw = xt.shape[2:] if data_format == "NCHW" else xt.shape[1:3]
    ks = list(hw) if global_pooling else list(kernel_size)
    pad = "SAME" if padding_algorithm == "SAME" else ("VALID" if padding_algorithm == "VALID" else list(paddings))
    if adaptive:
        fn = F.adaptive_max_pool2d if pooling_type == "max" else F.adaptive_avg_pool2d
        return fn(x, ks, data_format=data_format) if pooling_type != "max" else fn(x, ks)
    if pooling_type == "max":
        return F.max_pool2d(x, ks, strides, 0 if global_pooling else pad, ceil_mode=ceil_mode, data_format=data_format)
    return F.avg_pool2d(x, ks, strides, 0 if global_pooling else pad, ceil_mode=ceil_mode, exclusive=exclusive,
                        data_format=data_format)


@impl("max_pool2d_with_index")
def _max_pool2d_with_index(x, kernel_size, strides=(1, 1), paddings=(0, 0), global_pooling=False, adaptive=False,
                           ceil_mode=False):
    F = _F()
    ks = list(_t(x).shape[2:]) if global_pooling else list(kernel_size)
    if adaptive:
        return F.adaptive_max_pool2d(x, ks, return_mask=True)
    return F.max_pool2d(x, ks, strides, 0 if global_pooling else list(paddings), ceil_mode=ceil_mode,
                        return_mask=True)


@impl("pad3d")
def _pad3d(x, paddings, mode="constant", pad_value=0.0, data_format="NCDHW"):
    pads = [int(v) for v in (_t(paddings).tolist() if hasattr(paddings, "_t") else paddings)]
    return _F().pad(x, pads, mode=mode, value=pad_value, data_format=data_format)


@impl("tanh_shrink")
def _tanh_shrink(x):
    return _F().tanhshrink(x)


@impl("depthwise_conv2d")
def _depthwise_conv2d(input, filter, strides=(1, 1), paddings=(0, 0), padding_algorithm="EXPLICIT", groups=1,
                      dilations=(1, 1), data_format="NCHW"):
    pad = padding_algorithm if padding_algorithm in ("SAME", "VALID") else list(paddings)
    return _F().conv2d(input, filter, None, list(strides), pad, list(dilations), groups, data_format)


@impl("elementwise_pow")
def _elementwise_pow(x, y):
    return _pd().pow(x, y)


@impl("p_norm")
def _p_norm(x, porder=2.0, axis=-1, epsilon=1e-12, keepdim=False, asvector=False):
    xt = _t(x)
    if asvector:
        xt = xt.reshape(-1)
        axis = 0
    return _w(torch.linalg.vector_norm(xt, ord=porder, dim=axis, keepdim=keepdim))


@impl("frobenius_norm")
def _frobenius_norm(x, axis=(), keep_dim=False, reduce_all=False):
    xt = _t(x)
    dims = None if (reduce_all or not axis) else list(axis)
    return _w(torch.sqrt((xt.float() ** 2).sum(dim=dims, keepdim=keep_dim)).to(xt.dtype))


@impl("l1_norm")
def _l1_norm(x):
    return _w(_t(x).abs().sum())


@impl("squared_l2_norm")
def _squared_l2_norm(x):
    return _w((_t(x).float() ** 2).sum().reshape(1).to(_t(x).dtype))


@impl("mean_all")
def _mean_all(x):
    return _w(_t(x).mean())


@impl("clip_by_norm")
def _clip_by_norm(x, max_norm):
    xt = _t(x)
    n = torch.linalg.vector_norm(xt.float())
    return _w((xt.float() * (max_norm / torch.clamp(n, min=max_norm))).to(xt.dtype))


@impl("sigmoid_cross_entropy_with_logits")
def _sigmoid_ce(x, label, pos_weight=None, normalize=False, ignore_index=-100):
    xt, lt = _t(x).float(), _t(label).float()
    pw = None if pos_weight is None else _t(pos_weight).float()
    loss = torch.nn.functional.binary_cross_entropy_with_logits(xt, lt, reduction="none", pos_weight=pw)
    valid = lt != ignore_index
    loss = loss * valid
    if normalize:
        loss = loss / valid.sum().clamp_min(1)
    return _w(loss.to(_t(x).dtype))


@impl("identity_loss")
def _identity_loss(x, reduction=1):
    xt = _t(x)
    r = {0: "sum", 1: "mean", 2: "none"}.get(reduction, reduction)
    return _w(xt.sum() if r == "sum" else (xt.mean() if r == "mean" else xt))


@impl("fused_softmax_mask")
def _fused_softmax_mask(x, mask):
    from .incubate import softmax_mask_fuse
    return softmax_mask_fuse(x, mask)


@impl("fused_softmax_mask_upper_triangle")
def _fused_softmax_mask_ut(X):
    from .incubate import softmax_mask_fuse_upper_triangle
    return softmax_mask_fuse_upper_triangle(X)


@impl("accuracy")
def _accuracy(x, indices, label):
    it, lt = _t(indices), _t(label).reshape(-1, 1)
    correct = (it == lt).any(-1).sum()
    total = torch.tensor(it.shape[0], device=it.device)
    return _w((correct.float() / max(int(total), 1)).reshape(1)), _w(correct.reshape(1).int()), \
        _w(total.reshape(1).int())


@impl("shuffle_channel")
def _shuffle_channel(x, group=1):
    return _F().channel_shuffle(x, group)


@impl("split_with_num")
def _split_with_num(x, num, axis=0):
    return _pd().split(x, int(num), axis)


@impl("repeat_interleave_with_tensor_index")
def _repeat_interleave_t(x, repeats, axis=0):
    return _pd().repeat_interleave(x, repeats, axis)


@impl("shape64")
def _shape64(input):
    return _w(torch.tensor(list(_t(input).shape), dtype=torch.int64))


@impl("fill_diagonal")
def _fill_diagonal(x, value=0.0, offset=0, wrap=False):
    y = _w(_t(x).clone())
    return y.fill_diagonal_(value, offset, wrap)


@impl("exponential_")
def _exponential_(x, lam=1.0):
    with torch.no_grad():
        _t(x).exponential_(lam)
    return x


@impl("full_")
def _full_(output, shape, value, dtype=None, place=None):
    with torch.no_grad():
        _t(output).fill_(value)
    return output


@impl("uniform_inplace")
def _uniform_inplace(x, min=-1.0, max=1.0, seed=0, diag_num=0, diag_step=0, diag_val=1.0):  # noqa: A002
    with torch.no_grad():
        t = _t(x)
        g = torch.Generator(device=t.device).manual_seed(int(seed)) if seed else None
        t.copy_(torch.rand(t.shape, generator=g, device=t.device, dtype=torch.float32).mul_(max - min).add_(min))
        if diag_num > 0:
            flat = t.view(-1)
            for i in range(diag_num):
                flat[i * (diag_step + 1)] = diag_val
    return x


@impl("gaussian_inplace")
def _gaussian_inplace(x, mean=0.0, std=1.0, seed=0):
    with torch.no_grad():
        t = _t(x)
        g = torch.Generator(device=t.device).manual_seed(int(seed)) if seed else None
        t.copy_(torch.randn(t.shape, generator=g, device=t.device, dtype=torch.float32).mul_(std).add_(mean))
    return x


@impl("segment_pool")
def _segment_pool(x, segment_ids, pooltype="SUM"):
    from . import geometric as G
    fn = {"SUM": G.segment_sum, "MEAN": G.segment_mean, "MAX": G.segment_max, "MIN": G.segment_min}[pooltype.upper()]
    out = fn(x, segment_ids)
    ids = _t(segment_ids).long()
    counts = torch.bincount(ids, minlength=_t(out).shape[0]).to(_t(x).dtype).reshape(-1, 1)
    return out, _w(counts)


@impl("viterbi_decode")
def _viterbi(potentials, transition_params, lengths, include_bos_eos_tag=True):
    from .text import viterbi_decode
    return viterbi_decode(potentials, transition_params, lengths, include_bos_eos_tag)


@impl("update_loss_scaling_")
def _update_loss_scaling_(x, found_infinite, prev_loss_scaling, in_good_steps, in_bad_steps, incr_every_n_steps,
                          decr_every_n_nan_or_inf, incr_ratio, decr_ratio, stop_update=False):
    """Dynamic loss scaling (reference update_loss_scaling_kernel): with an inf/nan the gradients are zeroed, the
    bad-step counter grows and the scale shrinks after decr_every_n_nan_or_inf of them; otherwise the good-step counter
    grows and the scale grows after incr_every_n_steps."""
    found = bool(_t(found_infinite).reshape(-1)[0].item())
    sc, good, bad = _t(prev_loss_scaling), _t(in_good_steps), _t(in_bad_steps)
    with torch.no_grad():
        if found:
            for t in x:
                _t(t).zero_()
        if not (stop_update if not hasattr(stop_update, "_t") else bool(_t(stop_update).item())):
            if found:
                good.zero_()
                bad.add_(1)
                if int(bad.reshape(-1)[0]) >= decr_every_n_nan_or_inf:
                    sc.mul_(decr_ratio).clamp_(min=1.0)
                    bad.zero_()
            else:
                bad.zero_()
                good.add_(1)
                if int(good.reshape(-1)[0]) >= incr_every_n_steps:
                    new = sc * incr_ratio
                    if torch.isfinite(new).all():
                        sc.copy_(new)
                    good.zero_()
    return list(x), prev_loss_scaling, in_good_steps, in_bad_steps


@impl("merged_adam_")
def _merged_adam_(param, grad, learning_rate, moment1, moment2, moment2_max, beta1_pow, beta2_pow, master_param,
                  beta1=0.9, beta2=0.999, epsilon=1e-8, multi_precision=False, use_global_beta_pow=False,
                  amsgrad=False):
    outs = [[] for _ in range(7)]
    n = len(param)
    for i in range(n):
        r = _adam_like(param[i], grad[i], learning_rate[i] if isinstance(learning_rate, (list, tuple))
                       else learning_rate, moment1[i], moment2[i], moment2_max[i] if moment2_max else None,
                       beta1_pow[i], beta2_pow[i], master_param[i] if master_param else None, None, beta1, beta2,
                       epsilon, multi_precision, use_global_beta_pow, amsgrad)
        for j in range(7):
            outs[j].append(r[j])
    return tuple(outs)


@impl("merged_momentum_")
def _merged_momentum_(param, grad, velocity, learning_rate, master_param, mu, use_nesterov=False,
                      regularization_method=(), regularization_coeff=(), multi_precision=False, rescale_grad=1.0):
    outs = ([], [], [])
    for i in range(len(param)):
        rm = regularization_method[i] if regularization_method else ""
        rc = regularization_coeff[i] if regularization_coeff else 0.0
        lr = learning_rate[i] if isinstance(learning_rate, (list, tuple)) and len(learning_rate) > 1 else (
            learning_rate[0] if isinstance(learning_rate, (list, tuple)) else learning_rate)
        r = _momentum_(param[i], grad[i], velocity[i], lr, master_param[i] if master_param else None, mu,
                       use_nesterov, rm, rc, multi_precision, rescale_grad)
        for j in range(3):
            outs[j].append(r[j])
    return outs


@impl("adagrad_")
def _adagrad_(param, grad, moment, learning_rate, master_param, epsilon=1e-6, multi_precision=False):
    lr = _t(learning_rate).float().reshape(-1)[0]
    p = _t(master_param) if (multi_precision and master_param is not None) else _t(param)
    with torch.no_grad():
        g = _t(grad).float()
        mo = _t(moment)
        mf = mo.float() + g * g
        pf = p.float() - lr * g / (torch.sqrt(mf) + epsilon)
        mo.copy_(mf.to(mo.dtype))
        p.copy_(pf.to(p.dtype))
        if multi_precision and master_param is not None:
            _t(param).copy_(pf.to(_t(param).dtype))
    return param, moment, master_param


@impl("adamax_")
def _adamax_(param, grad, learning_rate, moment, inf_norm, beta1_pow, master_param, beta1=0.9, beta2=0.999,
             epsilon=1e-8, multi_precision=False):
    lr = _t(learning_rate).float().reshape(-1)[0]
    p = _t(master_param) if (multi_precision and master_param is not None) else _t(param)
    with torch.no_grad():
        g = _t(grad).float()
        m, u = _t(moment), _t(inf_norm)
        mf = beta1 * m.float() + (1 - beta1) * g
        uf = torch.maximum(beta2 * u.float(), g.abs() + epsilon)
        b1p = _t(beta1_pow).float().reshape(-1)[0]
        pf = p.float() - (lr / (1 - b1p)) * mf / uf
        m.copy_(mf.to(m.dtype))
        u.copy_(uf.to(u.dtype))
        p.copy_(pf.to(p.dtype))
        if multi_precision and master_param is not None:
            _t(param).copy_(pf.to(_t(param).dtype))
    return param, moment, inf_norm, master_param


@impl("adadelta_")
def _adadelta_(param, grad, avg_squared_grad, avg_squared_update, learning_rate, master_param, rho=0.95,
               epsilon=1e-6, multi_precision=False):
    lr = _t(learning_rate).float().reshape(-1)[0]
    p = _t(master_param) if (multi_precision and master_param is not None) else _t(param)
    with torch.no_grad():
        g = _t(grad).float()
        sg, su = _t(avg_squared_grad), _t(avg_squared_update)
        sgf = rho * sg.float() + (1 - rho) * g * g
        upd = -torch.sqrt((su.float() + epsilon) / (sgf + epsilon)) * g
        suf = rho * su.float() + (1 - rho) * upd * upd
        pf = p.float() + lr * upd
        sg.copy_(sgf.to(sg.dtype))
        su.copy_(suf.to(su.dtype))
        p.copy_(pf.to(p.dtype))
        if multi_precision and master_param is not None:
            _t(param).copy_(pf.to(_t(param).dtype))
    return param, avg_squared_grad, avg_squared_update, master_param


@impl("rmsprop_")
def _rmsprop_(param, mean_square, grad, moment, learning_rate, mean_grad, master_param, epsilon=1e-10, decay=0.9,
              momentum=0.0, centered=False, multi_precision=False):
    lr = _t(learning_rate).float().reshape(-1)[0]
    p = _t(master_param) if (multi_precision and master_param is not None) else _t(param)
    with torch.no_grad():
        g = _t(grad).float()
        ms, mo = _t(mean_square), _t(moment)
        msf = decay * ms.float() + (1 - decay) * g * g
        if centered and mean_grad is not None:
            mg = _t(mean_grad)
            mgf = decay * mg.float() + (1 - decay) * g
            denom = msf - mgf * mgf + epsilon
            mg.copy_(mgf.to(mg.dtype))
        else:
            denom = msf + epsilon
        mof = momentum * mo.float() + lr * g / torch.sqrt(denom)
        pf = p.float() - mof
        ms.copy_(msf.to(ms.dtype))
        mo.copy_(mof.to(mo.dtype))
        p.copy_(pf.to(p.dtype))
        if multi_precision and master_param is not None:
            _t(param).copy_(pf.to(_t(param).dtype))
    return param, moment, mean_square, mean_grad, master_param


@impl("lamb_")
def _lamb_(param, grad, learning_rate, moment1, moment2, beta1_pow, beta2_pow, master_param, skip_update,
           weight_decay, beta1=0.9, beta2=0.999, epsilon=1e-6, always_adapt=False, multi_precision=False):
    if skip_update is not None and bool(_t(skip_update).reshape(-1)[0].item()):
        return param, moment1, moment2, beta1_pow, beta2_pow, master_param
    lr = _t(learning_rate).float().reshape(-1)[0]
    p = _t(master_param) if (multi_precision and master_param is not None) else _t(param)
    with torch.no_grad():
        g = _t(grad).float()
        m, v = _t(moment1), _t(moment2)
        b1p, b2p = _t(beta1_pow).float().reshape(-1)[0], _t(beta2_pow).float().reshape(-1)[0]
        mf = beta1 * m.float() + (1 - beta1) * g
        vf = beta2 * v.float() + (1 - beta2) * g * g
        r = (mf / (1 - b1p)) / (torch.sqrt(vf / (1 - b2p)) + epsilon) + weight_decay * p.float()
        pn, rn = torch.linalg.vector_norm(p.float()), torch.linalg.vector_norm(r)
        trust = torch.where((pn > 0) & (rn > 0), pn / rn, torch.ones_like(pn)) if (weight_decay or always_adapt) \
            else torch.ones_like(pn)
        pf = p.float() - lr * trust * r
        m.copy_(mf.to(m.dtype))
        v.copy_(vf.to(v.dtype))
        p.copy_(pf.to(p.dtype))
        if multi_precision and master_param is not None:
            _t(param).copy_(pf.to(_t(param).dtype))
        _t(beta1_pow).mul_(beta1)
        _t(beta2_pow).mul_(beta2)
    return param, moment1, moment2, beta1_pow, beta2_pow, master_param


# ---- collectives (ring_id -> the communication group of that id; 0 = the global group)
def _group(ring_id):
    from .distributed.collective import get_group
    return get_group(int(ring_id)) if ring_id else None


def _reduce_op(t):
    from .distributed import ReduceOp
    return {0: ReduceOp.SUM, 1: ReduceOp.MAX, 2: ReduceOp.MIN, 3: ReduceOp.PROD, 4: getattr(ReduceOp, "AVG",
                                                                                            ReduceOp.SUM)}[int(t)]


def _allreduce_copy(x, ring_id, op):
    from . import distributed as D
    y = _w(_t(x).clone())
    D.all_reduce(y, op=op, group=_group(ring_id))
    return y


@impl("all_reduce")
def _all_reduce(x, ring_id=0, reduce_type=0):
    return _allreduce_copy(x, ring_id, _reduce_op(reduce_type))


for _nm, _rt in (("c_allreduce_sum", 0), ("c_allreduce_max", 1), ("c_allreduce_min", 2), ("c_allreduce_prod", 3)):
    def _mk(rt):
        def f(x, ring_id=0, use_calc_stream=False, use_model_parallel=False):
            return _allreduce_copy(x, ring_id, _reduce_op(rt))
        return f
    _IMPL[_nm] = _mk(_rt)


@impl("mp_allreduce_sum")
def _mp_allreduce_sum(x, ring_id=0):
    return _allreduce_copy(x, ring_id, _reduce_op(0))


@impl("all_gather", "c_allgather")
def _all_gather(x, ring_id=0, nranks=1, use_calc_stream=False):
    from . import distributed as D
    parts = []
    D.all_gather(parts, x, group=_group(ring_id))
    return _w(torch.cat([_t(p) for p in parts], 0))


@impl("c_concat")
def _c_concat(x, rank=0, nranks=1, ring_id=0, use_calc_stream=False, use_model_parallel=True):
    from . import distributed as D
    parts = []
    D.all_gather(parts, x, group=_group(ring_id))
    return _w(torch.cat([_t(p) for p in parts], -1))


@impl("c_identity")
def _c_identity(x, ring_id=0, use_calc_stream=False, use_model_parallel=True):
    return _w(_t(x).clone())


@impl("broadcast", "c_broadcast")
def _broadcast(x, ring_id=0, root=0, use_calc_stream=False):
    from . import distributed as D
    y = _w(_t(x).clone())
    D.broadcast(y, src=int(root), group=_group(ring_id))
    return y


@impl("reduce", "c_reduce_sum")
def _reduce(x, ring_id=0, root_id=0, reduce_type=0, use_calc_stream=False):
    from . import distributed as D
    y = _w(_t(x).clone())
    D.reduce(y, dst=int(root_id), op=_reduce_op(reduce_type), group=_group(ring_id))
    return y


@impl("reduce_scatter")
def _reduce_scatter(x, ring_id=0, nranks=1):
    from . import distributed as D
    xt = _t(x)
    n = max(int(nranks), 1)
    out = _w(torch.empty((xt.shape[0] // n,) + tuple(xt.shape[1:]), dtype=xt.dtype, device=xt.device))
    D.reduce_scatter(out, [_w(c) for c in xt.chunk(n, 0)], group=_group(ring_id))
    return out


@impl("all_to_all")
def _all_to_all(x, ring_id=0):
    from . import distributed as D
    xt = _t(x)
    g = _group(ring_id)
    n = D.get_world_size(g) if g is not None else D.get_world_size()
    outs = []
    D.alltoall(outs, [_w(c.contiguous()) for c in xt.chunk(n, 0)], group=g)
    return _w(torch.cat([_t(o) for o in outs], 0))


@impl("c_embedding")
def _c_embedding(weight, x, start_index=0, vocab_size=-1):
    """Vocab-parallel lookup on this rank's rows [start_index, start_index + rows): ids outside give zero rows."""
    w, ids = _t(weight), _t(x).long()
    local = ids - int(start_index)
    mask = (local < 0) | (local >= w.shape[0])
    emb = torch.nn.functional.embedding(local.masked_fill(mask, 0), w)
    return _w(emb.masked_fill(mask.unsqueeze(-1), 0.0))
