"""Run-time half of the AST dy2static conversion: the functions the rewritten source calls in place of
Python ``if`` / ``while`` / ``for range`` / ``and`` / ``or`` / ``not`` / ``len`` / ``assert``.

Reference behaviour: python/paddle/jit/dy2static/convert_operators.py:167 (convert_while_loop), :398
(convert_ifelse), :270/321/372 (logical ops), :607 (convert_len), :784 (convert_assert).

Each helper looks at what it is given. Python values and concrete (device) tensors keep Python semantics, so a
converted function runs unchanged in dygraph. Traced values of a static program being recorded (meta tensors,
static/program.py) turn the statement into ONE control-flow node with sub-blocks (program.CFNode): ``if``
records both branches and the replay runs the taken one; ``while`` records the condition and the body over
loop-variable slots and the replay iterates on device values. Branch and body functions take the variables
they assign as arguments and return their new values (the transformer's calling convention, transformer.py),
so a variable first assigned inside a branch / body arrives as an ``UndefinedVar``.
"""
from __future__ import annotations

import numbers

import torch

from ...framework.tensor import Tensor, _wrap

__all__ = ["UndefinedVar", "Vars", "convert_ifelse", "convert_ifexp", "convert_while_loop", "convert_logical_and",
           "convert_logical_or", "convert_logical_not", "convert_len", "convert_assert", "convert_range_cond",
           "convert_shape", "convert_var_dtype", "convert_attr", "convert_load", "indexable", "unpack_by_structure",
           "to_static_variable", "create_bool_as_type", "Dygraph2StaticException"]


class Dygraph2StaticException(Exception):
    """A construct the converted program cannot express (e.g. a variable bound in only one branch of a
    tensor-predicated ``if`` and read afterwards)."""


class UndefinedVar:
    """Value of a name that is not bound on the path taken so far (reference: dy2static utils.UndefinedVar)."""
    __slots__ = ("name",)

    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return f"UndefinedVar({self.name!r})"

    def _fail(self, *a, **k):
        raise Dygraph2StaticException(
            f"variable '{self.name}' is not defined on every path of the converted control flow (it is bound in "
            "only one branch of a tensor-dependent if, or only inside a tensor-dependent loop body)")

    __bool__ = __call__ = __getattr__ = __add__ = __radd__ = __mul__ = __rmul__ = __sub__ = __rsub__ = _fail
    __truediv__ = __getitem__ = __iter__ = __len__ = __neg__ = __lt__ = __le__ = __gt__ = __ge__ = _fail

    def __eq__(self, other):
        return other is self

    def __hash__(self):
        return id(self)


def Vars(scope, names):
    """Current values of ``names`` in ``scope`` (a ``locals()`` snapshot); unbound names -> UndefinedVar."""
    return tuple(scope[n] if n in scope else UndefinedVar(n) for n in names)


# ----------------------------------------------------------------------------------------------- helpers
def _static(x):
    return isinstance(x, Tensor) and x._t.device.type == "meta"


def _prog():
    from ...framework.trace_hook import _active_program
    return _active_program()


def _as_pred(pred):
    if pred.numel() != 1:
        raise Dygraph2StaticException(f"the predicate of a tensor-dependent if / while must hold one element, got "
                                      f"shape {list(pred.shape)}")
    p = pred.reshape([])
    if p._t.dtype != torch.bool:
        p = p != 0
    return p


def _py_truth(x):
    if isinstance(x, Tensor):
        return bool(x._t.reshape(()).item())
    return bool(x)


def _const_like(v, other):
    """A Python number as a constant tensor of ``other``'s shape / dtype (a branch that sets a tensor variable
    in one arm and a number in the other)."""
    with torch._C.DisableTorchFunction():
        return _wrap(torch.full(tuple(other._t.shape), v, dtype=other._t.dtype))


def _merge_branch(i, a, b, names):
    """Merge rule for output ``i`` of the two branches -> (kind, a', b').
    kind: 'tensor' (both tensors after number promotion), 'same' (identical non-tensor), 'undef' (bound in one
    branch only: stays undefined after the if and fails when read)."""
    nm = names[i] if names and i < len(names) else f"#{i}"
    if isinstance(a, UndefinedVar) or isinstance(b, UndefinedVar):
        if isinstance(a, UndefinedVar) and isinstance(b, UndefinedVar):
            return "same", a, b
        return "undef", None, None
    ta, tb = isinstance(a, Tensor), isinstance(b, Tensor)
    if ta and not tb and isinstance(b, numbers.Number):
        b, tb = _const_like(b, a), True
    elif tb and not ta and isinstance(a, numbers.Number):
        a, ta = _const_like(a, b), True
    if ta and tb:
        if list(a.shape) != list(b.shape):
            raise Dygraph2StaticException(f"variable '{nm}' gets shape {list(a.shape)} in the true branch and "
                                          f"{list(b.shape)} in the false branch of a tensor-dependent if")
        if a._t.dtype != b._t.dtype:
            raise Dygraph2StaticException(f"variable '{nm}' gets dtype {a._t.dtype} in the true branch and "
                                          f"{b._t.dtype} in the false branch of a tensor-dependent if")
        return "tensor", a, b
    if ta or tb:
        raise Dygraph2StaticException(f"variable '{nm}' is a Tensor in one branch of a tensor-dependent if and "
                                      f"{type(b if ta else a).__name__} in the other")
    if isinstance(a, bool) and isinstance(b, bool) and a != b:
        # a flag set in one branch only (break / continue lowering, or user flags): a bool tensor after the if
        with torch._C.DisableTorchFunction():
            return "tensor", _wrap(torch.tensor(a)), _wrap(torch.tensor(b))
    try:
        same = a is b or bool(a == b)
    except Exception:
        same = False
    if not same:
        raise Dygraph2StaticException(f"variable '{nm}' takes different Python values in the two branches of a "
                                      f"tensor-dependent if ({a!r} / {b!r}); make it a Tensor")
    return "same", a, b


def _t(x):
    return x._t if isinstance(x, Tensor) else x


# ------------------------------------------------------------------------------------------------- if / else
def convert_ifelse(pred, true_fn, false_fn, args=(), names=None):
    """``if pred: ... else: ...`` — the branch functions take ``args`` (the current values of the variables the
    statement assigns) and return their new values as a tuple (or the statement's return value)."""
    if _static(pred):
        return _static_ifelse(pred, true_fn, false_fn, args, names)
    return true_fn(*args) if _py_truth(pred) else false_fn(*args)


def convert_ifexp(pred, true_fn, false_fn):
    """``a if pred else b``."""
    if _static(pred):
        return _static_ifelse(pred, true_fn, false_fn, (), None)
    return true_fn() if _py_truth(pred) else false_fn()


def _static_ifelse(pred, true_fn, false_fn, args, names):
    from ...static.program import CFNode, _SubBlock
    prog = _prog()
    if prog is None:
        raise Dygraph2StaticException("a traced tensor predicate outside of a program being recorded")
    p = _as_pred(pred)
    with prog._sub_block() as tb:
        t = true_fn(*args)
    with prog._sub_block() as fb:
        f = false_fn(*args)
    ts, fs = [], []
    spec = _flatten_pair(t, f, ts, fs)
    leaf_names = _leaf_names(t, names)
    kinds, ra, rb = [], [], []
    for i, (a, b) in enumerate(zip(ts, fs)):
        k, a2, b2 = _merge_branch(i, a, b, leaf_names)
        kinds.append(k)
        if k == "tensor":
            # number promotions created in this scope are constants (no node): template them per branch
            ra.append(_t(a2))
            rb.append(_t(b2))
    res = [prog._template(ra), prog._template(rb)]
    with torch._C.DisableTorchFunction():
        metas = [torch.empty(x.shape, dtype=x.dtype, device="meta") for x in ra]
    node = CFNode("cond", (prog._template(p._t),), prog._out_template(metas), [_SubBlock(tb), _SubBlock(fb)], res)
    prog._append(node)
    outs, j = [], 0
    for i, (k, a) in enumerate(zip(kinds, ts)):
        if k == "tensor":
            outs.append(_wrap(metas[j]))
            j += 1
        elif k == "undef":
            outs.append(UndefinedVar(leaf_names[i]))
        else:
            outs.append(a)
    return _unflatten(spec, iter(outs))


def _flatten_pair(a, b, la, lb):
    """Flatten two branch results of the same container structure into leaf lists; returns the structure."""
    if isinstance(a, (list, tuple)) and not isinstance(a, Tensor):
        if not isinstance(b, (list, tuple)) or len(a) != len(b) or type(a) is not type(b):
            raise Dygraph2StaticException("the branches of a tensor-dependent if return different structures "
                                          f"({type(a).__name__} of {len(a)} / {type(b).__name__})")
        return (type(a), [_flatten_pair(x, y, la, lb) for x, y in zip(a, b)])
    if isinstance(a, dict):
        if not isinstance(b, dict) or set(a) != set(b):
            raise Dygraph2StaticException("the branches of a tensor-dependent if return different dict keys")
        return (dict, {k: _flatten_pair(a[k], b[k], la, lb) for k in a})
    la.append(a)
    lb.append(b)
    return None


def _unflatten(spec, it):
    if spec is None:
        return next(it)
    kind, sub = spec
    if kind is dict:
        return {k: _unflatten(v, it) for k, v in sub.items()}
    return kind(_unflatten(v, it) for v in sub)


def _leaf_names(t, names):
    """Display names of the flattened leaves (top-level tuple positions carry the variable names)."""
    out = []

    def walk(x, nm):
        if isinstance(x, (list, tuple)) and not isinstance(x, Tensor):
            for i, v in enumerate(x):
                walk(v, f"{nm}[{i}]")
        elif isinstance(x, dict):
            for k, v in x.items():
                walk(v, f"{nm}[{k!r}]")
        else:
            out.append(nm)
    if isinstance(t, tuple) and names and len(t) == len(names):
        for v, n in zip(t, names):
            walk(v, n)
    else:
        walk(t, "<value>")
    return out


# ---------------------------------------------------------------------------------------------------- while
def convert_while_loop(cond_fn, body_fn, args=(), names=None):
    """``while cond: body`` — both functions take the loop variables (the names the body assigns); the body
    returns their new values."""
    vals = tuple(args)
    c = cond_fn(*vals)
    while True:
        # a Python loop turns static once a tensor-dependent break flag (or other carried tensor) reaches its
        # test: the remaining iterations become one while node
        if _static(c) or (isinstance(c, Tensor) and any(_static(v) for v in vals)):
            return _static_while(cond_fn, body_fn, vals, names)
        if not _py_truth(c):
            return vals
        vals = tuple(body_fn(*vals))
        c = cond_fn(*vals)


def _loop_init(v):
    if isinstance(v, Tensor):
        return v
    if isinstance(v, bool):
        return _wrap(torch.tensor(v))
    if isinstance(v, numbers.Integral):
        return _wrap(torch.tensor(int(v), dtype=torch.int64))
    if isinstance(v, numbers.Real):
        return _wrap(torch.tensor(float(v), dtype=torch.float32))
    return None


def _static_while(cond_fn, body_fn, vals, names):
    from ...static.program import CFNode, _SubBlock
    prog = _prog()
    if prog is None:
        raise Dygraph2StaticException("a traced loop condition outside of a program being recorded")
    nm = lambda i: names[i] if names and i < len(names) else f"#{i}"  # noqa: E731
    carried = []  # positions of loop-carried variables (bound before the loop)
    init = list(vals)
    for i, v in enumerate(vals):
        if isinstance(v, UndefinedVar):
            continue
        iv = _loop_init(v)
        if iv is None:
            continue  # a non-numeric Python object the body rebinds: body-local in the static loop
        init[i] = iv
        carried.append(i)
    for _attempt in range(2):
        ph = {i: _wrap(prog._new_like(init[i]._t)) for i in carried}
        slots = [prog._slot_of[id(ph[i]._t)] for i in carried]
        cur = tuple(ph[i] if i in ph else vals[i] for i in range(len(vals)))
        with prog._sub_block() as cb:
            c = cond_fn(*cur)
            if isinstance(c, Tensor):
                c = _as_pred(c)
        with prog._sub_block() as bb:
            out = tuple(body_fn(*cur))
        if len(out) != len(vals):
            raise Dygraph2StaticException(f"loop body returned {len(out)} values for {len(vals)} variables")
        new = []
        retry = False
        for i in carried:
            o = out[i]
            if isinstance(o, numbers.Number):
                o = _const_like(o, init[i])
            if not isinstance(o, Tensor):
                raise Dygraph2StaticException(f"loop variable '{nm(i)}' becomes {type(o).__name__} in the body of "
                                              "a tensor-dependent loop")
            if list(o.shape) != list(init[i].shape):
                raise Dygraph2StaticException(f"loop variable '{nm(i)}' changes shape {list(init[i].shape)} -> "
                                              f"{list(o.shape)} in a tensor-dependent loop")
            if o._t.dtype != init[i]._t.dtype:
                # promote the initial value (e.g. an int counter accumulating floats) and record the loop again
                init[i] = init[i].astype(o._t.dtype) if _static(init[i]) else _wrap(init[i]._t.to(o._t.dtype))
                retry = True
            new.append(o)
        if not retry:
            break
    else:
        raise Dygraph2StaticException("loop variable dtypes do not settle in a tensor-dependent loop")
    if not isinstance(c, Tensor):
        raise Dygraph2StaticException("the condition of a tensor-dependent loop must stay a Tensor")
    res = [prog._template(c._t), prog._template([o._t for o in new])]
    with torch._C.DisableTorchFunction():
        metas = [torch.empty(init[i]._t.shape, dtype=init[i]._t.dtype, device="meta") for i in carried]
    node = CFNode("while", prog._template([init[i]._t for i in carried]), prog._out_template(metas),
                  [_SubBlock(cb), _SubBlock(bb)], res, slots)
    prog._append(node)
    result = list(vals)
    for j, i in enumerate(carried):
        result[i] = _wrap(metas[j])
    for i, v in enumerate(vals):
        if i not in carried and not isinstance(v, UndefinedVar) and isinstance(out[i], Tensor) and _static(out[i]):
            result[i] = UndefinedVar(nm(i))  # a body-local tensor: its last value is not carried out of the loop
    return tuple(result)


def convert_range_cond(i, stop, step):
    """Loop test of a converted ``for i in range(start, stop, step)``."""
    if isinstance(step, Tensor) and not _static(step):
        step = int(step)
    if isinstance(step, numbers.Number):
        return i < stop if step > 0 else i > stop
    return ((step > 0) & (i < stop)) | ((step < 0) & (i > stop))


# ----------------------------------------------------------------------------------------------- logical ops
def convert_logical_and(x_fn, y_fn):
    x = x_fn()
    if _static(x):
        y = y_fn()
        return x.astype("bool") & (y.astype("bool") if isinstance(y, Tensor) else bool(y))
    if not _py_truth(x):
        return x
    return y_fn()


def convert_logical_or(x_fn, y_fn):
    x = x_fn()
    if _static(x):
        y = y_fn()
        return x.astype("bool") | (y.astype("bool") if isinstance(y, Tensor) else bool(y))
    if _py_truth(x):
        return x
    return y_fn()


def convert_logical_not(x):
    if _static(x):
        return x.astype("bool").logical_not()
    return not _py_truth(x)


# ---------------------------------------------------------------------------------------------------- misc
def convert_len(x):
    if isinstance(x, Tensor):
        return x.shape[0]
    return len(x)


def convert_assert(cond, message=""):
    if _static(cond):
        return None  # a static assert needs the data: checked eagerly only (reference: Assert op in dygraph)
    if isinstance(cond, Tensor):
        assert _py_truth(cond), message
    else:
        assert cond, message
    return None


def convert_shape(x):
    return x.shape if isinstance(x, Tensor) else getattr(x, "shape", x)


def convert_var_dtype(var, dtype):
    if isinstance(var, Tensor):
        return var.astype({"bool": "bool", "int": "int64", "float": "float32"}[dtype])
    return {"bool": bool, "int": int, "float": float}[dtype](var)


def convert_attr(x, attr):
    return getattr(x, attr)


def convert_load(x):
    return x


def indexable(x, code=None):
    return x if isinstance(x, (Tensor, list, tuple, dict, str)) else list(x)


def unpack_by_structure(target, structure):
    if structure == 1:
        return target
    return [target[i] for i in range(structure)] if isinstance(structure, int) else target


def to_static_variable(x, dtype=None):
    if isinstance(x, Tensor):
        return x
    iv = _loop_init(x)
    return iv if iv is not None else x


def create_bool_as_type(x, value=True):
    if isinstance(x, Tensor):
        return _wrap(torch.full((), value, dtype=torch.bool))
    return value
