"""paddle._legacy_C_ops: the legacy (fluid operator) eager entry points of the reference
(paddle/fluid/pybind/eager_legacy_op_function_generator.cc), called as ``op(input, ..., 'attr', value, ...)``:
the tensor inputs first, then attribute name / value pairs.

Each call is mapped onto ``_C_ops``: legacy operator names to their phi names (elementwise_add -> add,
matmul_v2 -> matmul, reshape2 -> reshape, ...), the inputs onto the op's yaml tensor arguments in order, the
attributes onto yaml arguments by name (with the legacy attribute renames below); attributes the op does not take
are accepted when they only steer the reference's execution (use_calc_stream, use_mkldnn, ...). Names that are
not operators resolve to the public function of that name, as before.
"""
from __future__ import annotations

from . import _C_ops
from ._c_ops_sigs import SIGS

_OP = {"elementwise_add": "add", "elementwise_sub": "subtract", "elementwise_mul": "multiply",
       "elementwise_div": "divide", "elementwise_max": "maximum", "elementwise_min": "minimum",
       "elementwise_pow": "elementwise_pow", "matmul_v2": "matmul", "reshape2": "reshape", "transpose2": "transpose",
       "squeeze2": "squeeze", "unsqueeze2": "unsqueeze", "flatten_contiguous_range": "flatten",
       "lookup_table_v2": "embedding", "reduce_sum": "sum", "reduce_mean": "mean", "reduce_max": "max",
       "reduce_min": "min", "reduce_prod": "prod", "fill_constant": "full", "softmax_with_cross_entropy":
       "cross_entropy_with_softmax", "top_k_v2": "topk", "arg_max": "argmax", "arg_min": "argmin",
       "expand_v2": "expand", "gaussian_random": "gaussian", "uniform_random": "uniform"}

# legacy attribute name -> yaml argument name, per phi op ("*" = every op)
_ATTR = {"*": {"axes": "axis", "dim": "axis", "keep_dim": "keepdim", "in_dtype": None, "out_dtype": "dtype",
               "use_mkldnn": None, "use_calc_stream": None, "use_model_parallel": None, "op_role": None,
               "op_device": None, "op_namescope": None, "op_callstack": None, "with_quant_attr": None,
               "mkldnn_data_type": None, "use_cudnn": None, "data_format": "data_format", "reduce_all": None},
         "matmul": {"trans_x": "transpose_x", "trans_y": "transpose_y"},
         "dropout": {"dropout_prob": "p", "dropout_implementation": "mode"},
         "transpose": {"axis": "perm"},
         "full": {"value": "value", "str_value": None},
         "cross_entropy_with_softmax": {}}

_PASSTHROUGH = {"use_calc_stream", "use_model_parallel", "use_mkldnn", "op_role", "op_device", "op_namescope",
                "op_callstack", "with_quant_attr", "mkldnn_data_type", "use_cudnn", "in_dtype", "reduce_all",
                "str_value"}


def _legacy(name):
    inplace = name.endswith("_") and name[:-1] in (set(_OP) | set(SIGS))
    base = name[:-1] if inplace else name
    op = _OP.get(base, base)
    if op not in SIGS:
        return None
    sig = SIGS[op][0]
    tensor_args = [n for n, kind, _ in sig if kind.startswith("Tensor")]
    ren = dict(_ATTR["*"])
    ren.update(_ATTR.get(op, {}))
    target = getattr(_C_ops, op + "_") if inplace and SIGS[op][3] else getattr(_C_ops, op)

    def f(*args):
        inputs, i = [], 0
        while i < len(args) and not isinstance(args[i], str):
            inputs.append(args[i])
            i += 1
        rest = args[i:]
        if len(rest) % 2:
            raise TypeError(f"_legacy_C_ops.{name}: attributes must come as name / value pairs")
        kw = dict(zip(tensor_args, inputs))
        names = {n for n, _, _ in sig}
        for k, v in zip(rest[::2], rest[1::2]):
            if base.startswith("elementwise_") and k == "axis" and v == -1:
                continue  # numpy broadcasting, the only form the phi op has
            k2 = ren.get(k, k)
            if k2 is None or (k2 not in names and k in _PASSTHROUGH):
                continue
            if k2 not in names:
                raise TypeError(f"_legacy_C_ops.{name}: attribute {k!r} has no counterpart in _C_ops.{op}")
            kw[k2] = v
        return target(**kw)
    f.__name__ = name
    return f


def __getattr__(name):
    if name.startswith("__"):
        raise AttributeError(name)
    fn = _legacy(name)
    if fn is not None:
        return fn
    return getattr(_C_ops, name)
