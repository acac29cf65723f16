"""Finding and rewriting the quantizable ops of a static Program (conv2d / linear / matmul nodes whose weight is
a program constant)."""
from __future__ import annotations

import torch

from .. import program as P

# op name suffix -> (reference op type, weight channel axis)
_QUANTIZABLE = {
    "conv2d": ("conv2d", 0),
    "conv1d": ("conv2d", 0),
    "conv3d": ("conv3d", 0),
    "fused_linear": ("mul", -1),
    "linear": ("mul", 0),
    "matmul": ("matmul", -1),
    "mm": ("mul", -1),
}


def quantizable_nodes(prog, op_types=None):
    """[(index, node, ref_type, weight const template, channel axis)] of the top-level nodes."""
    out = []
    for i, n in enumerate(prog.nodes):
        if isinstance(n, P.GuardNode) or not n.args:
            continue
        short = n.name.rsplit(":", 1)[-1]
        spec = _QUANTIZABLE.get(short)
        if spec is None:
            continue
        ref_type, axis = spec
        if op_types is not None and ref_type not in op_types and not (
                ref_type == "conv2d" and "depthwise_conv2d" in op_types):
            continue
        if len(n.args) < 2 or not isinstance(n.args[0], P._Ref):
            continue
        w = n.args[1]
        if not isinstance(w, P._Const) or not torch.is_floating_point(w.t) or w.t.dim() < 2:
            continue
        out.append((i, n, ref_type, w, axis))
    return out


def raw():
    """Graph edits run outside the static-mode tracer (TorchFunctionMode): the tensors they create are not ops."""
    return torch._C.DisableTorchFunction()


def insert_before(prog, node, func, extra_args, arg_pos=0):
    """Inserts ``func(node.args[arg_pos], *extra_args)`` ahead of ``node`` and rewires that argument to it."""
    src = node.args[arg_pos]
    with raw():
        if isinstance(src, P._Ref):
            new_meta = torch.empty_like(prog._metas[src.i])
        else:  # a constant (weight): the new value is traced like an activation
            new_meta = torch.empty_like(src.t, device="meta")
    out = prog._out_template(new_meta)
    q = P.OpNode(func, (src,) + tuple(extra_args), {}, out)
    args = list(node.args)
    args[arg_pos] = out
    node.args = tuple(args)
    idx = next(i for i, n in enumerate(prog.nodes) if n is node)
    prog.nodes.insert(idx, q)
    prog._version += 1
    prog._plans.clear()
    return q


def const_of(prog, t):
    return prog._const(t)
