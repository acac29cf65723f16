"""Lower a PIR program to the native interpreter (csrc/interpreter/interpreter.cpp, module ``_C_interp``).

Reference: paddle/fluid/framework/new_executor/program_interpreter.cc — the program becomes a flat instruction
list executed in C++ with last-use garbage collection. Lowering here:
  * matmul + bias add (+ GELU) is fused into one ``fused_linear`` instruction (the GEMM epilogue);
  * every PIR value gets a slot; parameters are bound once (persistent), feeds per run, fetch targets kept;
  * ``builtin.combine`` / ``builtin.split`` disappear (their slot lists are spliced into the consumers /
    producers);
  * the reference's mutable attributes (an operand produced by ``pd_op.full`` / ``full_int_array``, e.g. a
    reshape's shape, concat's axis, slice's starts / ends) are folded into instruction attributes;
  * any op outside the interpreter's table makes ``compile_program`` return None, and the caller keeps the
    Python replay (PirRunner)."""
from __future__ import annotations

import numpy as np

# operand index -> attribute name, for the operands that carry the reference's mutable attributes
_MUTABLE = {
    "reshape": {1: "shape"}, "unsqueeze": {1: "axis"}, "squeeze": {1: "axis"}, "concat": {1: "axis"},
    "split": {1: "sections", 2: "axis"}, "split_with_num": {1: "axis"}, "slice": {1: "starts", 2: "ends"},
    "scale": {1: "scale"}, "full_like": {1: "value"}, "sum": {1: "axis"}, "max": {1: "axis"}, "min": {1: "axis"},
    "argmax": {1: "axis"}, "gather": {2: "axis"}, "expand": {1: "shape"}, "tile": {1: "repeat_times"},
    "clip": {1: "min", 2: "max"}, "pool2d": {1: "kernel_size"},
}


def _module():
    try:
        from .. import _C_interp
        return _C_interp
    except ImportError:
        return None


def available():
    return _module() is not None


def _attr_value(v):
    if isinstance(v, (bool, int, float, str)):
        return v
    if isinstance(v, (list, tuple)) and all(isinstance(x, (bool, int, np.integer)) for x in v):
        return [int(x) for x in v]
    if isinstance(v, np.generic):
        return v.item()
    return None


class NativeRunner:
    """Same interface as PirRunner (feed_names / fetch_names / run(feeds)) over the C++ interpreter."""

    def __init__(self, program, interp, feed_slots, fetch_slots):
        self.program = program
        self.interp = interp
        self._feed_slots = feed_slots   # feed name -> slot, in feed order
        self._fetch_slots = fetch_slots

    @property
    def feed_names(self):
        return self.program.feed_names

    @property
    def fetch_names(self):
        return self.program.fetch_names

    def run(self, feeds):
        import torch
        from .tensor import Tensor, _wrap
        items = []
        for k, (name, slot) in enumerate(self._feed_slots):
            v = feeds[name] if isinstance(feeds, dict) else feeds[k]
            t = v._t if isinstance(v, Tensor) else torch.as_tensor(np.asarray(v))
            items.append((slot, t.to(self.device) if t.device != self.device else t))
        return [_wrap(t) for t in self.interp.run(items)]


def _fuse_linear(ops):
    """Peephole: ``matmul(x, W)`` whose only reader is ``add(., bias)`` with a 1-D parameter bias (and, when that
    sum's only reader is ``gelu``, the activation too) becomes one ``fused_linear`` instruction: the MFMA GEMM
    with its bias / GELU epilogue (reference: the fused_gemm_epilogue pass, fuse_gemm_epilogue_pass.cc)."""
    from .pir_json import decode_type
    uses, producer = {}, {}
    for i, (name, operands, results, attrs, types) in enumerate(ops):
        for v in operands:
            uses.setdefault(v, []).append(i)
        for k, r in enumerate(results):
            producer[r] = (i, k)
    param_shape = {}
    for name, operands, results, attrs, types in ops:
        if name == "builtin.parameter":
            t = decode_type(types[0]) if types and types[0] else None
            param_shape[results[0]] = t[1] if isinstance(t, tuple) else None
    out = list(ops)
    dead = set()
    for i, (name, operands, results, attrs, types) in enumerate(ops):
        if name != "pd_op.matmul" or attrs.get("transpose_x") or len(uses.get(results[0], [])) != 1:
            continue
        j = uses[results[0]][0]
        an, aops, ares, _, atypes = ops[j]
        if an != "pd_op.add" or len(aops) != 2:
            continue
        bias = aops[1] if aops[0] == results[0] else aops[0]
        if len(param_shape.get(bias) or []) != 1 or (len(param_shape.get(operands[1]) or []) != 2):
            continue
        fa = {"transpose_y": bool(attrs.get("transpose_y", False)), "activation": "none"}
        res, tys, at = ares, atypes, j
        users = uses.get(ares[0], [])
        if len(users) == 1 and ops[users[0]][0] == "pd_op.gelu":
            g = users[0]
            fa["activation"] = "gelu"
            fa["approximate"] = bool(ops[g][3].get("approximate", False))
            res, tys, at = ops[g][2], ops[g][4], g
            dead.add(j)
        dead.add(i)
        out[at] = ("pd_op.fused_linear", [operands[0], operands[1], bias], res, fa, tys)
    return [op for k, op in enumerate(out) if k not in dead]


def compile_program(program, params, device):
    """PirProgram + {name: Tensor} -> NativeRunner, or None when an op has no native kernel."""
    m = _module()
    if m is None:
        return None
    supported = set(m.supported_ops())
    slot_of = {}
    lists = {}       # builtin.combine result -> [slots]
    consts = {}      # value id -> python constant (full / full_int_array results)

    def slot(v):
        if v not in slot_of:
            slot_of[v] = len(slot_of)
        return slot_of[v]

    plan = []        # (op, in_slots, out_slots, attrs)
    feed_slots, fetch_slots, bound = [], [], []

    def emit(op, ins, outs, a):
        plan.append((op, ins, outs, a))
        return a

    def lower(ops):
        """Appends the instructions of one block; False when an op has no native mapping."""
        for op in _fuse_linear([o for o in ops if o[0] != "cf.yield"]):
            name, operands, results, attrs, _types = op
            dialect, _, short = name.partition(".")
            if name == "builtin.parameter":
                bound.append((slot(results[0]), params[attrs["parameter_name"]]._t))
                continue
            if name in ("pd_op.data", "pd_op.feed"):
                feed_slots.append((attrs["name"], slot(results[0])))
                continue
            if name in ("pd_op.fetch", "builtin.shadow_output"):
                continue
            if name == "builtin.combine":
                lists[results[0]] = list(operands)
                continue
            if name == "builtin.split":
                lists.setdefault(("split", operands[0]), results)
                continue
            if name == "pd_op.if":
                # jump_if_false -> else; true block; move yields -> results; jump -> end; else: false block; move
                t_blk, f_blk = op.regions
                jf = emit("__jump_if_false", [slot(operands[0])], [], {"target": -1})
                if not lower(t_blk.ops):
                    return False
                emit("__move", [slot(v) for v in t_blk.yields()], [slot(r) for r in results], {})
                je = emit("__jump", [], [], {"target": -1})
                jf["target"] = len(plan)
                if not lower(f_blk.ops):
                    return False
                emit("__move", [slot(v) for v in f_blk.yields()], [slot(r) for r in results], {})
                je["target"] = len(plan)
                continue
            if name == "pd_op.while":
                # args <- loop values, c <- cond; top: jump_if_false c -> exit; body; (c, args) <- yields;
                # jump -> top; exit: results <- args
                body = op.regions[0]
                c = slot(("while_cond", id(op)))
                emit("__move", [slot(v) for v in operands[1:]] + [slot(operands[0])],
                     [slot(a) for a in body.args] + [c], {})
                top = len(plan)
                jf = emit("__jump_if_false", [c], [], {"target": -1})
                if not lower(body.ops):
                    return False
                y = body.yields()
                emit("__move", [slot(v) for v in y], [c] + [slot(a) for a in body.args], {})
                emit("__jump", [], [], {"target": top})
                jf["target"] = len(plan)
                emit("__move", [slot(a) for a in body.args], [slot(r) for r in results], {})
                continue
            if dialect != "pd_op" or short not in supported:
                return False
            a = {k: _attr_value(v) for k, v in attrs.items()}
            a = {k: v for k, v in a.items() if v is not None}
            if short == "full":
                consts[results[0]] = a.get("value", 0.0)
            elif short == "full_int_array":
                consts[results[0]] = [int(x) for x in (a.get("value") or [])]
            mut = _MUTABLE.get(short, {})
            ins = []
            for i, v in enumerate(operands):
                if i in mut:
                    if v not in consts:
                        return False  # a data-dependent shape / axis: keep the Python replay
                    a[mut[i]] = consts[v]
                    continue
                if v == 0:
                    ins.append(-1)
                elif v in lists:  # a combined operand list (concat / stack inputs)
                    ins.extend(slot(x) for x in lists[v])
                else:
                    ins.append(slot(v))
            outs = []
            for r in results:
                split = lists.get(("split", r))
                if split is not None:
                    outs.extend(slot(x) for x in split)
                else:
                    outs.append(slot(r))
            if short in ("pool2d",) and "kernel_size" in a and not isinstance(a["kernel_size"], list):
                a["kernel_size"] = [int(a["kernel_size"])] * 2
            for key in ("axis",):
                if short in ("concat", "split", "split_with_num", "gather", "argmax") and isinstance(a.get(key), list):
                    a[key] = a[key][0] if a[key] else 0
            emit(short, ins, outs, a)
        return True

    if not lower(program.ops):
        return None
    # builtin.split results whose producer was not a multi-output op stay unresolved
    fetch_slots = [slot(v) for _, v in program.fetch]
    dev = str(device)
    interp = m.Interpreter(len(slot_of), dev)
    for op, ins, outs, a in plan:
        interp.add(op, ins, outs, a)
    for s, t in bound:
        interp.bind(s, t.to(device) if t.device != device else t)
    interp.finalize([s for s, _ in bound], fetch_slots)
    r = NativeRunner(program, interp, feed_slots, fetch_slots)
    r.device = device
    return r


def kernel_calls():
    """Launches of the hand-written HIP kernels made by native interpreters in this process, per kind."""
    m = _module()
    return dict(m.kernel_calls()) if m is not None and hasattr(m, "kernel_calls") else {}


def reset_kernel_calls():
    m = _module()
    if m is not None and hasattr(m, "reset_kernel_calls"):
        m.reset_kernel_calls()
