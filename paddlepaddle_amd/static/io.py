"""Static-graph persistence. Reference: python/paddle/static/io.py (save_inference_model:458,
load_inference_model:777, save/load:1467/1540, serialize_program, deserialize_program...).

On-disk format (ours, not protobuf): ``<prefix>.pdmodel`` is a JSON program (see
``Program.to_dict``) and ``<prefix>.pdiparams`` holds the parameters in the reference save_combine binary
layout (framework/combine_io.py; names in the program's "params" list, sorted) — previously a ``paddle.save``
dict name -> ndarray of every
parameter / captured constant. Both load without executing anything from the files.
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from ..framework.tensor import Tensor, Parameter, _wrap
from ..framework import io as _io
from . import program as P
from .executor import _slot_of, default_main_program


def _const_names(prog):
    names, used = [], set()
    params = {id(p._t): p for p in prog.all_parameters()}
    alias = prog.__dict__.get("_const_alias", {})  # names of a deserialized / loaded program's persistables
    for i, t in enumerate(prog._consts):
        p = params.get(id(t))
        n = p.name if p is not None else alias.get(i, f"__const_{i}")
        while n in used:
            n = n + "_"
        used.add(n)
        names.append(n)
    return names


def _used_consts(prog, plan_nodes):
    used = set()

    def walk(x):
        if isinstance(x, P._Const):
            used.add(x.idx)
        elif isinstance(x, (list, tuple)):
            for v in x:
                walk(v)
        elif isinstance(x, dict):
            for v in x.values():
                walk(v)
    def node(n):
        walk((n.args, getattr(n, "kwargs", None)))
        if isinstance(n, P.CFNode):
            # constants read inside a cond / while body or returned by it (e.g. a branch's literal result)
            walk(n.res)
            for b in n.blocks:
                for x in b.nodes:
                    node(x)
    for n in plan_nodes:
        node(n)
    return used


def _prune(prog, fetch_slots):
    plan = P.build_plan(prog, fetch_slots)
    q = P.Program.__new__(P.Program)
    q.__dict__.update(prog.__dict__)
    q.nodes = [prog.nodes[i] for i in sorted(plan.order)]
    q._plans = {}
    q._optimize = None
    return q


def _pruned(feed_vars, fetch_vars, program):
    prog = program or default_main_program()
    fetch = [_slot_of(prog, v) for v in (fetch_vars if isinstance(fetch_vars, (list, tuple)) else [fetch_vars])]
    q = _prune(prog, fetch)
    feeds = [v if isinstance(v, str) else v.name for v in (feed_vars if isinstance(feed_vars, (list, tuple))
                                                            else [feed_vars])]
    q.feeds = {k: v for k, v in prog.feeds.items() if k in feeds}
    return q, fetch


def _persistable_order(prog):
    """(names, const indices) of the persistables a program uses, sorted by name (the reference's order)."""
    names = _const_names(prog)
    used = _used_consts(prog, prog.nodes)
    order = sorted(used, key=lambda i: names[i])
    return [names[i] for i in order], order


def serialize_program(feed_vars, fetch_vars, program=None, **kw):
    """The pruned program as bytes (this framework's program JSON; persistables travel separately through
    serialize_persistables, as in the reference)."""
    q, fetch = _pruned(feed_vars, fetch_vars, program)
    d = q.to_dict(fetch, _const_names(q))
    names, order = _persistable_order(q)
    d["params"] = names
    d["param_meta"] = {n: [list(q._consts[i].shape), str(q._consts[i].dtype).replace("torch.", "")]
                       for n, i in zip(names, order)}
    return json.dumps(d).encode()


def serialize_persistables(feed_vars, fetch_vars, executor=None, program=None, **kw):
    """The persistables the pruned program reads, as bytes in the reference save_combine layout (sorted by
    name) — what save_to_file writes and deserialize_persistables reads back."""
    from ..framework.combine_io import combined_bytes
    q, _ = _pruned(feed_vars, fetch_vars, program)
    _, order = _persistable_order(q)
    return combined_bytes([q._consts[i].detach() for i in order])


def save_inference_model(path_prefix, feed_vars, fetch_vars, executor=None, program=None, **kwargs):
    prog = program or default_main_program()
    fetch_vars = fetch_vars if isinstance(fetch_vars, (list, tuple)) else [fetch_vars]
    feed_vars = feed_vars if isinstance(feed_vars, (list, tuple)) else [feed_vars]
    fetch = [_slot_of(prog, v) for v in fetch_vars]
    q = _prune(prog, fetch)
    feeds = [v if isinstance(v, str) else v.name for v in feed_vars]
    q.feeds = {k: prog.feeds[k] for k in feeds}
    fmt = kwargs.get("program_format", "json")
    if fmt == "protobuf":
        # the reference's ProgramDesc .pdmodel + save_combine .pdiparams (framework/program_desc.py)
        from ..framework import program_desc as _pd
        _pd.export(q, fetch, feeds, _const_names(q)).save(path_prefix)
        return
    if fmt == "pir":  # the reference's Paddle 3.x format only: <prefix>.json (PIR) + .pdiparams
        _pir_writer(q, fetch, feeds, kwargs).save(path_prefix)
        return
    # default: this framework's program (<prefix>.pdmodel, every recorded op, hipGraph replay in the Predictor)
    # plus, when every op lowers to reference operations, the PIR <prefix>.json over the same .pdiparams — the
    # file Paddle 3.x's load_inference_model / paddle.inference read
    order = write_program(path_prefix, q, fetch)
    try:
        w = _pir_writer(q, fetch, feeds, kwargs)
    except NotImplementedError:
        return
    if sorted(w.params) == order:
        with open(path_prefix + ".json", "w") as f:
            json.dump(w.to_json(), f)


def _pir_writer(q, fetch, feeds, kwargs):
    from ..framework import program_desc as _pd, pir_json as _pir
    return _pir.from_builder(_pd.export(q, fetch, feeds, _const_names(q)), trainable=kwargs.get("trainable", False))


def write_program(path_prefix, prog, fetch_slots):
    d = os.path.dirname(path_prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    names = _const_names(prog)
    used = _used_consts(prog, prog.nodes)
    order = sorted(used, key=lambda i: names[i])  # the reference writes persistables sorted by name
    d = prog.to_dict(fetch_slots, names)
    d["params"] = [names[i] for i in order]
    with open(path_prefix + ".pdmodel", "w") as f:
        json.dump(d, f)
    # parameters in the reference save_combine layout (framework/combine_io.py)
    from ..framework.combine_io import write_combined
    write_combined(path_prefix + ".pdiparams", [prog._consts[i].detach() for i in order])
    return [names[i] for i in order]


def read_program(path_prefix, device=None, params_file=None):
    with open(path_prefix + ".pdmodel" if not path_prefix.endswith(".pdmodel") else path_prefix) as f:
        d = json.load(f)
    base = path_prefix[:-len(".pdmodel")] if path_prefix.endswith(".pdmodel") else path_prefix
    pfile = params_file or base + ".pdiparams"
    from ..framework.combine_io import is_combined, read_combined
    if is_combined(pfile):
        sd = dict(zip(d.get("params", []), read_combined(pfile)))
    else:  # files written before the save_combine layout: a restricted-unpickler paddle.save dict
        sd = _io.load(pfile)
    consts = {}
    for k, v in sd.items():
        t = v._t if isinstance(v, Tensor) else v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))
        if device is not None:
            t = t.to(device)
        consts[k] = t
    prog, fetch = P.Program.from_dict(d, consts)
    return prog, fetch, consts


def load_inference_model(path_prefix, executor=None, **kwargs):
    """Loads either format: a reference ProgramDesc protobuf ``.pdmodel`` (run by
    framework/program_desc.ProgramDescRunner over this framework's ops; Executor.run accepts it as the
    program) or this framework's JSON program."""
    dev = None
    if executor is not None and executor.place is not None:
        from ..framework.place import to_torch_device
        dev = to_torch_device(executor.place)
    from ..framework import program_desc as _pd, pir_json as _pir
    base = path_prefix
    for ext in (".pdmodel", ".json"):
        if base.endswith(ext):
            base = base[:-len(ext)]
    own = os.path.exists(base + ".pdmodel") and not _pd.is_program_desc(base + ".pdmodel")
    if not own and os.path.exists(base + ".json") and _pir.is_pir_json(base + ".json"):
        runner = _pir.load(base, dev)  # a Paddle 3.x PIR program: run op by op over this framework's ops
        return [runner, list(runner.feed_names), list(runner.fetch_names)]
    if os.path.exists(base + ".pdmodel") and _pd.is_program_desc(base + ".pdmodel"):
        runner = _pd.load(base, dev)
        return [runner, list(runner.program.feed_names), list(runner.program.fetch_names)]
    path_prefix = base
    prog, fetch, _ = read_program(path_prefix, dev)
    feed_names = list(prog.feeds)
    fetch_vars = [P._Var(prog, s, f"fetch_{i}") for i, s in enumerate(fetch)]
    for v, s in zip(fetch_vars, fetch):
        prog._names[v.name] = s
    return [prog, feed_names, fetch_vars]


def save(program, model_path, protocol=4, **configs):
    params = {p.name: p for p in program.all_parameters()}
    _io.save(params, model_path + ".pdparams")
    if program._optimize is not None:
        _io.save(program._optimize[0].state_dict(), model_path + ".pdopt")


def load(program, model_path, executor=None, var_list=None):
    path = model_path if model_path.endswith(".pdparams") else model_path + ".pdparams"
    sd = _io.load(path)
    set_program_state(program, sd)
    opt_path = path[:-len(".pdparams")] + ".pdopt"
    if program._optimize is not None and os.path.exists(opt_path):
        program._optimize[0].set_state_dict(_io.load(opt_path))


def load_program_state(model_path, var_list=None):
    path = model_path if model_path.endswith(".pdparams") else model_path + ".pdparams"
    return {k: (v.numpy() if isinstance(v, Tensor) else np.asarray(v)) for k, v in _io.load(path).items()}


def set_program_state(program, state_dict):
    with torch.no_grad():
        for p in program.all_parameters():
            if p.name in state_dict:
                v = state_dict[p.name]
                v = v._t if isinstance(v, Tensor) else torch.as_tensor(np.asarray(v))
                p._t.copy_(v.to(p._t.dtype))


def save_to_file(path, content):
    with open(path, "wb") as f:
        f.write(content)


def load_from_file(path):
    with open(path, "rb") as f:
        return f.read()


def deserialize_program(data):
    """A Program from serialize_program bytes. Its persistables are zero-filled placeholders of the recorded
    shape / dtype until deserialize_persistables (or load_vars / set_program_state) fills them."""
    d = json.loads(data.decode() if isinstance(data, (bytes, bytearray)) else data)
    consts = {n: torch.zeros(shape, dtype=getattr(torch, dt)) for n, (shape, dt) in d.get("param_meta", {}).items()}
    prog, fetch = P.Program.from_dict(d, consts)
    prog._serialized_params = list(d.get("params", []))
    prog._serialized_fetch = fetch
    return prog


def deserialize_persistables(program, data, executor=None):
    """Fill ``program``'s persistables from serialize_persistables bytes (save_combine layout, sorted names)."""
    from ..framework.combine_io import parse_combined
    tensors = parse_combined(bytes(data))
    names = getattr(program, "_serialized_params", None)
    if names is None:
        names, _ = _persistable_order(program)
    if len(names) != len(tensors):
        raise ValueError(f"{len(tensors)} serialized tensors for {len(names)} persistables of the program")
    by_name = dict(zip(names, tensors))
    cn = _const_names(program)
    with torch.no_grad():
        for i, n in enumerate(cn):
            if n in by_name:
                program._consts[i].copy_(by_name[n].to(program._consts[i].dtype))
    return program


def get_program_persistable_vars(program):
    """The persistable variables (parameters and captured persistable tensors) of ``program``."""
    return list(program.all_parameters())


def get_program_parameter(program):
    return list(program.all_parameters())


def is_persistable(var):
    return bool(getattr(var, "persistable", False)) or isinstance(var, Parameter)


def is_parameter(var):
    return isinstance(var, Parameter)


def _select_vars(main_program, vars, predicate):
    if vars is not None:
        return list(vars)
    prog = main_program or default_main_program()
    pool = list(prog.all_parameters())
    return [v for v in pool if predicate is None or predicate(v)]


def save_vars(executor=None, dirname=None, main_program=None, vars=None, predicate=None, filename=None):
    """Save variables: one file per variable named after it in ``dirname``, or all of them in ``filename`` (the
    reference save_combine layout, in the given order); with neither ``dirname`` nor ``filename`` the combined
    bytes are returned. Reference: static/io.py:1049 save_vars."""
    from ..framework.combine_io import combined_bytes
    vs = _select_vars(main_program, vars, predicate)
    ts = [v._t.detach() if isinstance(v, Tensor) else torch.as_tensor(np.asarray(v)) for v in vs]
    if dirname is None and filename is None:
        return combined_bytes(ts)
    if dirname:
        os.makedirs(dirname, exist_ok=True)
    if filename is not None:
        with open(os.path.join(dirname or "", filename), "wb") as f:
            f.write(combined_bytes(ts))
        return None
    for v, t in zip(vs, ts):
        with open(os.path.join(dirname, v.name), "wb") as f:
            f.write(combined_bytes([t]))
    return None


def load_vars(executor=None, dirname=None, main_program=None, vars=None, predicate=None, filename=None):
    """Inverse of save_vars: fill the variables in place (shapes must match). Reference: static/io.py:1236."""
    from ..framework.combine_io import parse_combined
    vs = _select_vars(main_program, vars, predicate)
    if filename is not None:
        with open(os.path.join(dirname or "", filename), "rb") as f:
            ts = parse_combined(f.read())
        if len(ts) != len(vs):
            raise ValueError(f"{filename} holds {len(ts)} tensors, {len(vs)} variables requested")
    else:
        ts = []
        for v in vs:
            with open(os.path.join(dirname, v.name), "rb") as f:
                ts.append(parse_combined(f.read())[0])
    with torch.no_grad():
        for v, t in zip(vs, ts):
            if tuple(t.shape) != tuple(v._t.shape):
                raise ValueError(f"variable {v.name}: file shape {tuple(t.shape)} != {tuple(v._t.shape)}")
            v._t.copy_(t.to(v._t.dtype))


def normalize_program(program, feed_vars, fetch_vars, **kw):
    fetch = [_slot_of(program, v) for v in (fetch_vars if isinstance(fetch_vars, (list, tuple)) else [fetch_vars])]
    return _prune(program, fetch)


def save_persistables(executor, dirname, main_program=None, filename=None):
    prog = main_program or default_main_program()
    os.makedirs(dirname, exist_ok=True)
    _io.save({p.name: p for p in prog.all_parameters()}, os.path.join(dirname, filename or "persistables.pdparams"))


def load_persistables(executor, dirname, main_program=None, filename=None):
    prog = main_program or default_main_program()
    set_program_state(prog, _io.load(os.path.join(dirname, filename or "persistables.pdparams")))
