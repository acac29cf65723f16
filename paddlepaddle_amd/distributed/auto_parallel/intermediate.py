"""Intermediate auto-parallel API: turn a plain single-card model into a PP x TP x DP distributed one by plan.

Reference: python/paddle/distributed/auto_parallel/intermediate/ (parallelize.py:22 parallelize,
tensor_parallel.py ColWiseParallel / RowWiseParallel / PrepareLayerInput / PrepareLayerOutput /
SequenceParallel*, pipeline_parallel.py pipeline_parallel + SplitPoint, sharded_data_parallel.py).

    model, opt = dist.parallelize(model, opt, mesh, dp_config={"sharding_level": 0},
                                  mp_config={"parallelize_plan": {"layers.*.self_attn.q_proj": ColWiseParallel(),
                                                                  "layers.*.self_attn.o_proj": RowWiseParallel()}},
                                  pp_config={"split_spec": "layers"})
    dm = dist.to_static(model, loader, loss_fn, opt, strategy)   # static engine: trace, propagate, partition

What the passes do, in order:
  * pipeline: the layers under ``split_spec`` (a LayerList prefix, a list of layer names, or
    {name: SplitPoint}) are cut into ``pp`` contiguous stages; each stage's parameters live on the stage
    mesh ``mesh.get_mesh_with_dim("pp", s)``, sublayers before the first cut on stage 0, after the last on
    the final stage; a forward pre-hook on each stage's first layer reshards the incoming activation onto
    that stage's mesh (batch dim sharded over "dp") — the stage hand-off the static engine turns into
    point-to-point transfers.
  * tensor parallel: every layer whose name matches a plan key (``*`` matches one name component) gets
    its weight / bias sharded over the "mp" dim of its stage mesh: ColWise = Linear weight Shard(1) +
    bias Shard(0) (Embedding: Shard(1)), RowWise = Linear weight Shard(0), bias replicated (Embedding:
    Shard(0), vocab-parallel); the static engine inserts the matching collectives.
  * data parallel: parameters left dense are replicated on their stage mesh (the engine all-reduces their
    gradients over "dp"); sharding_level 1/2/3 additionally wraps the optimizer with ShardingStageN.
Parameters are re-placed in place, so an optimizer built before ``parallelize`` keeps working."""
from __future__ import annotations

import re
from enum import Enum

from ... import nn
from .api import _is_dist, reshard, shard_tensor, shard_optimizer, ShardingStage1, ShardingStage2, ShardingStage3
from .placement_type import Replicate, Shard
from .process_mesh import get_mesh


class SplitPoint(Enum):
    BEGINNING = 0
    END = 1


def _dim(mesh, name):
    return mesh.dim_names.index(name) if name in mesh.dim_names else None


def _placements(mesh, **shards):
    pl = [Replicate() for _ in range(mesh.ndim)]
    for dim_name, d in shards.items():
        i = _dim(mesh, dim_name)
        if i is not None and d is not None:
            pl[i] = Shard(d)
    return pl


def _stage_mesh(mesh, s):
    return mesh.get_mesh_with_dim("pp", s) if _dim(mesh, "pp") is not None else mesh


def _pattern(key):
    return re.compile("^" + re.escape(key).replace(r"\*", r"[^.]+") + "$")


# ------------------------------------------------------------------------------------------------ plans
class PlanBase:
    def apply(self, layer, mesh, shard_weight=True, shard_bias=True):
        raise NotImplementedError


class ColWiseParallel(PlanBase):
    """Column-parallel: output features split over "mp" (Linear weight [in, out] -> Shard(1))."""

    def __init__(self, gather_output=False):
        self.gather_output = gather_output

    def apply(self, layer, mesh, shard_weight=True, shard_bias=True):
        w = getattr(layer, "weight", None)
        if w is not None and shard_weight and not _is_dist(w._t):
            shard_tensor(w, mesh, _placements(mesh, mp=1))
        b = getattr(layer, "bias", None)
        if b is not None and shard_bias and not _is_dist(b._t):
            shard_tensor(b, mesh, _placements(mesh, mp=0 if not isinstance(layer, nn.Embedding) else None))
        if self.gather_output:
            layer.register_forward_post_hook(lambda l, i, out: reshard(out, mesh, _placements(mesh)))


class RowWiseParallel(PlanBase):
    """Row-parallel: input features split over "mp" (Linear weight -> Shard(0); Embedding vocab-parallel)."""

    def __init__(self, is_input_parallel=True):
        self.is_input_parallel = is_input_parallel

    def apply(self, layer, mesh, shard_weight=True, shard_bias=False):
        w = getattr(layer, "weight", None)
        if w is not None and shard_weight and not _is_dist(w._t):
            shard_tensor(w, mesh, _placements(mesh, mp=0))
        if not self.is_input_parallel:
            last = None if isinstance(layer, nn.Embedding) else -1

            def split(l, inputs):
                x = inputs[0]
                return (reshard(x, mesh, _placements(mesh, mp=x.ndim - 1 if last == -1 else None)),) + inputs[1:]
            layer.register_forward_pre_hook(split)


class PrepareLayerInput(PlanBase):
    """``fn(process_mesh)`` returns a forward pre-hook that places the layer's inputs."""

    def __init__(self, fn=None):
        self.fn = fn

    def apply(self, layer, mesh, shard_weight=None, shard_bias=None):
        if self.fn is not None:
            layer.register_forward_pre_hook(self.fn(process_mesh=mesh))


class PrepareLayerOutput(PlanBase):
    """``fn(process_mesh)`` returns a forward post-hook that places the layer's outputs."""

    def __init__(self, fn=None):
        self.fn = fn

    def apply(self, layer, mesh, shard_weight=None, shard_bias=None):
        if self.fn is not None:
            layer.register_forward_post_hook(self.fn(process_mesh=mesh))


def _seq_dim(x, need_transpose):
    return 0 if need_transpose else 1  # [S, B, H] after the reference's transpose, else [B, S, H]


class SequenceParallelBegin(PlanBase):
    """After this layer activations are split along the sequence over "mp"."""

    def __init__(self, need_transpose=True):
        self.need_transpose = need_transpose

    def apply(self, layer, mesh, shard_weight=None, shard_bias=None):
        layer.register_forward_post_hook(
            lambda l, i, out: reshard(out, mesh, _placements(mesh, mp=_seq_dim(out, self.need_transpose))))


class SequenceParallelEnd(PlanBase):
    """Before this layer the sequence-split activations are gathered back (replicated over "mp")."""

    def __init__(self, need_transpose=True):
        self.need_transpose = need_transpose

    def apply(self, layer, mesh, shard_weight=None, shard_bias=None):
        layer.register_forward_pre_hook(lambda l, inputs: (reshard(inputs[0], mesh, _placements(mesh)),)
                                        + tuple(inputs[1:]))


class SequenceParallelEnable(PlanBase):
    """The layer runs on sequence shards: input split along the sequence, output kept split."""

    def apply(self, layer, mesh, shard_weight=None, shard_bias=None):
        layer.register_forward_pre_hook(
            lambda l, inputs: (reshard(inputs[0], mesh, _placements(mesh, mp=1)),) + tuple(inputs[1:]))


class SequenceParallelDisable(PlanBase):
    """The layer runs on full sequences: input gathered, output re-split along the sequence."""

    def __init__(self, need_transpose=True):
        self.need_transpose = need_transpose

    def apply(self, layer, mesh, shard_weight=None, shard_bias=None):
        layer.register_forward_pre_hook(lambda l, inputs: (reshard(inputs[0], mesh, _placements(mesh)),)
                                        + tuple(inputs[1:]))
        layer.register_forward_post_hook(
            lambda l, i, out: reshard(out, mesh, _placements(mesh, mp=_seq_dim(out, self.need_transpose))))


# ------------------------------------------------------------------------------------------------ passes
def _stage_of_layers(model, split_spec, pp):
    """{sublayer name: stage} for the named pipeline units, plus the ordered unit list."""
    names = dict(model.named_sublayers())
    if isinstance(split_spec, str):
        prefix = split_spec
        units = sorted((n for n in names if n.startswith(prefix + ".") and n[len(prefix) + 1:].isdigit()),
                       key=lambda n: int(n.rsplit(".", 1)[1]))
        if not units:
            raise ValueError(f"split_spec {split_spec!r} matches no numbered sublayers")
        per = -(-len(units) // pp)
        return {u: min(i // per, pp - 1) for i, u in enumerate(units)}, units
    if isinstance(split_spec, (list, tuple)):
        units = list(split_spec)
        per = -(-len(units) // pp)
        return {u: min(i // per, pp - 1) for i, u in enumerate(units)}, units
    # {name: SplitPoint}: each entry closes (END) or opens (BEGINNING) a stage boundary
    order = [n for n in names]
    cuts = []
    for n, sp in split_spec.items():
        if n not in names:
            raise ValueError(f"split_spec layer {n!r} is not in the model")
        idx = order.index(n)
        cuts.append(idx + (1 if sp == SplitPoint.END else 0))
    if len(cuts) != pp - 1:
        raise ValueError(f"{len(cuts)} split points for {pp} pipeline stages")
    top = [n for n in order if "." not in n]
    stage_of, s = {}, 0
    for n in top:
        while s < len(cuts) and order.index(n) >= cuts[s]:
            s += 1
        stage_of[n] = s
    return stage_of, top


def pipeline_parallel(model, optimizer=None, config=None):
    mesh = get_mesh()
    cfg = config or {}
    spec = cfg.get("split_spec")
    pp = mesh.get_dim_size("pp") if _dim(mesh, "pp") is not None else 1
    if spec is None or pp == 1:
        return model, optimizer
    stage_of, units = _stage_of_layers(model, spec, pp)
    if len(set(stage_of[u] for u in units)) < pp:
        raise ValueError(f"pipeline degree {pp} exceeds the {len(units)} layers under split_spec {spec!r}")
    first_unit_stage = {}
    for u in units:
        first_unit_stage.setdefault(stage_of[u], u)
    names = dict(model.named_sublayers())
    # parameters: owner unit's stage; outside the units, before the first -> 0, after the last -> pp - 1
    order = list(names)
    first_idx, last_idx = order.index(units[0]), order.index(units[-1])
    for n, sub in names.items():
        owner = next((u for u in units if n == u or n.startswith(u + ".")), None)
        if owner is not None:
            s = stage_of[owner]
        else:
            s = 0 if order.index(n) < first_idx else (pp - 1 if order.index(n) > last_idx else None)
            if s is None:
                continue
        sub._pa_stage = s
    model._pa_stage = 0
    for s, u in first_unit_stage.items():
        if s == 0:
            continue
        sm = _stage_mesh(mesh, s)

        def hop(l, inputs, sm=sm):
            return (reshard(inputs[0], sm, _placements(sm, dp=0)),) + tuple(inputs[1:])
        names[u].register_forward_pre_hook(hop)
    tail = [n for n in order if "." not in n and order.index(n) > last_idx]
    if tail and stage_of[units[-1]] != pp - 1:  # the head runs on the last stage
        sm = _stage_mesh(mesh, pp - 1)
        names[tail[0]].register_forward_pre_hook(
            lambda l, inputs: (reshard(inputs[0], sm, _placements(sm, dp=0)),) + tuple(inputs[1:]))
    return model, optimizer


def _layer_mesh(model, name, layer, mesh):
    s = getattr(layer, "_pa_stage", None)
    if s is None:  # nearest annotated ancestor
        parts = name.split(".")
        subs = dict(model.named_sublayers())
        for k in range(len(parts) - 1, 0, -1):
            s = getattr(subs.get(".".join(parts[:k])), "_pa_stage", None)
            if s is not None:
                break
    return _stage_mesh(mesh, s or 0) if _dim(mesh, "pp") is not None else mesh


def tensor_parallel(model, optimizer=None, config=None):
    mesh = get_mesh()
    plan = (config or {}).get("parallelize_plan") or {}
    pats = [(_pattern(k), v if isinstance(v, (list, tuple)) else [v]) for k, v in plan.items()]
    for name, layer in model.named_sublayers():
        for pat, plans in pats:
            if pat.match(name):
                lm = _layer_mesh(model, name, layer, mesh)
                for p in plans:
                    p.apply(layer, lm)
    return model, optimizer


def sharded_data_parallel(model, optimizer=None, config=None):
    level = int((config or {}).get("sharding_level", 0))
    if optimizer is not None and level > 0:
        mesh = get_mesh()
        stage = {1: ShardingStage1, 2: ShardingStage2, 3: ShardingStage3}[level]
        optimizer = shard_optimizer(optimizer, stage("dp", mesh) if _dim(mesh, "dp") is not None else stage())
    return model, optimizer


def _replicate_rest(model, mesh):
    for name, layer in model.named_sublayers(include_self=True):
        lm = _layer_mesh(model, name, layer, mesh) if name else _stage_mesh(mesh, getattr(layer, "_pa_stage", 0))
        for p in layer._parameters.values():
            if p is not None and not _is_dist(p._t):
                shard_tensor(p, lm, _placements(lm), stop_gradient=p.stop_gradient)


def parallelize(model, optimizer=None, mesh=None, dp_config=None, mp_config=None, pp_config=None):
    """Apply the pipeline, tensor-parallel and data-parallel plans (in that order) to ``model`` in place;
    returns (model, optimizer). ``mesh`` defaults to the global mesh (``dist.auto_parallel.set_mesh``)."""
    if mesh is not None:
        from .process_mesh import set_mesh
        set_mesh(mesh)
    mesh = get_mesh()
    if mesh is None:
        raise ValueError("parallelize needs a process mesh (argument or dist.auto_parallel.set_mesh)")
    if pp_config is not None:
        model, optimizer = pipeline_parallel(model, optimizer, pp_config)
    if mp_config is not None:
        model, optimizer = tensor_parallel(model, optimizer, mp_config)
    _replicate_rest(model, mesh)
    if dp_config is not None:
        model, optimizer = sharded_data_parallel(model, optimizer, dp_config)
    return model, optimizer


_PARALLELIZED = {"model": False}


def parallelize_model(model, mesh=None, dp_config=None, mp_config=None, pp_config=None):
    _PARALLELIZED["model"] = True
    return parallelize(model, None, mesh, dp_config, mp_config, pp_config)[0]


def parallelize_optimizer(optimizer, mesh=None, dp_config=None, mp_config=None, pp_config=None):
    if not _PARALLELIZED["model"]:
        raise RuntimeError("parallelize the model before the optimizer")
    for p in optimizer._parameter_list:
        params = p["params"] if isinstance(p, dict) else [p]
        for q in params:
            if not _is_dist(q._t):
                raise RuntimeError("build the optimizer from the parallelized model's parameters")
    return sharded_data_parallel(None, optimizer, dp_config)[1]
