"""Static semi-auto parallel engine (dist.to_static): LLaMA annotated with placements on a ["pp", "dp", "mp"]
mesh trains through traced programs partitioned per rank (TP collectives, DP gradient reduction, pipeline
p2p) and must reproduce single-process training. Reference: test/auto_parallel/hybrid_strategy/
semi_auto_llama.py (semi-auto LLaMA PP x TP x DP), static/engine.py."""
import os
import sys

import numpy as np
import pytest
import torch

from test_distributed_cpu import ROOT, _setup, _spawn

STEPS = 3


def _data():
    g = torch.Generator().manual_seed(5)
    return torch.randint(0, 512, (4, 17), generator=g)


_FUSED = {}
_EXTRA = {}  # other LlamaConfig overrides (virtual_pp_degree)


def _cfg():
    from paddlepaddle_amd.models.llama_auto import LlamaConfig
    return LlamaConfig.tiny(num_hidden_layers=4, num_attention_heads=4, num_key_value_heads=2, **_FUSED, **_EXTRA)


def _worker(rank, world, port, shape, acc, schedule, q, recompute=False, overlap=False, zero=False, checkpoints=None,
            gm=1, refined=None, vpp=1, native=False):
    paddle = _setup(rank, world, port)
    import paddlepaddle_amd.distributed as dist
    from paddlepaddle_amd.models.llama_auto import LlamaForCausalLMAuto, LlamaPretrainingCriterionAuto
    pp, dp, mp = shape
    mesh = dist.ProcessMesh(np.arange(pp * dp * mp).reshape(pp, dp, mp), dim_names=["pp", "dp", "mp"])
    dist.auto_parallel.set_mesh(mesh)
    paddle.seed(4)
    cfg = _cfg()
    model, crit = LlamaForCausalLMAuto(cfg), LlamaPretrainingCriterionAuto(cfg)
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    strategy = dist.Strategy()
    strategy.pipeline.enable = pp > 1 or acc > 1
    strategy.pipeline.accumulate_steps = acc
    strategy.pipeline.schedule_mode = schedule
    if vpp > 1:
        strategy.pipeline.vpp_degree = vpp
        strategy.pipeline.vpp_seg_method = "LlamaDecoderLayerAuto"
    strategy.recompute.enable = recompute
    if checkpoints:
        strategy.recompute["checkpoints"] = checkpoints
    if refined:
        strategy.recompute["refined_ops_patterns"] = refined
    if gm > 1:
        strategy.gradient_merge["enable"] = True
        strategy.gradient_merge["k_steps"] = gm
    strategy.mp_optimization["allreduce_matmul_grad_overlapping"] = overlap
    if zero:
        strategy.sharding["enable"] = True
        strategy.sharding["degree"] = dp
        strategy.sharding["stage"] = int(zero)
    dm = dist.to_static(model, None, crit, opt, strategy)
    assert dm._engine is not None
    ids = _data()
    losses = []
    for _ in range(STEPS * gm):
        loss = dm(paddle.Tensor(ids[:, :-1]), paddle.Tensor(ids[:, 1:]))
        losses.append(float(loss))
    if gm > 1:  # no update inside a merge window; k identical batches averaged == one step on that batch
        np.testing.assert_allclose(losses[1::gm], losses[::gm], rtol=1e-6)
        losses = losses[::gm]
    eng = dm._engine
    kinds = sorted({n.name for nodes in eng.stage_nodes for n in nodes if n.name in (
        "allreduce", "allgather", "slice", "copy_to_parallel")})
    if mp > 1 and eng.my_stage == len(eng.meshes) - 1:
        # the vocab-sharded LM head feeds the vocab-parallel cross entropy (no logits gather)
        assert eng.vocab_parallel_ops >= 1, eng.vocab_parallel_ops
    if pp > 1:
        # pipeline p2p (parallel/p2p.py): the meta of each (peer, direction, slot) crossed once in the whole run
        ep = eng._p2p.ep
        assert ep.meta_exchanges == len(ep.sent_meta) and ep.messages == STEPS * acc * len(ep.sent_meta), (
            ep.meta_exchanges, len(ep.sent_meta), ep.messages)
        if vpp == 1:
            assert ep.ordered and ep.headers == STEPS * len(ep.sent_meta), ep.headers  # one header per class per run
        else:  # chunks of a ring channel interleave: tagged messages
            assert not ep.ordered
            # every virtual stage holds one layer chunk; this rank runs vpp of them
            mine = [vs for vs in range(len(eng.stage_nodes)) if vs % pp == eng.my_stage]
            assert len(mine) == vpp and all(eng.stage_nodes[vs] for vs in mine)
    if zero:  # optimizer state exists for this rank's shards only
        shards = eng.opt._parameter_list
        assert shards and all(sp.name.startswith("zero_shard") for sp in shards)
        if int(zero) == 3:
            # between steps only the shards are resident; state_dict gathers the full local parameters
            held = [p for z in eng._zero for p, _ in z["items"]]
            assert held and all(p._t.numel() == 0 for p in held) and eng.zero3_gathers == STEPS
            dm.state_dict(mode="param")
            assert all(p._t.numel() > 0 for p in held)
        assert sum(sp._t.numel() for sp in shards) * dp >= sum(p._t.numel() for p in eng.local_params.values()
                                                                 if p._t.requires_grad)
    if overlap:  # the column-parallel linears' dX all-reduces became overlapped hooks (2 per layer)
        assert eng.tp_overlapped >= 2 * cfg.num_hidden_layers // pp, eng.tp_overlapped  # + the LM head
    if _FUSED:
        names = [n.name.split(":")[-1] for nodes in eng.stage_nodes for n in nodes]
        assert names.count("qkv_rope_attention") == cfg.num_hidden_layers, names  # all stages
    if checkpoints:  # ops between consecutive checkpoints (auto_parallel_recompute pass) are segments
        from paddlepaddle_amd.distributed.auto_parallel.static_engine import _Seg
        assert eng.pass_stats_rc == len(checkpoints), eng.pass_stats_rc
        segs = [it for it in eng.stage_items[eng.my_stage] if isinstance(it, _Seg)]
        assert segs, eng.stage_items[eng.my_stage]
    elif refined:  # the first matmul of every layer segment is kept: each layer splits into two segments
        assert eng.refined_kept == cfg.num_hidden_layers, eng.refined_kept  # counted over all stages
    elif recompute:  # every decoder layer of this stage runs as one checkpointed segment
        from paddlepaddle_amd.distributed.auto_parallel.static_engine import _Seg
        segs = [it for it in eng.stage_items[eng.my_stage] if isinstance(it, _Seg)]
        assert len(segs) == cfg.num_hidden_layers // pp, len(segs)
        assert all(len(sg.outputs) == 1 for sg in segs), [sg.outputs for sg in segs]
    if native:  # every stage of this rank lowered after its first micro-batch and ran natively afterwards
        mine = [vs for vs in range(len(eng.stage_nodes)) if vs % pp == eng.my_stage]
        assert all(eng.native_reason.get(vs) is None for vs in mine), eng.native_reason
        nat = [eng._native[vs] for vs in mine]
        assert all(n.runs == STEPS * acc - 1 for n in nat), [n.runs for n in nat]
        assert sum(n.num_py for n in nat) > 0 and all(n.num_instructions > 10 for n in nat)
    q.put((rank, losses, kinds, eng.my_stage))
    paddle.distributed.barrier()


def _worker_native(rank, world, port, shape, acc, schedule, q):
    """The engine's stage programs on the native executor (FLAGS_static_engine_native=force lowers CPU stages)."""
    import paddlepaddle_amd as paddle
    paddle.set_flags({"FLAGS_static_engine_native": "force"})
    vpp = 2 if schedule == "VPP" else 1
    if vpp > 1:
        _EXTRA["virtual_pp_degree"] = 2
    _worker(rank, world, port, shape, acc, schedule, q, vpp=vpp, native=True, recompute=schedule == "FThenB")


def _worker_vpp(rank, world, port, shape, acc, schedule, q):
    _EXTRA["virtual_pp_degree"] = 2
    _worker(rank, world, port, shape, acc, schedule, q, vpp=2)


def _worker_rc(rank, world, port, shape, acc, schedule, q):
    _worker(rank, world, port, shape, acc, schedule, q, recompute=True)


def _worker_cp(rank, world, port, shape, acc, schedule, q):
    _worker(rank, world, port, shape, acc, schedule, q, recompute=True, checkpoints=["layers.0", "layers.2"])


def _worker_gm(rank, world, port, shape, acc, schedule, q):
    _worker(rank, world, port, shape, acc, schedule, q, gm=2, zero=shape[1] > 1)


def _worker_refined(rank, world, port, shape, acc, schedule, q):
    _worker(rank, world, port, shape, acc, schedule, q, recompute=True, refined=[{"main_ops": ["matmul"], "num": 1}])


def _worker_zero(rank, world, port, shape, acc, schedule, q):
    _worker(rank, world, port, shape, acc, schedule, q, zero=True)


def _worker_zero3(rank, world, port, shape, acc, schedule, q):
    _worker(rank, world, port, shape, acc, schedule, q, zero=3)


@pytest.mark.parametrize("shape,acc", [((1, 2, 1), 2), ((2, 2, 1), 2), ((1, 2, 2), 1)])
def test_static_engine_zero3_matches_single_process(shape, acc):
    """strategy.sharding stage 3 (reference passes/auto_parallel_sharding.py:741): parameters sharded between
    steps — all-gathered when a step starts, gradients reduce-scattered, the shard updated, the full buffers
    released — same losses as single-process training."""
    ref = _reference()
    res = _spawn(_worker_zero3, shape, acc, "1F1B", world=int(np.prod(shape)))
    for rank, losses, kinds, stage in res:
        np.testing.assert_allclose(losses, ref, rtol=2e-4, atol=1e-5, err_msg=f"rank {rank} stage {stage}")


@pytest.mark.parametrize("shape,acc", [((1, 2, 1), 2), ((1, 2, 2), 1), ((2, 2, 1), 2)])
def test_static_engine_zero_sharding_matches_single_process(shape, acc):
    """strategy.sharding (ZeRO-1 over "dp"): local gradients reduce-scattered once per step, the optimizer on this
    rank's shard of the flat parameters, parameters all-gathered: same losses as single-process training."""
    ref = _reference()
    res = _spawn(_worker_zero, shape, acc, "1F1B", world=int(np.prod(shape)))
    for rank, losses, kinds, stage in res:
        np.testing.assert_allclose(losses, ref, rtol=2e-4, atol=1e-5, err_msg=f"rank {rank} stage {stage}")


@pytest.mark.parametrize("shape,acc", [((1, 1, 2), 1), ((2, 1, 2), 2)])
def test_static_engine_selective_recompute_matches_single_process(shape, acc):
    """strategy.recompute.refined_ops_patterns: the first matmul of every recompute segment is kept (not
    recomputed); the segment splits around it and training matches the single process."""
    ref = _reference()
    res = _spawn(_worker_refined, shape, acc, "1F1B", world=int(np.prod(shape)))
    for rank, losses, kinds, stage in res:
        np.testing.assert_allclose(losses, ref, rtol=2e-4, atol=1e-5, err_msg=f"rank {rank} stage {stage}")


@pytest.mark.parametrize("shape,acc", [((1, 1, 2), 1), ((1, 2, 2), 2)])
def test_static_engine_gradient_merge_matches_single_process(shape, acc):
    """strategy.gradient_merge (k_steps 2, avg): the optimizer runs every second call on the averaged gradients
    (also with ZeRO over dp); with the same batch each call this equals single-process training."""
    ref = _reference()
    res = _spawn(_worker_gm, shape, acc, "1F1B", world=int(np.prod(shape)))
    for rank, losses, kinds, stage in res:
        np.testing.assert_allclose(losses, ref, rtol=2e-4, atol=1e-5, err_msg=f"rank {rank} stage {stage}")


def _fused_cfg(mp):
    return {"fuse_attention_qkv": True, "fuse_attention_ffn": True, "tensor_parallel_degree": mp}


def _worker_fused(rank, world, port, shape, acc, schedule, q):
    _FUSED.update(_fused_cfg(shape[2]))
    _worker(rank, world, port, shape, acc, schedule, q, overlap=shape[0] == 1)


LLAMA_PLAN = {
    "layers.*.self_attn.q_proj": "col", "layers.*.self_attn.k_proj": "col", "layers.*.self_attn.v_proj": "col",
    "layers.*.self_attn.o_proj": "row", "layers.*.mlp.gate_proj": "col", "layers.*.mlp.up_proj": "col",
    "layers.*.mlp.down_proj": "row", "lm_head": "col", "embed_tokens": "row"}  # vocab-parallel embedding


def _worker_parallelize(rank, world, port, shape, acc, q, level=0):
    """Plain single-card LLaMA built without a mesh, then distributed by dist.parallelize plans."""
    paddle = _setup(rank, world, port)
    import paddlepaddle_amd.distributed as dist
    from paddlepaddle_amd.models.llama_auto import LlamaForCausalLMAuto, LlamaPretrainingCriterionAuto
    pp, dp, mp = shape
    dist.auto_parallel.set_mesh(None)
    paddle.seed(4)
    cfg = _cfg()
    model, crit = LlamaForCausalLMAuto(cfg), LlamaPretrainingCriterionAuto(cfg)
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    mesh = dist.ProcessMesh(np.arange(pp * dp * mp).reshape(pp, dp, mp), dim_names=["pp", "dp", "mp"])
    plan = {k: (dist.ColWiseParallel() if v == "col" else dist.RowWiseParallel()) for k, v in LLAMA_PLAN.items()}
    model, opt = dist.parallelize(model, opt, mesh, dp_config={"sharding_level": level},
                                  mp_config={"parallelize_plan": plan}, pp_config={"split_spec": "layers"})
    strategy = dist.Strategy()
    strategy.pipeline.enable = pp > 1 or acc > 1
    strategy.pipeline.accumulate_steps = acc
    strategy.fused_passes["sibling_linears"] = level == 0  # opt-in pass (off by default), exercised here for parity
    dm = dist.to_static(model, None, crit, opt, strategy)
    assert dm._engine is not None
    ids = _data()
    losses = [float(dm(paddle.Tensor(ids[:, :-1]), paddle.Tensor(ids[:, 1:]))) for _ in range(STEPS)]
    eng = dm._engine
    kinds = sorted({n.name for nodes in eng.stage_nodes for n in nodes if n.name in (
        "allreduce", "allgather", "slice", "copy_to_parallel")})
    if mp > 1:  # vocab-parallel embedding (Partial output) and cross entropy on the local vocabulary slices
        assert eng.vocab_parallel_ops >= 2, eng.vocab_parallel_ops
    # program passes on the traced model (static_engine._apply_passes): q / k / v and gate / up of every layer are
    # one multi_linear node, both RMSNorms of every layer carry the residual gradient
    L = cfg.num_hidden_layers
    if level == 0:
        assert eng.pass_stats == {"rms_norm_residual": 2 * L, "sibling_linears": 5 * L}, eng.pass_stats
        names = [n.name.split(":")[-1] for nodes in eng.stage_nodes for n in nodes]
        assert names.count("multi_linear") == 2 * L and names.count("rms_norm_residual") == 2 * L, names
    else:  # dist.shard_optimizer(ShardingStage1) from dp_config: ZeRO on the engine
        assert eng._zero and all(sp.name.startswith("zero_shard") for sp in eng.opt._parameter_list)
    q.put((rank, losses, kinds, eng.my_stage))
    paddle.distributed.barrier()


def _reference():
    sys.path.insert(0, ROOT)
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.models.llama_auto import LlamaForCausalLMAuto, LlamaPretrainingCriterionAuto
    paddle.distributed.auto_parallel.set_mesh(None)
    paddle.seed(4)
    cfg = _cfg()
    model, crit = LlamaForCausalLMAuto(cfg), LlamaPretrainingCriterionAuto(cfg)
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    ids = _data()
    out = []
    for _ in range(STEPS):
        loss = crit(model(paddle.Tensor(ids[:, :-1])), paddle.Tensor(ids[:, 1:]))
        loss.backward()
        opt.step()
        opt.clear_grad()
        out.append(float(loss))
    return out


@pytest.mark.parametrize("shape,acc,schedule", [
    ((1, 1, 2), 1, "1F1B"),     # tensor parallel
    ((1, 2, 2), 1, "1F1B"),     # data x tensor parallel
    ((2, 1, 2), 2, "1F1B"),     # pipeline x tensor parallel
    ((4, 1, 2), 4, "1F1B"),     # the reference's PP4 x TP2 configuration, 8 ranks
    ((2, 2, 2), 2, "FThenB"),   # pipeline x data x tensor parallel, 8 ranks
    ((2, 1, 2), 4, "ZBH1"),     # zero-bubble: weight gradients deferred into the cool-down
    ((2, 1, 2), 4, "Eager1F1B"),  # 2 (pp - stage) - 1 warm-up forwards
])
def test_static_auto_parallel_llama_matches_single_process(shape, acc, schedule):
    ref = _reference()
    world = int(np.prod(shape))
    res = _spawn(_worker, shape, acc, schedule, world=world)
    for rank, losses, kinds, stage in res:
        np.testing.assert_allclose(losses, ref, rtol=2e-4, atol=1e-5, err_msg=f"rank {rank} stage {stage}")
        if shape[2] > 1:
            assert "allreduce" in kinds and "copy_to_parallel" in kinds


@pytest.mark.parametrize("shape,acc,schedule", [((1, 1, 2), 1, "1F1B"), ((2, 1, 2), 2, "1F1B"),
                                                ((2, 1, 2), 4, "ZBH1")])
def test_static_engine_recompute_matches_single_process(shape, acc, schedule):
    """strategy.recompute: each decoder layer is a checkpointed segment of the stage program (its activations,
    TP collectives included, rebuilt in backward); losses equal single-process training."""
    ref = _reference()
    res = _spawn(_worker_rc, shape, acc, schedule, world=int(np.prod(shape)))
    for rank, losses, kinds, stage in res:
        np.testing.assert_allclose(losses, ref, rtol=2e-4, atol=1e-5, err_msg=f"rank {rank} stage {stage}")


@pytest.mark.parametrize("shape,acc", [((1, 1, 2), 1), ((2, 1, 2), 2)])
def test_static_engine_recompute_checkpoints_pass(shape, acc):
    """strategy.recompute.checkpoints (sublayer outputs) -> the registered auto_parallel_recompute pass marks the
    ops between consecutive checkpoints as recompute segments; losses equal single-process training."""
    ref = _reference()
    res = _spawn(_worker_cp, shape, acc, "1F1B", world=int(np.prod(shape)))
    for rank, losses, kinds, stage in res:
        np.testing.assert_allclose(losses, ref, rtol=2e-4, atol=1e-5, err_msg=f"rank {rank} stage {stage}")


@pytest.mark.parametrize("shape,acc", [((1, 1, 2), 1), ((2, 1, 2), 2)])
def test_static_engine_fused_qkv_ffn_llama_matches_single_process(shape, acc):
    """fuse_attention_qkv / fuse_attention_ffn: one [q_r | k_r | v_r] and one [gate_r | up_r] projection per
    tensor-parallel rank, attention as qkv_rope_attention with its heads localized per rank: same losses as the
    single-process model of the same layout."""
    _FUSED.update(_fused_cfg(shape[2]))
    try:
        ref = _reference()
    finally:
        _FUSED.clear()
    res = _spawn(_worker_fused, shape, acc, "1F1B", world=int(np.prod(shape)))
    for rank, losses, kinds, stage in res:
        np.testing.assert_allclose(losses, ref, rtol=2e-4, atol=1e-5, err_msg=f"rank {rank} stage {stage}")
        assert "allreduce" in kinds


def _worker_parallelize_zero(rank, world, port, shape, acc, q):
    _worker_parallelize(rank, world, port, shape, acc, q, level=1)


def test_parallelize_sharding_level1_zero_matches_single_process():
    """dp_config sharding_level 1 -> dist.shard_optimizer(ShardingStage1) -> ZeRO on the static engine."""
    ref = _reference()
    res = _spawn(_worker_parallelize_zero, (1, 2, 2), 2, world=4)
    for rank, losses, kinds, stage in res:
        np.testing.assert_allclose(losses, ref, rtol=2e-4, atol=1e-5, err_msg=f"rank {rank} stage {stage}")


@pytest.mark.parametrize("shape,acc", [((1, 1, 2), 1), ((4, 1, 2), 4)])
def test_parallelize_plan_llama_matches_single_process(shape, acc):
    """dist.parallelize (pipeline split_spec + ColWise / RowWise plan) then dist.to_static: same losses as
    single-process training; at PP4 x TP2 every stage holds its own layers."""
    ref = _reference()
    res = _spawn(_worker_parallelize, shape, acc, world=int(np.prod(shape)))
    stages = set()
    for rank, losses, kinds, stage in res:
        np.testing.assert_allclose(losses, ref, rtol=2e-4, atol=1e-5, err_msg=f"rank {rank} stage {stage}")
        assert "allreduce" in kinds and "copy_to_parallel" in kinds
        stages.add(stage)
    assert stages == set(range(shape[0]))


@pytest.mark.parametrize("shape,acc,schedule", [((2, 1, 1), 4, "VPP"), ((2, 1, 2), 4, "VPP"), ((2, 1, 1), 2, "ZBVPP")])
def test_static_engine_vpp_matches_single_process(shape, acc, schedule):
    """strategy.pipeline vpp_degree 2 + vpp_seg_method: the decoder layers form pp x 2 chunks (chunk c on pp mesh
    c % pp, LlamaConfig.virtual_pp_degree), each rank runs two model chunks through the interleaved (VPP) or
    zero-bubble interleaved (ZBVPP) job list of the pipeline_scheduler pass; losses equal single-process
    training (reference passes/pipeline_scheduler_pass/pipeline_vpp.py, pipeline_zero_bubble.py ZBVPP)."""
    _EXTRA["virtual_pp_degree"] = 2
    try:
        ref = _reference()
    finally:
        _EXTRA.clear()
    res = _spawn(_worker_vpp, shape, acc, schedule, world=int(np.prod(shape)))
    for rank, losses, kinds, stage in res:
        np.testing.assert_allclose(losses, ref, rtol=2e-4, atol=1e-5, err_msg=f"rank {rank} stage {stage}")


@pytest.mark.parametrize("shape,acc,schedule", [((1, 1, 2), 2, "1F1B"), ((2, 1, 2), 4, "1F1B"),
                                                ((1, 2, 2), 2, "FThenB"), ((2, 1, 1), 4, "VPP")])
def test_static_engine_native_stage_execution(shape, acc, schedule):
    """Each rank's partitioned stage program runs on the native training executor after its first micro-batch
    (hot ops as native instructions, collectives / other ops of this framework as Python-call instructions, torch
    ops as ATen calls; distributed/auto_parallel/native_stage.py): the same losses as single-process training
    at TP2, PP2 x TP2, DP2 x TP2 (with recompute: each checkpointed decoder layer one Python-call instruction) and
    PP2 x VPP2 (reference: the engine runs the partitioned program on the standalone executor,
    auto_parallel/static/engine.py)."""
    if schedule == "VPP":
        _EXTRA["virtual_pp_degree"] = 2
    try:
        ref = _reference()
    finally:
        _EXTRA.clear()
    res = _spawn(_worker_native, shape, acc, schedule, world=int(np.prod(shape)))
    for rank, losses, kinds, stage in res:
        np.testing.assert_allclose(losses, ref, rtol=2e-4, atol=1e-5, err_msg=f"rank {rank} stage {stage}")


def test_static_engine_rejects_unimplemented_strategy_fields():
    """Strategy fields the engine does not implement raise instead of being silently ignored."""
    sys.path.insert(0, ROOT)
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    import paddlepaddle_amd.distributed as dist
    from paddlepaddle_amd.distributed.auto_parallel.static_engine import StaticEngine
    from paddlepaddle_amd.models.llama_auto import LlamaForCausalLMAuto, LlamaPretrainingCriterionAuto
    dist.auto_parallel.set_mesh(None)
    cfg = _cfg()
    model = LlamaForCausalLMAuto(cfg)
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters())
    st = dist.Strategy()
    st.pipeline.enable = True
    st.pipeline.schedule_mode = "VPP"
    with pytest.raises(NotImplementedError, match="schedule_mode"):
        StaticEngine(model, LlamaPretrainingCriterionAuto(cfg), opt, st)

