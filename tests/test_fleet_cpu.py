"""Fleet hybrid parallel on CPU (gloo, world_size=2): tensor parallel GPT, 1F1B pipeline, sequence
parallel ops. Each parallel run must reproduce single-process training of the same model.
Reference test strategy: test/collective/fleet/hybrid_parallel_mp_model.py, hybrid_parallel_pp_layer.py
(parallel loss == single-card loss with the same weights)."""
import os
import sys

import numpy as np
import pytest
import torch

from test_distributed_cpu import ROOT, _data, _setup, _spawn


def _fleet_init(paddle, acc=2, schedule="1F1B", **hc):
    from paddlepaddle_amd.distributed import fleet
    s = fleet.DistributedStrategy()
    cfg = dict(dp_degree=1, mp_degree=1, pp_degree=1)
    cfg.update(hc)
    s.hybrid_configs = cfg
    s.pipeline_configs = {"accumulate_steps": acc, "micro_batch_size": 2, "schedule_mode": schedule}
    fleet.init(is_collective=True, strategy=s)
    return fleet


def _gpt_full(paddle):
    from paddlepaddle_amd.models.gpt import GPTConfig, GPTForPretraining, GPTPretrainingCriterion
    paddle.seed(11)
    cfg = GPTConfig.tiny(num_hidden_layers=2, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    return cfg, GPTForPretraining(cfg), GPTPretrainingCriterion(cfg)


def _shard_like(full, local, rank, world):
    """Slice a full weight to the local TP shape (the dim that differs is the split one)."""
    if tuple(full.shape) == tuple(local.shape):
        return full
    for d in range(full.dim()):
        if full.shape[d] != local.shape[d]:
            return full.chunk(world, d)[rank]
    raise AssertionError


def _train(paddle, model, crit, opt, ids, steps=3):
    losses = []
    for _ in range(steps):
        loss = crit(model(paddle.Tensor(ids[:, :-1])), paddle.Tensor(ids[:, 1:]))
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    return losses


def _tp_worker(rank, world, port, q):
    paddle = _setup(rank, world, port)
    from paddlepaddle_amd.models.gpt import GPTConfig, GPTForPretraining, GPTPretrainingCriterion
    _, full, _ = _gpt_full(paddle)
    full_sd = {k: v._t.detach().clone() for k, v in full.state_dict().items()}
    fleet = _fleet_init(paddle, mp_degree=2)
    cfg = GPTConfig.tiny(num_hidden_layers=2, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0,
                         tensor_parallel_degree=2)
    model, crit = GPTForPretraining(cfg), GPTPretrainingCriterion(cfg)
    with torch.no_grad():
        for k, v in model.state_dict().items():
            v._t.copy_(_shard_like(full_sd[k], v._t, rank, world))
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    model = fleet.distributed_model(model)
    opt = fleet.distributed_optimizer(opt)
    losses = _train(paddle, model, crit, opt, _data(cfg))
    sd = {k: v.numpy() for k, v in model.state_dict().items()}
    q.put((rank, losses, sd))
    paddle.distributed.barrier()


def _single_gpt():
    sys.path.insert(0, ROOT)
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    cfg, model, crit = _gpt_full(paddle)
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    losses = _train(paddle, model, crit, opt, _data(cfg))
    return losses, {k: v.numpy() for k, v in model.state_dict().items()}


def test_tensor_parallel_gpt_matches_single_process():
    ref_losses, ref_sd = _single_gpt()
    res = _spawn(_tp_worker)
    (_, l0, sd0), (_, l1, sd1) = res
    np.testing.assert_allclose(l0, ref_losses, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(l1, l0, rtol=0, atol=0)
    for k, full in ref_sd.items():
        t = torch.from_numpy(full)
        for r, sd in enumerate((sd0, sd1)):
            exp = _shard_like(t, torch.from_numpy(sd[k]), r, 2).numpy()
            np.testing.assert_allclose(sd[k], exp, rtol=2e-3, atol=2e-4, err_msg=f"rank{r}:{k}")


# ----------------------------------------------------------------------------- pipeline
def _mlp_descs(paddle):
    from paddlepaddle_amd.parallel.pipeline import LayerDesc
    nn = paddle.nn
    return [LayerDesc(nn.Linear, 16, 32), LayerDesc(nn.Tanh), LayerDesc(nn.Linear, 32, 32), LayerDesc(nn.GELU),
            LayerDesc(nn.Linear, 32, 32), LayerDesc(nn.Tanh), LayerDesc(nn.Linear, 32, 8)]


def _pp_data():
    g = torch.Generator().manual_seed(3)
    return torch.randn(8, 16, generator=g), torch.randn(8, 8, generator=g)


def _mse(out, label):
    return ((out - label) ** 2).mean()


def _pp_full_params(paddle):
    """Build every layer once with a fixed seed; returns state tensors in layer order."""
    paddle.seed(7)
    layers = [d.build_layer() for d in _mlp_descs(paddle)]
    return layers


def _pp_worker(rank, world, port, q, schedule="1F1B"):
    paddle = _setup(rank, world, port)
    from paddlepaddle_amd.parallel.pipeline import PipelineLayer
    full = _pp_full_params(paddle)
    fleet = _fleet_init(paddle, pp_degree=2, schedule=schedule)
    pl = PipelineLayer(_mlp_descs(paddle), num_stages=2, loss_fn=_mse)
    lo = pl.segment_parts[pl._stage_id]
    with torch.no_grad():
        for i, f in enumerate(pl.run_function):
            for (k, v), (_, fv) in zip(f.state_dict().items(), full[lo + i].state_dict().items()):
                v._t.copy_(fv._t)
    opt = paddle.optimizer.AdamW(1e-2, parameters=pl.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    model = fleet.distributed_model(pl)
    opt = fleet.distributed_optimizer(opt)
    x, y = _pp_data()
    losses = [float(model.train_batch([paddle.Tensor(x), paddle.Tensor(y)], opt)) for _ in range(3)]
    ev = model.eval_batch([paddle.Tensor(x), paddle.Tensor(y)], compute_loss=True)
    params = {f"{lo + i}.{k}": v.numpy() for i, f in enumerate(pl.run_function) for k, v in f.state_dict().items()}
    if schedule == "ZBH1":  # weight gradients really were deferred into W jobs
        from paddlepaddle_amd.parallel.pipeline import PipelineParallelZeroBubble
        assert type(model) is PipelineParallelZeroBubble and model.deferred_wgrads > 0
        assert any(k == "W" for k, _ in model.jobs)
    elif schedule in ("FThenB", "Eager1F1B"):  # the stage walked that schedule's job list
        from paddlepaddle_amd.parallel import pp_schedules as PS
        assert model.schedule_mode == schedule.upper()
        assert model.jobs == PS.schedule(schedule.upper(), model.num_stages, model.stage_id, model.accumulate_steps)
    # p2p meta (shape / dtype) crossed each directed channel once; every later message carried only its tag
    ep = model._p2p
    assert ep.meta_exchanges == 1 and ep.messages == 3 * 2 + (2 if rank == 0 else 0), (ep.meta_exchanges,
                                                                                          ep.messages)
    # ordered channels: a host-side header only for the first message of each run (3 train runs + 1 eval run on
    # the forward channel, 3 on the backward one), every other payload receive posted from the cached meta
    assert ep.ordered and ep.headers == (4 if rank == 0 else 3), ep.headers
    q.put((rank, losses, params, None if isinstance(ev, list) else float(ev)))
    paddle.distributed.barrier()


@pytest.mark.parametrize("schedule", ["1F1B", "ZBH1", "FThenB", "Eager1F1B"])
def test_pipeline_1f1b_matches_single_process(schedule):
    sys.path.insert(0, ROOT)
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    layers = _pp_full_params(paddle)
    params = [p for l in layers for p in l.parameters()]
    opt = paddle.optimizer.AdamW(1e-2, parameters=params, grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    x, y = _pp_data()

    def fwd(t):
        for l in layers:
            t = l(t)
        return t
    ref = []
    for _ in range(3):
        # 2 micro-batches, loss averaged (== pipeline accumulate_steps=2)
        l0 = _mse(fwd(paddle.Tensor(x[:4])), paddle.Tensor(y[:4]))
        l1 = _mse(fwd(paddle.Tensor(x[4:])), paddle.Tensor(y[4:]))
        loss = (l0 + l1) * 0.5
        loss.backward()
        opt.step()
        opt.clear_grad()
        ref.append(float(loss))
    ref_params = {f"{i}.{k}": v.numpy() for i, l in enumerate(layers) for k, v in l.state_dict().items()}
    with paddle.no_grad():
        ref_eval = 0.5 * (float(_mse(fwd(paddle.Tensor(x[:4])), paddle.Tensor(y[:4]))) +
                          float(_mse(fwd(paddle.Tensor(x[4:])), paddle.Tensor(y[4:]))))

    import functools
    res = _spawn(functools.partial(_pp_worker, schedule=schedule))
    (_, l0, p0, _), (_, l1, p1, ev1) = res
    np.testing.assert_allclose(l0, ref, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(l1, ref, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(ev1, ref_eval, rtol=1e-5, atol=1e-6)
    got = dict(p0)
    got.update(p1)
    assert set(got) == set(ref_params)
    for k in ref_params:
        np.testing.assert_allclose(got[k], ref_params[k], rtol=1e-4, atol=1e-6, err_msg=k)


# ----------------------------------------------------------------------------- sequence parallel
def _sp_worker(rank, world, port, q):
    paddle = _setup(rank, world, port)
    from paddlepaddle_amd.distributed.fleet.utils import sequence_parallel_utils as spu
    _fleet_init(paddle, mp_degree=2)
    g = torch.Generator().manual_seed(1)
    full = torch.randn(6, 2, 4, generator=g)
    x = paddle.Tensor(full.clone().requires_grad_(True))
    x.stop_gradient = False
    s = spu.ScatterOp.apply(x)
    ag = spu.AllGatherOp.apply(s * (rank + 1.0))
    rs = spu.ReduceScatterOp.apply(ag)
    rs.sum().backward()
    q.put((rank, s.numpy(), ag.numpy(), rs.numpy(), x.grad.numpy()))
    paddle.distributed.barrier()


def test_sequence_parallel_ops():
    res = _spawn(_sp_worker)
    g = torch.Generator().manual_seed(1)
    full = torch.randn(6, 2, 4, generator=g).numpy()
    (_, s0, ag0, rs0, gx0), (_, s1, ag1, rs1, gx1) = res
    np.testing.assert_allclose(s0, full[:3])
    np.testing.assert_allclose(s1, full[3:])
    exp_ag = np.concatenate([full[:3] * 1.0, full[3:] * 2.0])
    np.testing.assert_allclose(ag0, exp_ag, rtol=1e-6)
    np.testing.assert_allclose(ag1, exp_ag, rtol=1e-6)
    np.testing.assert_allclose(rs0, 2 * exp_ag[:3], rtol=1e-6)
    np.testing.assert_allclose(rs1, 2 * exp_ag[3:], rtol=1e-6)
    # d ag = gather(ones) = 1; d(s*(r+1)) = reduce-scatter(d ag) = 2 -> d s_r = 2(r+1); d x = gather(d s)
    exp_gx = np.concatenate([np.full((3, 2, 4), 2.0), np.full((3, 2, 4), 4.0)])
    np.testing.assert_allclose(gx0, exp_gx, rtol=1e-6)
    np.testing.assert_allclose(gx1, exp_gx, rtol=1e-6)


# ----------------------------------------------------------------------------- llama TP
def _llama_tp_shard(name, full, rank, world, cfg):
    H, Hk, D, f = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim, cfg.intermediate_size
    if name.endswith("qkv_proj.weight"):
        q, k, v = full.split([H * D, Hk * D, Hk * D], -1)
        return torch.cat([q.chunk(world, -1)[rank], k.chunk(world, -1)[rank], v.chunk(world, -1)[rank]], -1)
    if name.endswith("gate_up_proj.weight"):
        g, u = full.chunk(2, -1)
        return torch.cat([g.chunk(world, -1)[rank], u.chunk(world, -1)[rank]], -1)
    if name.endswith("o_proj.weight") or name.endswith("down_proj.weight") or "embed_tokens" in name \
            or name == "lm_head_weight":
        return full.chunk(world, 0)[rank]
    return full


def _llama_tp_worker(rank, world, port, q, sp=False):
    paddle = _setup(rank, world, port)
    from paddlepaddle_amd.models.llama import LlamaConfig, LlamaForCausalLM, LlamaPretrainingCriterion
    paddle.seed(4)
    cfg1 = LlamaConfig.tiny()
    full = LlamaForCausalLM(cfg1)
    full_sd = {k: v._t.detach().clone() for k, v in full.state_dict().items()}
    fleet = _fleet_init(paddle, mp_degree=2)
    cfg = LlamaConfig.tiny(tensor_parallel_degree=2, sequence_parallel=sp)
    model, crit = LlamaForCausalLM(cfg), LlamaPretrainingCriterion(cfg)
    with torch.no_grad():
        for k, v in model.state_dict().items():
            v._t.copy_(_llama_tp_shard(k, full_sd[k], rank, world, cfg))
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    inner = model
    model = fleet.distributed_model(model)
    opt = fleet.distributed_optimizer(opt)
    losses = _train(paddle, model, crit, opt, _data(cfg))
    assert (inner.llama.sp_bs is not None) == sp  # the sequence-parallel path ran
    q.put((rank, losses))
    paddle.distributed.barrier()


def test_llama_tensor_parallel_matches_single_process():
    sys.path.insert(0, ROOT)
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.models.llama import LlamaConfig, LlamaForCausalLM, LlamaPretrainingCriterion
    paddle.seed(4)
    cfg = LlamaConfig.tiny()
    model, crit = LlamaForCausalLM(cfg), LlamaPretrainingCriterion(cfg)
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    ref = _train(paddle, model, crit, opt, _data(cfg))
    res = _spawn(_llama_tp_worker)
    for _, l in res:
        np.testing.assert_allclose(l, ref, rtol=1e-4, atol=1e-5)
    # sequence parallelism: norms / residuals on token blocks, all-gather / reduce-scatter around the TP linears
    res = _spawn(_llama_tp_sp_worker)
    for _, l in res:
        np.testing.assert_allclose(l, ref, rtol=1e-4, atol=1e-5)


def _llama_tp_sp_worker(rank, world, port, q):
    _llama_tp_worker(rank, world, port, q, sp=True)


# ----------------------------------------------------------------------------- interleaved pipeline (VPP)
def _vpp_descs(paddle):
    from paddlepaddle_amd.parallel.pipeline import LayerDesc
    nn = paddle.nn
    return [LayerDesc(nn.Linear, 16, 32), LayerDesc(nn.Tanh), LayerDesc(nn.Linear, 32, 32), LayerDesc(nn.GELU),
            LayerDesc(nn.Linear, 32, 32), LayerDesc(nn.Tanh), LayerDesc(nn.Linear, 32, 8), LayerDesc(nn.Tanh)]


def _vpp_worker(rank, world, port, acc, schedule, q):
    paddle = _setup(rank, world, port)
    from paddlepaddle_amd.parallel.pipeline import (PipelineLayer, PipelineParallelWithInterleave,
                                                    PipelineParallelWithInterleaveFthenB, PipelineParallelZeroBubbleVPP)
    paddle.seed(11)
    full = [d.build_layer() for d in _vpp_descs(paddle)]
    fleet = _fleet_init(paddle, acc=acc, schedule=schedule, pp_degree=2)
    pl = PipelineLayer(_vpp_descs(paddle), num_stages=2, loss_fn=_mse, num_virtual_pipeline_stages=2)
    # chunks: segments of 2 layers; stage s holds segments s and 2 + s
    idx = {}
    for v, fns in enumerate(pl.get_model_chunks()):
        c = v * 2 + pl._stage_id
        for j, f in enumerate(fns):
            idx[pl.segment_parts[c] + j] = f
    with torch.no_grad():
        for i, f in idx.items():
            for (k, v), (_, fv) in zip(f.state_dict().items(), full[i].state_dict().items()):
                v._t.copy_(fv._t)
    opt = paddle.optimizer.SGD(0.1, parameters=pl.parameters())
    model = fleet.distributed_model(pl)
    # fleet picks the schedule like the reference: interleaved 1F1B for acc >= 2 pp, FThenB for pp <= acc < 2 pp
    if schedule == "ZBVPP":
        assert type(model) is PipelineParallelZeroBubbleVPP
    else:
        assert type(model) is (PipelineParallelWithInterleave if acc >= 4 else PipelineParallelWithInterleaveFthenB)
    x, y = _pp_data()
    losses = [float(model.train_batch([paddle.Tensor(x), paddle.Tensor(y)], opt)) for _ in range(2)]
    if schedule == "ZBVPP":  # weight gradients really were deferred into W jobs
        assert model.deferred_wgrads > 0 and any(k == "W" for k, _ in model.jobs)
    params = {f"{i}.{k}": v.numpy() for i, f in idx.items() for k, v in f.state_dict().items()}
    q.put((rank, losses, params, None))
    paddle.distributed.barrier()


@pytest.mark.parametrize("acc,schedule", [(4, "1F1B"), (2, "1F1B"), (4, "ZBVPP")])
def test_pipeline_interleaved_matches_single_process(acc, schedule):
    sys.path.insert(0, ROOT)
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    paddle.seed(11)
    layers = [d.build_layer() for d in _vpp_descs(paddle)]
    params = [p for l in layers for p in l.parameters()]
    opt = paddle.optimizer.SGD(0.1, parameters=params)
    x, y = _pp_data()

    def fwd(t):
        for l in layers:
            t = l(t)
        return t
    ref = []
    for _ in range(2):
        loss = sum(_mse(fwd(paddle.Tensor(x[i:i + 2])), paddle.Tensor(y[i:i + 2])) for i in range(0, 8, 2)) * 0.25
        loss.backward()
        opt.step()
        opt.clear_grad()
        ref.append(float(loss))
    ref_params = {f"{i}.{k}": v.numpy() for i, l in enumerate(layers) for k, v in l.state_dict().items()}
    res = _spawn(_vpp_worker, acc, schedule)
    (_, l0, p0, _), (_, l1, p1, _) = res
    np.testing.assert_allclose(l0, ref, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(l1, ref, rtol=1e-5, atol=1e-6)
    got = dict(p0)
    got.update(p1)
    assert set(got) == set(ref_params)
    for k in ref_params:
        np.testing.assert_allclose(got[k], ref_params[k], rtol=1e-4, atol=1e-6, err_msg=k)


# ----------------------------------------------------------------------------- llama PP x TP (4 ranks)
def _pipe_to_full_name(stage_layer_index, name, n_layers):
    """Parameter name of a LlamaForCausalLMPipe segment layer -> LlamaForCausalLM name."""
    i = stage_layer_index
    if i == 0:
        return "llama." + name                      # embed_tokens.weight
    if i == n_layers + 1:
        return "llama.norm.weight" if name.startswith("norm.") else "lm_head_weight"
    return f"llama.layers.{i - 1}." + name


def _llama_pp_tp_worker(rank, world, port, q):
    paddle = _setup(rank, world, port)
    from paddlepaddle_amd.models.llama import (LlamaConfig, LlamaForCausalLM, LlamaForCausalLMPipe)
    paddle.seed(4)
    cfg1 = LlamaConfig.tiny(num_hidden_layers=2)
    full = LlamaForCausalLM(cfg1)
    full_sd = {k: v._t.detach().clone() for k, v in full.state_dict().items()}
    fleet = _fleet_init(paddle, acc=2, mp_degree=2, pp_degree=2)
    hcg = fleet.get_hybrid_communicate_group()
    mp_rank = hcg.get_model_parallel_rank()
    cfg = LlamaConfig.tiny(num_hidden_layers=2, tensor_parallel_degree=2)
    pipe = LlamaForCausalLMPipe(cfg)
    with torch.no_grad():
        for j, f in enumerate(pipe.run_function):
            li = pipe.segment_parts[pipe._stage_id] + j
            for k, v in f.state_dict().items():
                fk = _pipe_to_full_name(li, k, cfg.num_hidden_layers)
                v._t.copy_(_llama_tp_shard(fk, full_sd[fk], mp_rank, 2, cfg))
    opt = paddle.optimizer.SGD(0.05, parameters=pipe.parameters())
    model = fleet.distributed_model(pipe)
    ids = torch.randint(0, cfg.vocab_size, (4, 17), generator=torch.Generator().manual_seed(9))
    x, y = paddle.Tensor(ids[:, :-1].clone()), paddle.Tensor(ids[:, 1:].clone())
    losses = [float(model.train_batch([x, y], opt)) for _ in range(2)]
    q.put((rank, losses))
    paddle.distributed.barrier()


def test_llama_pipeline_x_tensor_parallel_matches_single_process():
    sys.path.insert(0, ROOT)
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.models.llama import LlamaConfig, LlamaForCausalLM, LlamaPretrainingCriterion
    paddle.seed(4)
    cfg = LlamaConfig.tiny(num_hidden_layers=2)
    model, crit = LlamaForCausalLM(cfg), LlamaPretrainingCriterion(cfg)
    opt = paddle.optimizer.SGD(0.05, parameters=model.parameters())
    ids = torch.randint(0, cfg.vocab_size, (4, 17), generator=torch.Generator().manual_seed(9))
    ref = []
    for _ in range(2):
        l0 = crit(model(paddle.Tensor(ids[:2, :-1].clone())), paddle.Tensor(ids[:2, 1:].clone()))
        l1 = crit(model(paddle.Tensor(ids[2:, :-1].clone())), paddle.Tensor(ids[2:, 1:].clone()))
        loss = (l0 + l1) * 0.5
        loss.backward()
        opt.step()
        opt.clear_grad()
        ref.append(float(loss))
    res = _spawn(_llama_pp_tp_worker, world=4)
    for _, l in res:
        np.testing.assert_allclose(l, ref, rtol=1e-4, atol=1e-5)


# ----------------------------------------------------------------------------- sharding x mp / sharding x dp
def _hybrid_sharding_worker(rank, world, port, mp_deg, stage, q):
    """fleet hybrid topology with sharding_degree > 1 (reference: dygraph_sharding_optimizer.py:54 over
    hcg's sharding group, group_sharded_stage3.py:85): data split over the sharding (and dp) ranks,
    weights split over the mp ranks. The averaged loss and the gathered weights must match the
    single-process run on the whole batch."""
    paddle = _setup(rank, world, port)
    from paddlepaddle_amd.models.gpt import GPTConfig, GPTForPretraining, GPTPretrainingCriterion
    _, full, _ = _gpt_full(paddle)
    full_sd = {k: v._t.detach().clone() for k, v in full.state_dict().items()}
    n_data = world // mp_deg
    shard_deg = 2
    fleet = _fleet_init(paddle, mp_degree=mp_deg, sharding_degree=shard_deg, dp_degree=n_data // shard_deg)
    fleet.fleet._strategy.sharding_configs["stage"] = stage
    hcg = fleet.get_hybrid_communicate_group()
    mp_rank = hcg.get_model_parallel_rank()
    data_rank = hcg.get_data_parallel_rank() * shard_deg + hcg.get_sharding_parallel_rank()
    cfg = GPTConfig.tiny(num_hidden_layers=2, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0,
                         tensor_parallel_degree=mp_deg)
    model, crit = GPTForPretraining(cfg), GPTPretrainingCriterion(cfg)
    with torch.no_grad():
        for k, v in model.state_dict().items():
            v._t.copy_(_shard_like(full_sd[k], v._t, mp_rank, mp_deg))
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    model = fleet.distributed_model(model)
    opt = fleet.distributed_optimizer(opt)
    ids = _data(cfg)
    per = ids.shape[0] // n_data
    losses = _train(paddle, model, crit, opt, ids[data_rank * per:(data_rank + 1) * per])
    sd = {k: v.numpy() for k, v in model.state_dict().items()}
    q.put((rank, mp_rank, losses, sd))
    paddle.distributed.barrier()


def _check_hybrid(res, mp_deg):
    ref_losses, ref_sd = _single_gpt()
    mean_loss = np.mean([r[2] for r in res], axis=0)
    np.testing.assert_allclose(mean_loss, ref_losses, rtol=1e-4, atol=1e-5)
    for _, mp_rank, _, sd in res:
        for k, full in ref_sd.items():
            exp = _shard_like(torch.from_numpy(full), torch.from_numpy(sd[k]), mp_rank, mp_deg).numpy()
            np.testing.assert_allclose(sd[k], exp, rtol=2e-3, atol=2e-4, err_msg=f"mp{mp_rank}:{k}")


def test_sharding_stage3_x_tensor_parallel_gpt_four_ranks():
    _check_hybrid(_spawn(_hybrid_sharding_worker, 2, 3, world=4), 2)


def test_sharding_stage2_x_data_parallel_gpt_four_ranks():
    _check_hybrid(_spawn(_hybrid_sharding_worker, 1, 2, world=4), 1)


# ----------------------------------------------------------------------------- segment parallel (sep)
def _sep_worker(rank, world, port, q):
    paddle = _setup(rank, world, port)
    from paddlepaddle_amd.models.llama import LlamaConfig, LlamaForCausalLM, LlamaPretrainingCriterion
    from paddlepaddle_amd.parallel.segment_parallel import SegmentParallel, split_sequence
    fleet = _fleet_init(paddle, sep_degree=2)
    hcg = fleet.get_hybrid_communicate_group()
    paddle.seed(4)
    cfg = LlamaConfig.tiny(sep_parallel_degree=2)
    model, crit = LlamaForCausalLM(cfg), LlamaPretrainingCriterion(cfg)
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    model = fleet.distributed_model(model)
    assert isinstance(model, SegmentParallel)
    opt = fleet.distributed_optimizer(opt)
    g = hcg.get_sep_parallel_group()
    ids = _data(cfg)
    x = split_sequence(paddle.Tensor(ids[:, :-1]), g)
    y = split_sequence(paddle.Tensor(ids[:, 1:]), g)
    losses = []
    for _ in range(3):
        # segment losses are summed over the sep group (reference: sep gradients are not scaled)
        loss = crit(model(x), y) * 0.5
        loss.backward()
        opt.step()
        opt.clear_grad()
        t = loss._t.detach().clone()
        paddle.distributed.all_reduce(paddle.Tensor(t), group=g)
        losses.append(float(t))
    q.put((rank, losses))
    paddle.distributed.barrier()


def test_llama_segment_parallel_matches_single_process():
    sys.path.insert(0, ROOT)
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.models.llama import LlamaConfig, LlamaForCausalLM, LlamaPretrainingCriterion
    paddle.seed(4)
    cfg = LlamaConfig.tiny()
    model, crit = LlamaForCausalLM(cfg), LlamaPretrainingCriterion(cfg)
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    ref = _train(paddle, model, crit, opt, _data(cfg))
    res = _spawn(_sep_worker)
    for _, l in res:
        np.testing.assert_allclose(l, ref, rtol=1e-4, atol=1e-5)


def _sep_sharding_worker(rank, world, port, q):
    """sep 2 x sharding 2 (stage 2): the batch split over the sharding ranks, the sequence over the sep ranks;
    the sharding engine sums the shard gradients over sep and averages them over sharding."""
    paddle = _setup(rank, world, port)
    from paddlepaddle_amd.models.llama import LlamaConfig, LlamaForCausalLM, LlamaPretrainingCriterion
    from paddlepaddle_amd.parallel.segment_parallel import split_sequence
    fleet = _fleet_init(paddle, sep_degree=2, sharding_degree=2)
    fleet.fleet._strategy.sharding_configs["stage"] = 2
    hcg = fleet.get_hybrid_communicate_group()
    paddle.seed(4)
    cfg = LlamaConfig.tiny(sep_parallel_degree=2)
    model, crit = LlamaForCausalLM(cfg), LlamaPretrainingCriterion(cfg)
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    model = fleet.distributed_model(model)
    opt = fleet.distributed_optimizer(opt)
    g = hcg.get_sep_parallel_group()
    ids = _data(cfg)
    per = ids.shape[0] // 2
    sr = hcg.get_sharding_parallel_rank()
    part = ids[sr * per:(sr + 1) * per]
    x = split_sequence(paddle.Tensor(part[:, :-1]), g)
    y = split_sequence(paddle.Tensor(part[:, 1:]), g)
    losses = []
    for _ in range(3):
        loss = crit(model(x), y) * 0.5
        loss.backward()
        opt.step()
        opt.clear_grad()
        t = loss._t.detach().clone()
        paddle.distributed.all_reduce(paddle.Tensor(t), group=g)
        losses.append(float(t))
    q.put((rank, losses))
    paddle.distributed.barrier()


def test_llama_segment_parallel_x_sharding_matches_single_process():
    sys.path.insert(0, ROOT)
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.models.llama import LlamaConfig, LlamaForCausalLM, LlamaPretrainingCriterion
    paddle.seed(4)
    cfg = LlamaConfig.tiny()
    model, crit = LlamaForCausalLM(cfg), LlamaPretrainingCriterion(cfg)
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    ref = _train(paddle, model, crit, opt, _data(cfg))
    res = _spawn(_sep_sharding_worker, world=4)
    mean = np.mean([l for _, l in res], axis=0)  # the two sharding ranks' halves of the batch
    np.testing.assert_allclose(mean, ref, rtol=1e-4, atol=1e-5)


def test_segment_all_to_all_roundtrip_single_process():
    """seq_to_head / head_to_seq are inverse layouts (checked with a fake 1-rank group: identity)."""
    from paddlepaddle_amd.parallel.segment_parallel import head_to_seq, seq_to_head
    x = torch.randn(2, 8, 4, 16)
    assert torch.equal(head_to_seq(seq_to_head(x, None), None), x)


# ----------------------------------------------------------------------------- sequence parallel GPT
def _sp_gpt_worker(rank, world, port, q):
    """GPT with tensor parallel + sequence parallel (token shards between the TP regions, overlapped
    all-gather / reduce-scatter linears) reproduces single-process training; rank 0 records the order of
    collectives and GEMMs of one step."""
    paddle = _setup(rank, world, port)
    from paddlepaddle_amd.models.gpt import GPTConfig, GPTForPretraining, GPTPretrainingCriterion
    from paddlepaddle_amd.parallel import sequence_parallel as SP
    _, full, _ = _gpt_full(paddle)
    full_sd = {k: v._t.detach().clone() for k, v in full.state_dict().items()}
    fleet = _fleet_init(paddle, mp_degree=2)
    cfg = GPTConfig.tiny(num_hidden_layers=2, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0,
                         tensor_parallel_degree=2, sequence_parallel=True)
    model, crit = GPTForPretraining(cfg), GPTPretrainingCriterion(cfg)
    with torch.no_grad():
        for k, v in model.state_dict().items():
            v._t.copy_(_shard_like(full_sd[k], v._t, rank, world))
    sp_names = sorted(n for n, p in model.named_parameters() if getattr(p, "sequence_parallel", False))
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    model = fleet.distributed_model(model)
    opt = fleet.distributed_optimizer(opt)
    ids = _data(cfg)
    SP.TRACE = []
    losses = _train(paddle, model, crit, opt, ids, steps=1)
    trace = list(SP.TRACE)
    SP.TRACE = None
    losses += _train(paddle, model, crit, opt, ids, steps=2)
    sd = {k: v.numpy() for k, v in model.state_dict().items()}
    q.put((rank, losses, sd, trace if rank == 0 else None, sp_names))
    paddle.distributed.barrier()


def test_sequence_parallel_gpt_matches_single_process():
    ref_losses, ref_sd = _single_gpt()
    res = sorted(_spawn(_sp_gpt_worker), key=lambda r: r[0])
    (_, l0, sd0, trace, sp_names), (_, l1, sd1, _, _) = res
    np.testing.assert_allclose(l0, ref_losses, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(l1, l0, rtol=0, atol=0)
    for k, full in ref_sd.items():
        t = torch.from_numpy(full)
        for r, sd in enumerate((sd0, sd1)):
            exp = _shard_like(t, torch.from_numpy(sd[k]), r, 2).numpy()
            np.testing.assert_allclose(sd[k], exp, rtol=2e-3, atol=2e-4, err_msg=f"rank{r}:{k}")
    # every LayerNorm, row-parallel bias and the position table see token shards
    assert "gpt.embeddings.position_embeddings.weight" in sp_names
    assert "gpt.norm.weight" in sp_names and "gpt.layers.0.mlp.linear2.bias" in sp_names
    assert not any("qkv_proj.weight" in n for n in sp_names)
    # overlap structure: every all-gather is issued asynchronously and waited only after the GEMM of this rank's
    # own token block; every dX reduce-scatter of a column-SP backward is waited after the dW GEMM
    for i, ev in enumerate(trace):
        if ev == ("issue", "all_gather"):
            j = trace.index(("wait", "all_gather"), i)
            between = [e for e in trace[i + 1:j] if e[0] == "gemm"]
            assert between, f"all-gather at {i} waited with no GEMM in flight: {trace[i:j + 1]}"
    rs_issues = [i for i, e in enumerate(trace) if e == ("issue", "reduce_scatter") and i > 0
                 and trace[i - 1] == ("gemm", "dgrad")]
    assert len(rs_issues) >= 4  # QKV + FFN1 of two layers
    for i in rs_issues:
        j = trace.index(("wait", "reduce_scatter"), i)
        assert ("gemm", "wgrad") in trace[i + 1:j], trace[i:j + 1]
    assert ("issue", "reduce") in trace  # row-SP forward: reduces pipelined with the next block's GEMM


def _sp_sharding_worker(rank, world, port, q, dp_deg=1):
    paddle = _setup(rank, world, port)
    from paddlepaddle_amd.models.gpt import GPTConfig, GPTForPretraining, GPTPretrainingCriterion
    _, full, _ = _gpt_full(paddle)
    full_sd = {k: v._t.detach().clone() for k, v in full.state_dict().items()}
    fleet = _fleet_init(paddle, mp_degree=2, sharding_degree=2, dp_degree=dp_deg)
    fleet.fleet._strategy.sharding_configs["stage"] = 3
    hcg = fleet.get_hybrid_communicate_group()
    mp_rank = hcg.get_model_parallel_rank()
    data_rank = hcg.get_data_parallel_rank() * 2 + hcg.get_sharding_parallel_rank()
    cfg = GPTConfig.tiny(num_hidden_layers=2, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0,
                         tensor_parallel_degree=2, sequence_parallel=True)
    model, crit = GPTForPretraining(cfg), GPTPretrainingCriterion(cfg)
    with torch.no_grad():
        for k, v in model.state_dict().items():
            v._t.copy_(_shard_like(full_sd[k], v._t, mp_rank, 2))
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    model = fleet.distributed_model(model)
    opt = fleet.distributed_optimizer(opt)
    ids = _data(cfg)
    per = ids.shape[0] // (2 * dp_deg)
    losses = _train(paddle, model, crit, opt, ids[data_rank * per:(data_rank + 1) * per])
    sd = {k: v.numpy() for k, v in model.state_dict().items()}
    q.put((rank, mp_rank, losses, sd))
    paddle.distributed.barrier()


def _sp_sharding_dp2_worker(rank, world, port, q):
    _sp_sharding_worker(rank, world, port, q, dp_deg=2)


def test_dp2_x_sharding_stage3_x_tensor_parallel_sequence_parallel_gpt_eight_ranks():
    """dp-2 x sharding-2 (stage 3) x TP-2 + sequence parallel on 8 gloo ranks: the sequence-parallel grads
    (LayerNorm, row-parallel bias, position table) are summed over mp AND averaged over the dp replicas, so
    every rank's weights match single-process training (the dp all-reduce raced the mp flat)."""
    _check_hybrid(_spawn(_sp_sharding_dp2_worker, world=8), 2)


def test_sharding_stage3_x_tensor_parallel_sequence_parallel_gpt_four_ranks():
    """sharding-2 (stage 3) x TP-2 + sequence parallel: losses and weights match single-process training."""
    _check_hybrid(_spawn(_sp_sharding_worker, world=4), 2)
