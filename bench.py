#!/usr/bin/env python3
"""Headline benchmark: GPT-3 13B pre-training step (Fleet sharding stage-3 over RCCL/xGMI, optionally
composed with tensor parallelism via fleet's hybrid topology; bf16 AMP-O2, fused AdamW, no activation
recompute by default) + ResNet-50 bf16 data-parallel, on N MI355X GPUs of one node.

Metric (BASELINE.json): "tokens/sec GPT-3-13B sharding-3 + ResNet50 img/s, at 1/2/4/8 MI355X".
`value` = whole-job GPT-3 13B training tokens/s; ResNet-50 img/s is reported in `secondary`.
Weak scaling: per-GPU micro-batch fixed as N grows. Data: synthetic tokens / images, random init.

Launch (N>1): python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
              --master-port P bench.py --gpus N --steps K --warmup W
`python bench.py --gpus N` without a launcher starts those N ranks itself (a child torchrun, before any
GPU call) and exits with its status; under a launcher WORLD_SIZE must equal --gpus.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402

BASELINE_METRIC = "tokens/sec GPT-3-13B sharding-3 + ResNet50 img/s, at 1/2/4/8 MI355X"
PEAK_BF16 = 2.5e15


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--model", default="gpt3-13b",
                   help="gpt3-13b | gpt3-6.7b | gpt3-1.3b | tiny | llama2-70b | llama2-13b | llama2-7b | llama-tiny")
    p.add_argument("--pp", type=int, default=1, help="pipeline degree (LLaMA pipeline path)")
    p.add_argument("--vpp", type=int, default=1, help="virtual pipeline stages per rank (interleaved 1F1B)")
    # global batch 16 sequences per GPU either way; GPT-3 13B defaults to 4 x 4 (M = 8192 tokens per GEMM: 2.5
    # rounds of 256x256 tiles on the N = 5120 shapes instead of 1.25, half the gradient-accumulation epilogues;
    # 243 GiB of the 288: 2.3-2.5 % over 2 x 8 on one box, profiles/gpt13b_microbatch_ab_r6.md); the other models 2 x 8
    p.add_argument("--micro-batch", type=int, default=None)
    p.add_argument("--accum", type=int, default=None, help="gradient accumulation steps per optimizer step")
    p.add_argument("--seq-len", type=int, default=2048)
    p.add_argument("--recompute", type=int, default=0)
    p.add_argument("--sharding-stage", type=int, default=3)
    p.add_argument("--pair-wgrad", type=int, default=0,
                   help="GPT: pair the weight-gradient GEMMs of consecutive accumulation micro-batches into one "
                        "K = 2T product (ops/linear.py pair_weight_grads)")
    p.add_argument("--tp", type=int, default=None,
                   help="tensor-parallel degree (GPT: sharding over world/tp ranks). Default: the BASELINE config "
                        "'GPT-3 13B sharding stage-3 + TP=2' -> 2 on any multi-GPU run of GPT, 1 on one GPU")
    p.add_argument("--llama-engine", default="static", choices=["static", "fleet"],
                   help="LLaMA: static-graph auto-parallel (dist.parallelize + dist.to_static, the BASELINE config) "
                        "or the dygraph fleet pipeline")
    p.add_argument("--fused-head-ce", type=int, default=0,
                   help="LM head + cross-entropy over vocabulary slices, logits never materialised (ops/lm_head.py)")
    p.add_argument("--sp", type=int, default=1,
                   help="GPT with tp > 1: sequence parallel (token shards between the TP regions; all-gather / "
                        "reduce-scatter overlapped with the GEMMs, parallel/sequence_parallel.py)")
    p.add_argument("--stage3-keep-params", default="auto",
                   help="sharding stage 3: auto | 1 (keep gathered params resident from first use until the "
                        "optimizer step) | 0 (release after each unit's forward/backward, re-gather per micro-batch)")
    p.add_argument("--static-passes", default="all",
                   help="static LLaMA engine program passes: all | none | comma list of sibling_linears, "
                        "rms_norm_residual (A/B)")
    p.add_argument("--llama-fused-attn", type=int, default=1,
                   help="LLaMA training attention as one qkv->RoPE->flash-attention op (one-buffer qkv gradient)")
    p.add_argument("--resnet", type=int, default=1, help="also run the ResNet-50 DP benchmark")
    p.add_argument("--resnet-batch", type=int, default=256, help="per-GPU ResNet-50 batch")
    p.add_argument("--resnet-steps", type=int, default=10)
    p.add_argument("--resnet-graph", type=int, default=1,
                   help="capture the ResNet-50 training step into a hipGraph and replay it (1 GPU only; "
                        "round 5 same-box A/B: 9,456 / 9,475 vs 9,245 / 9,308 img/s eager, "
                        "profiles/resnet50_graph_ab_r5.log); multi-rank runs keep eager steps")
    p.add_argument("--resnet-layout", default="nhwc", choices=["nhwc", "nchw-autotune"],
                   help="nhwc: channels-last model; nchw-autotune: Paddle's default NCHW model with "
                        "FLAGS_layout_autotune (NHWC kernels on channels-last views)")
    p.add_argument("--skip-gpt", type=int, default=0)
    p.add_argument("--allocator", default="native", choices=["native", "torch"],
                   help="device allocator: the framework's auto-growth best-fit allocator or PyTorch's")
    a = p.parse_args()
    mb, acc = (4, 4) if a.model == "gpt3-13b" else (2, 8)
    a.micro_batch = mb if a.micro_batch is None else a.micro_batch
    a.accum = acc if a.accum is None else a.accum
    return a


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def _dev():
    from paddlepaddle_amd.framework.place import _get_torch_device
    return _get_torch_device()


def _sync():
    if torch.cuda.is_available() and _dev().type == "cuda":
        torch.cuda.synchronize()


def timed(step_fn, steps, warmup, dist_on):
    import torch.distributed as dist
    for _ in range(warmup):
        step_fn()
    if dist_on:
        dist.barrier()
    _sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step_fn()
    _sync()
    if dist_on:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([dt], device=_dev())
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def gpt_bench(args, paddle, world, dist_on):
    from paddlepaddle_amd.models.gpt import GPTConfig, GPTForPretraining, GPTPretrainingCriterion
    cfgs = {"gpt3-13b": GPTConfig.gpt3_13b, "gpt3-6.7b": GPTConfig.gpt3_6_7b, "gpt3-1.3b": GPTConfig.gpt3_1_3b,
            "tiny": GPTConfig.tiny}
    tp = args.tp
    if world % tp:
        raise SystemExit(f"world {world} is not a multiple of tp {tp}")
    n_shard = world // tp
    data_rank = int(os.environ.get("RANK", "0"))
    shard_group = None
    if world > 1 or tp > 1:
        # fleet hybrid topology: mp = tp (contiguous ranks: one xGMI hop), sharding = world / tp
        from paddlepaddle_amd.distributed import fleet
        st = fleet.DistributedStrategy()
        st.hybrid_configs = dict(dp_degree=1, mp_degree=tp, pp_degree=1, sharding_degree=n_shard)
        fleet.init(is_collective=True, strategy=st)
        hcg = fleet.get_hybrid_communicate_group()
        data_rank = hcg.get_sharding_parallel_rank()
        shard_group = hcg.get_sharding_parallel_group()
    cfg = cfgs[args.model](max_position_embeddings=max(args.seq_len, 128), use_recompute=bool(args.recompute),
                           tensor_parallel_degree=tp, sequence_parallel=bool(args.sp) and tp > 1,
                           fused_head_ce=bool(args.fused_head_ce))
    paddle.set_default_dtype("bfloat16")
    paddle.seed(1234)
    t0 = time.time()
    model = GPTForPretraining(cfg)
    crit = GPTPretrainingCriterion(cfg)
    paddle.set_default_dtype("float32")
    nparams = sum(p.size for p in model.parameters())
    log(f"[gpt] built {args.model}: {nparams / 1e9:.2f}B params in {time.time() - t0:.1f}s")
    clip = paddle.nn.ClipGradByGlobalNorm(1.0)
    opt = paddle.optimizer.AdamW(learning_rate=1e-4, parameters=model.parameters(), weight_decay=0.01,
                                 grad_clip=clip, multi_precision=True,
                                 apply_decay_param_fun=lambda n: not ("norm" in n or n.endswith("b_0")))
    keep = None
    if args.sharding_stage > 0:  # same engine at every N (at N=1 the collectives are no-ops)
        from paddlepaddle_amd.distributed.sharding import group_sharded_parallel
        from paddlepaddle_amd.framework.flags import set_flags
        set_flags({"FLAGS_sharding_stage3_keep_params": args.stage3_keep_params})
        level = {1: "os", 2: "os_g", 3: "p_g_os"}[args.sharding_stage]
        model, opt, _ = group_sharded_parallel(model, opt, level=level, group=shard_group)
        keep = model._engine.keep_params
    elif world > 1:
        model = paddle.DataParallel(model)
    B, S = args.micro_batch, args.seq_len
    dev = _dev()
    # tensor-parallel ranks see the same tokens; sharding ranks see different ones
    gen = torch.Generator(device=dev).manual_seed(7 + data_rank)
    data = torch.randint(0, cfg.vocab_size, (args.accum, B, S + 1), device=dev, generator=gen)
    ids = [paddle.Tensor(data[i, :, :-1]) for i in range(args.accum)]
    lbl = [paddle.Tensor(data[i, :, 1:]) for i in range(args.accum)]
    state = {}
    import contextlib
    no_sync = getattr(model, "no_sync", None)

    from paddlepaddle_amd.ops import linear as LIN

    def step():
        for a in range(args.accum):
            # accumulation micro-batches skip the gradient reduce-scatter / all-reduce; the last one
            # reduces (overlapped with its backward)
            ctx = no_sync() if (no_sync is not None and n_shard > 1 and a < args.accum - 1) else \
                contextlib.nullcontext()
            # weight-gradient pairing (ops/linear.py): even micro-batches queue their dW GEMMs, the next one runs
            # each weight's pair as one K = 2T product into the main grad (every queued job is done inside it)
            pair = None
            if args.pair_wgrad and args.accum > 1:
                pair = "defer" if (a % 2 == 0 and a + 1 < args.accum) else "merge"
            with ctx, LIN.pair_weight_grads(pair):
                if cfg.fused_head_ce and tp == 1:
                    loss = model(ids[a], labels=lbl[a])
                else:
                    loss = crit(model(ids[a]), lbl[a])
                if args.accum > 1:
                    loss = loss * (1.0 / args.accum)
                loss.backward()
        opt.step()
        opt.clear_grad()
        state["loss"] = loss

    dt = timed(step, args.steps, args.warmup, dist_on)
    tokens = args.steps * args.accum * B * S * n_shard
    tps = tokens / dt
    fpt = cfg.flops_per_token(S, recompute=False)
    mfu = tps * fpt / (PEAK_BF16 * world)  # 6N + causal attention FLOPs
    # strict 6N: parameter GEMM FLOPs only (non-embedding parameters), the attention score / value products left out
    gpt_bench.mfu_strict = tps * 6 * (cfg.num_params() - cfg.max_position_embeddings * cfg.hidden_size) / (
        PEAK_BF16 * world)
    mem = paddle.device.cuda.max_memory_allocated() / 2**30 if dev.type == "cuda" else 0.0
    log(f"[gpt] loss={float(state['loss']):.4f} step={dt / args.steps * 1000:.1f}ms tokens/s={tps:.0f} "
        f"MFU(6N + attention)={mfu * 100:.1f}% MFU(strict 6N)={gpt_bench.mfu_strict * 100:.1f}% mem={mem:.1f}GiB")
    try:
        from paddlepaddle_amd.ops import gemm as _G
        ch = _G.choices()
        log(f"[gpt] GEMM backend per shape: {sum(v.startswith('hip') for v in ch.values())} hand-written / "
            f"{sum(v == 'blas' for v in ch.values())} hipBLASLt: " +
            "; ".join(f"{k[0]}{list(k[1:4])}={v}" for k, v in sorted(ch.items(), key=str)))
    except Exception:  # pragma: no cover
        pass
    del model, opt, ids, lbl
    if dev.type == "cuda":
        paddle.device.cuda.empty_cache()
    gpt_bench.keep_params = keep
    return tps, dt / args.steps * 1000, B * args.accum * n_shard, mfu


LLAMA_TP_PLAN = {
    "layers.*.self_attn.q_proj": "col", "layers.*.self_attn.k_proj": "col", "layers.*.self_attn.v_proj": "col",
    "layers.*.self_attn.qkv_proj": "col", "layers.*.self_attn.o_proj": "row", "layers.*.mlp.gate_proj": "col",
    "layers.*.mlp.up_proj": "col", "layers.*.mlp.gate_up_proj": "col", "layers.*.mlp.down_proj": "row",
    "lm_head": "col", "embed_tokens": "row"}  # vocab-parallel embedding and (engine) vocab-parallel cross entropy


def llama_static_bench(args, paddle, world, dist_on):
    """LLaMA-2 pre-training the BASELINE way: static-graph semi-auto parallel. A plain single-card LLaMA is
    distributed by plan (dist.parallelize: pipeline split over the decoder layers, ColWise / RowWise tensor
    parallel), then dist.to_static traces it once, propagates placements, partitions the program per rank
    (explicit RCCL collectives + stage-to-stage p2p) and runs a 1F1B schedule over the micro-batches;
    bf16 weights, AdamW with fp32 master weights."""
    import numpy as np
    import paddlepaddle_amd.distributed as dist
    from paddlepaddle_amd.models.llama_auto import LlamaConfig, LlamaForCausalLMAuto, LlamaPretrainingCriterionAuto
    pp, tp = args.pp, args.tp
    if world % (pp * tp):
        raise SystemExit(f"world {world} is not a multiple of pp*tp = {pp * tp}")
    dp = world // (pp * tp)
    presets = {"llama2-70b": LlamaConfig.llama2_70b, "llama2-13b": LlamaConfig.llama2_13b,
               "llama2-7b": LlamaConfig.llama2_7b, "llama-tiny": LlamaConfig.tiny,
               # one rank of the BASELINE LLaMA-2 70B PP4 x TP2 layout on one GPU: a pipeline stage's 20 layers at
               # the tensor-parallel-local widths (hidden 8192, 32 of the 64 query heads, 4 of the 8 KV heads,
               # ffn 28672 / 2), embedding and LM head included (the first / last stage's extra weights)
               "llama2-70b-stage": lambda **kw: LlamaConfig.llama2_70b(
                   num_hidden_layers=20, num_attention_heads=32, num_key_value_heads=4, intermediate_size=14336,
                   attention_head_dim=128, **kw)}
    extra = {"num_hidden_layers": max(2, 2 * pp)} if args.model == "llama-tiny" else {}
    # one [q|k|v] and one [gate|up] projection per tensor-parallel rank (PaddleNLP fuse_attention_qkv /
    # fuse_attention_ffn): the projection gradients come back as one buffer each (ops.qkv_rope_attention, swiglu)
    fused = dict(fuse_attention_qkv=bool(args.llama_fused_attn), fuse_attention_ffn=bool(args.llama_fused_attn),
                 tensor_parallel_degree=tp)
    cfg = presets[args.model](max_position_embeddings=max(args.seq_len, 128), **extra, **fused)
    dist.auto_parallel.set_mesh(None)
    paddle.set_default_dtype("bfloat16")
    paddle.seed(1234)
    model, crit = LlamaForCausalLMAuto(cfg), LlamaPretrainingCriterionAuto(cfg)
    paddle.set_default_dtype("float32")
    opt = paddle.optimizer.AdamW(learning_rate=1e-4, parameters=model.parameters(), weight_decay=0.01,
                                 multi_precision=True, grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    mesh = dist.ProcessMesh(np.arange(world).reshape(pp, dp, tp), dim_names=["pp", "dp", "mp"])
    plan = {k: (dist.ColWiseParallel() if v == "col" else dist.RowWiseParallel()) for k, v in LLAMA_TP_PLAN.items()}
    model, opt = dist.parallelize(model, opt, mesh, dp_config={"sharding_level": 0},
                                  mp_config={"parallelize_plan": plan}, pp_config={"split_spec": "layers"})
    strategy = dist.Strategy()
    strategy.pipeline.enable = True
    strategy.pipeline.schedule_mode = "1F1B"
    strategy.pipeline.accumulate_steps = args.accum
    strategy.pipeline.micro_batch_size = args.micro_batch
    strategy.recompute.enable = bool(args.recompute)  # each decoder layer a checkpointed segment of the program
    strategy.mp_optimization["allreduce_matmul_grad_overlapping"] = True  # TP dX all-reduce beside the dW GEMM
    sp = args.static_passes.split(",") if args.static_passes not in ("all", "none") else []
    if args.static_passes != "all":  # A/B of the engine's program passes
        strategy.fused_passes["sibling_linears"] = "sibling_linears" in sp
        strategy.fused_passes["rms_norm_residual"] = "rms_norm_residual" in sp
    dm = dist.to_static(model, None, crit, opt, strategy)
    if args.model == "llama2-70b-stage":
        # the proxy runs stage 0 of the PP4 1F1B pipeline: its job list (3 warm-up forwards, then 1F1B, so at most
        # 4 micro-batches in flight whatever accumulate_steps is); no p2p on one GPU, so no bubble is measured
        from paddlepaddle_amd.parallel.pp_schedules import one_f_one_b
        dm._engine._job_list = lambda mode, nst, s, n: one_f_one_b(4, 0, n)
    dev = _dev()
    gb = args.micro_batch * args.accum * dp
    gen = torch.Generator(device=dev).manual_seed(7)
    data = torch.randint(0, cfg.vocab_size, (gb, args.seq_len + 1), device=dev, generator=gen)
    x, y = paddle.Tensor(data[:, :-1].contiguous()), paddle.Tensor(data[:, 1:].contiguous())
    state = {}

    def step():
        state["loss"] = dm(x, y)

    dt = timed(step, args.steps, args.warmup, dist_on)
    tokens = args.steps * gb * args.seq_len
    tps = tokens / dt
    mfu = tps * cfg.flops_per_token(args.seq_len) / (PEAK_BF16 * world)
    mem = paddle.device.cuda.max_memory_allocated() / 2**30 if dev.type == "cuda" else 0.0
    eng = dm._engine
    log(f"[llama-static] {args.model} pp{pp} tp{tp} dp{dp}: loss={float(state['loss']):.4f} "
        f"step={dt / args.steps * 1000:.1f}ms tokens/s={tps:.0f} MFU={mfu * 100:.1f}% peak_mem={mem:.1f}GiB "
        f"params={cfg.num_params() / 1e9:.2f}B passes={getattr(eng, 'pass_stats', {})} "
        f"recompute_segments={getattr(eng, 'n_segments', 0)} fused_grad_params={getattr(eng, 'fused_grads', 0)} "
        f"native_stages={ {k: (v.num_native, v.num_py, v.num_instructions, v.runs) for k, v in getattr(eng, '_native', {}).items()} } "
        f"native_reason={getattr(eng, 'native_reason', {})}")
    return tps, dt / args.steps * 1000, gb, mfu


def llama_bench(args, paddle, world, dist_on):
    """LLaMA-2 pre-training with fleet hybrid parallel: PP (1F1B / interleaved) x TP x DP, bf16 AMP-O2 params,
    fused AdamW with fp32 master weights. BASELINE config: LLaMA-2 70B PP4 x TP2 on 8 MI355X."""
    from paddlepaddle_amd.distributed import fleet
    from paddlepaddle_amd.models.llama import LlamaConfig, LlamaForCausalLMPipe
    pp, tp = args.pp, args.tp
    if world % (pp * tp):
        raise SystemExit(f"world {world} is not a multiple of pp*tp = {pp * tp}")
    dp = world // (pp * tp)
    st = fleet.DistributedStrategy()
    st.hybrid_configs = dict(dp_degree=dp, mp_degree=tp, pp_degree=pp)
    st.pipeline_configs = {"accumulate_steps": args.accum, "micro_batch_size": args.micro_batch}
    fleet.init(is_collective=True, strategy=st)
    presets = {"llama2-70b": LlamaConfig.llama2_70b, "llama2-13b": LlamaConfig.llama2_13b,
               "llama2-7b": LlamaConfig.llama2_7b, "llama-tiny": LlamaConfig.tiny}
    cfg = presets[args.model](max_position_embeddings=max(args.seq_len, 128), tensor_parallel_degree=tp,
                              use_recompute=bool(args.recompute), fused_qkv_attention=bool(args.llama_fused_attn))
    paddle.set_default_dtype("bfloat16")
    paddle.seed(1234)
    model = LlamaForCausalLMPipe(cfg, num_stages=pp, num_virtual_pipeline_stages=args.vpp if args.vpp > 1 else None,
                                 recompute_interval=1 if args.recompute else 0)
    paddle.set_default_dtype("float32")
    opt = paddle.optimizer.AdamW(learning_rate=1e-4, parameters=model.parameters(), weight_decay=0.01,
                                 multi_precision=True, grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    model = fleet.distributed_model(model)
    opt = fleet.distributed_optimizer(opt)
    dev = _dev()
    gb = args.micro_batch * args.accum
    gen = torch.Generator(device=dev).manual_seed(7 + fleet.get_hybrid_communicate_group().get_data_parallel_rank())
    data = torch.randint(0, cfg.vocab_size, (gb, args.seq_len + 1), device=dev, generator=gen)
    x, y = paddle.Tensor(data[:, :-1].contiguous()), paddle.Tensor(data[:, 1:].contiguous())
    state = {}

    if pp > 1:
        def step():
            state["loss"] = model.train_batch([x, y], opt)
    else:  # no pipeline: plain gradient accumulation over the same PipelineLayer
        mbs = [(paddle.Tensor(c), paddle.Tensor(d)) for c, d in zip(x._t.chunk(args.accum), y._t.chunk(args.accum))]
        crit = model._layers._loss_fn if hasattr(model, "_layers") else model._loss_fn

        from paddlepaddle_amd.ops.linear import fuse_grad_accumulation
        fused = {"params": None}

        def step():
            # wgrad GEMMs / norm kernels accumulate the micro-batches' weight gradients into .grad in place
            fused["params"] = fuse_grad_accumulation(model, fused["params"])
            for xi, yi in mbs:
                loss = crit(model(xi), yi) * (1.0 / args.accum)
                loss.backward()
            opt.step()
            opt.clear_grad()
            state["loss"] = loss

    dt = timed(step, args.steps, args.warmup, dist_on)
    tokens = args.steps * gb * dp * args.seq_len
    tps = tokens / dt
    mfu = tps * cfg.flops_per_token(args.seq_len) / (PEAK_BF16 * world)
    log(f"[llama] {args.model} pp{pp} tp{tp} dp{dp}: loss={float(state['loss']):.4f} step={dt / args.steps * 1000:.1f}ms "
        f"tokens/s={tps:.0f} MFU={mfu * 100:.1f}%")
    return tps, dt / args.steps * 1000, gb * dp, mfu


def resnet_bench(args, paddle, world, dist_on):
    from paddlepaddle_amd.vision.models import resnet50
    paddle.seed(99)
    nchw = getattr(args, "resnet_layout", "nhwc") == "nchw-autotune"
    if nchw:
        paddle.set_flags({"FLAGS_layout_autotune": True})
    model = resnet50(num_classes=1000, data_format="NCHW" if nchw else "NHWC")
    opt = paddle.optimizer.Momentum(learning_rate=0.1, momentum=0.9, parameters=model.parameters(),
                                    weight_decay=1e-4, multi_precision=True)
    model, opt = paddle.amp.decorate(model, opt, level="O2", dtype="bfloat16")
    if world > 1:
        model = paddle.DataParallel(model)
    B = args.resnet_batch
    x = paddle.Tensor(torch.randn(*((B, 3, 224, 224) if nchw else (B, 224, 224, 3)), device=_dev(),
                                  dtype=torch.bfloat16))
    y = paddle.Tensor(torch.randint(0, 1000, (B,), device=_dev()))

    def step():
        with paddle.amp.auto_cast(level="O2", dtype="bfloat16"):
            out = model(x)
        loss = paddle.nn.functional.cross_entropy(out.astype("float32"), y)
        loss.backward()
        opt.step()
        # release the gradients (paddle's set_to_zero=False) instead of zero-filling them: the next backward
        # then writes each gradient instead of accumulating into a zeroed buffer (no fill + add per parameter)
        opt.clear_grad(set_to_zero=False)

    run = step
    resnet_bench.graph = False
    if args.resnet_graph and world == 1 and torch.cuda.is_available():
        # the whole training step (forward, backward, optimizer) captured once into a hipGraph after the warm-up
        # steps (per-shape backend choices, MIOpen find and optimizer state are settled by then) and replayed:
        # one launch per step instead of ~3000 (device/cuda/graphs.py; the framework's documented path for
        # launch-bound loops). Multi-rank runs keep eager steps (the gradient all-reduce is not captured).
        for _ in range(max(args.warmup, 3)):
            step()
        torch.cuda.synchronize()
        from paddlepaddle_amd.device.cuda.graphs import CUDAGraph
        try:
            g = CUDAGraph()
            g.capture_begin()
            try:
                step()
            finally:
                g.capture_end()
            run = g.replay
            resnet_bench.graph = True
        except Exception as e:  # pragma: no cover - capture unsupported here: keep eager steps
            log(f"[resnet50] hipGraph capture failed ({type(e).__name__}: {e}); timing eager steps")
            torch.cuda.synchronize()
    dt = timed(run, args.resnet_steps, max(args.warmup, 3), dist_on)
    ips = args.resnet_steps * B * world / dt
    log(f"[resnet50] step={dt / args.resnet_steps * 1000:.1f}ms img/s={ips:.0f}" +
        (" (hipGraph replay of the whole step)" if resnet_bench.graph else ""))
    try:
        from paddlepaddle_amd.ops import gemm as _G
        names = {"convf": "forward", "convd": "data grad", "convw": "weight grad"}
        for kind, what in names.items():
            cv = {k: v for k, v in _G.choices().items() if k[0] == kind}
            own = sum(v in ("hip", "hipu", "hip128", "skinny") for v in cv.values())
            log(f"[resnet50] conv {what} backend per shape: {own} hand-written "
                f"({sum(v == 'skinny' for v in cv.values())} on the memory-bound skinny kernel) / "
                f"{sum(v == 'mm' for v in cv.values())} hipBLASLt / {sum(v == 'blas' for v in cv.values())} MIOpen")
    except Exception:  # pragma: no cover
        pass
    return ips


def _relaunch(args):
    """--gpus N with no launcher: run N ranks under torch.distributed.run as a child process (this process
    has not touched the GPU) and exit with its status."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    sys.exit(subprocess.call(cmd, env=env))


def _native_alloc_on():
    try:
        from paddlepaddle_amd.device import allocator as A
        return A.is_enabled()
    except Exception:  # pragma: no cover
        return False


def main():
    args = parse()
    if args.tp is None:
        args.tp = 2 if (args.gpus > 1 and args.gpus % 2 == 0 and not args.model.startswith("llama")) else 1
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        _relaunch(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    if args.allocator == "native":
        os.environ.setdefault("PADDLE_AMD_ALLOCATOR", "auto_growth")  # installed at package import
    import paddlepaddle_amd as paddle
    dist_on = world > 1
    if dist_on:
        paddle.distributed.init_parallel_env()
    elif torch.cuda.is_available() and os.environ.get("PADDLE_AMD_FORCE_CPU", "0") != "1":
        torch.cuda.set_device(0)
    tps = step_ms = gb = mfu = None
    is_llama = args.model.startswith("llama")
    if is_llama:
        fn = llama_static_bench if args.llama_engine == "static" else llama_bench
        tps, step_ms, gb, mfu = fn(args, paddle, world, dist_on)
        args.resnet = 0
    elif not args.skip_gpt:
        tps, step_ms, gb, mfu = gpt_bench(args, paddle, world, dist_on)
    ips = resnet_bench(args, paddle, world, dist_on) if args.resnet else None
    if int(os.environ.get("RANK", "0")) == 0:
        ns = world // max(args.tp, 1)
        par = (f"sharding_stage{args.sharding_stage}_degree{ns}" if args.sharding_stage else f"dp{ns}") + \
              (f"_tp{args.tp}" if args.tp > 1 else "") + ("_sp" if (args.tp > 1 and args.sp) else "")
        if is_llama:
            par = f"pp{args.pp}_tp{args.tp}_dp{world // (args.pp * args.tp)}" + (f"_vpp{args.vpp}" if args.vpp > 1 else "")
            if args.llama_engine == "static":
                par += "_static_auto_parallel"
        metric = BASELINE_METRIC if args.model == "gpt3-13b" else \
            f"tokens/sec {args.model} training ({par})"
        line = {
            "metric": metric,
            "value": round(tps, 1) if tps is not None else None,
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_ms, 2) if step_ms is not None else None,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic tokens/images, random-init weights",
            "config": {"model": f"GPT-3 {args.model.split('-')[-1].upper()} (h5120 L40 a40 ffn20480 V50304)"
                       if args.model == "gpt3-13b" else args.model.replace("llama2-", "LLaMA-2 ").upper()
                       if is_llama else args.model,
                       "global_batch": gb, "seq_len": args.seq_len, "micro_batch": args.micro_batch,
                       "accum_steps": args.accum, "parallelism": par, "recompute": bool(args.recompute),
                       "fused_head_ce": bool(args.fused_head_ce),
                       **({"paired_wgrad": bool(args.pair_wgrad and args.accum > 1)} if not is_llama else {}),
                       "optimizer": "AdamW fp32-master fused HIP", "amp": "O2 bf16",
                       "allocator": ("native auto-growth best-fit" if _native_alloc_on() else "torch caching"),
                       **({"stage3_params": ("gathered once per step, resident until the optimizer step"
                                             if getattr(gpt_bench, "keep_params", None) else
                                             "released after each block, re-gathered per micro-batch")}
                          if (args.sharding_stage == 3 and not is_llama and world // max(args.tp, 1) > 1) else {})},
            # model-FLOPs utilisation at the 2.5 PF dense bf16 peak: 6N plus the causal attention products, and the
            # strict 6N form (parameter GEMMs only)
            "mfu_6N_plus_attn": round(mfu, 4) if mfu is not None else None,
            "mfu_6N_strict": (round(gpt_bench.mfu_strict, 4) if (mfu is not None and not is_llama
                                                                  and hasattr(gpt_bench, "mfu_strict")) else None),
            "secondary": {"metric": "ResNet50 img/s (bf16 NHWC, DP)", "value": round(ips, 1) if ips else None,
                          "per_gpu_batch": args.resnet_batch,
                          "step": "hipGraph replay" if getattr(resnet_bench, "graph", False) else "eager"},
        }
        print(json.dumps(line), flush=True)
    dump = os.environ.get("PADDLE_AMD_TUNING_DUMP")
    if dump and int(os.environ.get("RANK", "0")) == 0:  # refresh paddlepaddle_amd/ops/tuning/<arch>.json
        from paddlepaddle_amd.ops import gemm as _G
        _G.dump_tuning_table(dump)
    if dist_on:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
