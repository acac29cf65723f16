"""Multi-process (gloo, world_size=2, CPU) tests of collectives, DataParallel and sharding stage 1/2/3.
Each parallel run must reproduce single-process full-batch training of the same model."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(rank, world, port):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), PADDLE_AMD_FORCE_CPU="1")
    import paddlepaddle_amd as paddle
    paddle.distributed.init_parallel_env(backend="gloo")
    return paddle


def _make_model(paddle):
    from paddlepaddle_amd.models.gpt import GPTConfig, GPTForPretraining, GPTPretrainingCriterion
    paddle.seed(11)
    cfg = GPTConfig.tiny(num_hidden_layers=3, hidden_dropout_prob=0.0)
    return cfg, GPTForPretraining(cfg), GPTPretrainingCriterion(cfg)


def _data(cfg):
    g = torch.Generator().manual_seed(5)
    return torch.randint(0, cfg.vocab_size, (4, 17), generator=g)


def _train(paddle, model, crit, opt, ids, steps=3):
    losses = []
    for _ in range(steps):
        loss = crit(model(ids[:, :-1]), ids[:, 1:])
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    return losses


def _collectives_worker(rank, world, port, q):
    paddle = _setup(rank, world, port)
    import paddlepaddle_amd.distributed as dist
    t = paddle.to_tensor([float(rank + 1)] * 4)
    dist.all_reduce(t)
    out = {"allreduce": t.numpy().tolist()}
    lst = []
    dist.all_gather(lst, paddle.to_tensor([rank]))
    out["allgather"] = [int(x.numpy()[0]) for x in lst]
    b = paddle.to_tensor([rank * 10])
    dist.broadcast(b, src=1)
    out["broadcast"] = int(b.numpy()[0])
    rs = paddle.zeros([2])
    dist.reduce_scatter(rs, [paddle.to_tensor([1.0, 2.0]), paddle.to_tensor([3.0, 4.0])])
    out["reduce_scatter"] = rs.numpy().tolist()
    objs = []
    dist.all_gather_object(objs, {"r": rank})
    out["objs"] = objs
    outs = []
    dist.alltoall(outs, [paddle.to_tensor([rank * 2]), paddle.to_tensor([rank * 2 + 1])])
    out["alltoall"] = [int(x.numpy()[0]) for x in outs]
    q.put((rank, out))
    dist.barrier()


def _dp_worker(rank, world, port, mode, q):
    paddle = _setup(rank, world, port)
    cfg, model, crit = _make_model(paddle)
    ids = _data(cfg)
    local = ids[rank * 2:(rank + 1) * 2]
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    if mode == "dp":
        model = paddle.DataParallel(model)
    else:
        from paddlepaddle_amd.distributed.sharding import group_sharded_parallel
        level, _, off = mode.partition("+")
        model, opt, _ = group_sharded_parallel(model, opt, level=level, offload=off == "offload")
    losses = _train(paddle, model, crit, opt, paddle.Tensor(local))
    if mode.endswith("+offload"):
        assert model._engine.offloaded_bytes() > 0
    sd = {k: v.numpy() for k, v in model.state_dict().items()}
    q.put((rank, losses, sd))
    paddle.distributed.barrier()


def _spawn(fn, *args, world=2):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=fn, args=(r, world, port, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    import time
    res = []
    try:
        deadline = time.time() + 240
        while len(res) < world:
            try:
                res.append(q.get(timeout=1))
            except queue.Empty:
                dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
                if dead or time.time() > deadline:
                    raise RuntimeError(f"worker failed (exit codes {dead})" if dead else "workers timed out")
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    for p in procs:
        p.join(timeout=60)
    return sorted(res, key=lambda x: x[0])


def test_collectives_gloo():
    res = _spawn(_collectives_worker)
    for rank, out in res:
        assert out["allreduce"] == [3.0] * 4
        assert out["allgather"] == [0, 1]
        assert out["broadcast"] == 10
        assert out["objs"] == [{"r": 0}, {"r": 1}]
    assert res[0][1]["reduce_scatter"] == [2.0, 4.0] and res[1][1]["reduce_scatter"] == [6.0, 8.0]
    assert res[0][1]["alltoall"] == [0, 2] and res[1][1]["alltoall"] == [1, 3]


def _reference():
    sys.path.insert(0, ROOT)
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    cfg, model, crit = _make_model(paddle)
    ids = _data(cfg)
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    # full batch == mean of the two half-batch losses (equal sizes)
    losses = []
    for _ in range(3):
        l0 = crit(model(paddle.Tensor(ids[:2, :-1])), paddle.Tensor(ids[:2, 1:]))
        l1 = crit(model(paddle.Tensor(ids[2:, :-1])), paddle.Tensor(ids[2:, 1:]))
        loss = (l0 + l1) * 0.5
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    return losses, {k: v.numpy() for k, v in model.state_dict().items()}


@pytest.mark.parametrize("mode", ["dp", "os", "os_g", "p_g_os", "p_g_os+offload"])
def test_data_parallel_and_sharding_match_single_process(mode):
    ref_losses, ref_sd = _reference()
    res = _spawn(_dp_worker, mode)
    (_, l0, sd0), (_, l1, sd1) = res
    np.testing.assert_allclose((np.array(l0) + np.array(l1)) / 2, ref_losses, rtol=1e-4, atol=1e-5)
    for k in ref_sd:
        np.testing.assert_allclose(sd0[k], ref_sd[k], rtol=2e-3, atol=2e-4, err_msg=f"{mode}:{k}")
        np.testing.assert_allclose(sd1[k], sd0[k], rtol=0, atol=0, err_msg=f"{mode}:{k} replicas differ")


def _accum_worker(rank, world, port, level, keep, q):
    paddle = _setup(rank, world, port)
    paddle.set_flags({"FLAGS_sharding_stage3_keep_params": keep})
    cfg, model, crit = _make_model(paddle)
    ids = _data(cfg)
    local = ids[rank * 2:(rank + 1) * 2]
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    from paddlepaddle_amd.distributed.sharding import group_sharded_parallel
    model, opt, _ = group_sharded_parallel(model, opt, level=level)
    assert model._engine.keep_params == (level == "p_g_os" and keep == "1")
    for _ in range(2):
        for a in range(2):  # 2 micro-batches of 1 sequence; first one without reduce-scatter
            x = paddle.Tensor(local[a:a + 1])
            ctx = model.no_sync() if a == 0 else __import__("contextlib").nullcontext()
            with ctx:
                loss = crit(model(x[:, :-1]), x[:, 1:]) * 0.5
                loss.backward()
        opt.step()
        opt.clear_grad()
    sd = {k: v.numpy() for k, v in model.state_dict().items()}
    q.put((rank, sd))
    paddle.distributed.barrier()


@pytest.mark.parametrize("level,keep", [("os_g", "auto"), ("p_g_os", "0"), ("p_g_os", "1")])
def test_sharding_no_sync_accumulation_matches_single_process(level, keep):
    """no_sync micro-batches + (stage 3) resident gathered params == single-process accumulation."""
    sys.path.insert(0, ROOT)
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    cfg, model, crit = _make_model(paddle)
    ids = _data(cfg)
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    for _ in range(2):
        # global batch = 4 sequences = 2 ranks x 2 micro-batches; mean over everything
        for i in range(4):
            x = paddle.Tensor(ids[i:i + 1])
            loss = crit(model(x[:, :-1]), x[:, 1:]) * 0.25
            loss.backward()
        opt.step()
        opt.clear_grad()
    ref = {k: v.numpy() for k, v in model.state_dict().items()}
    (_, sd0), (_, sd1) = _spawn(_accum_worker, level, keep)
    for k in ref:
        np.testing.assert_allclose(sd0[k], ref[k], rtol=2e-3, atol=2e-4, err_msg=f"{level}/{keep}:{k}")
        np.testing.assert_allclose(sd1[k], sd0[k], rtol=0, atol=0)


@pytest.mark.parametrize("level", ["os", "os_g", "p_g_os"])
def test_sharding_degree1_matches_plain(level):
    """Degree-1 sharding (single process, no collectives) must equal plain training, incl. accumulation."""
    sys.path.insert(0, ROOT)
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.distributed.sharding import group_sharded_parallel

    def run(shard):
        cfg, model, crit = _make_model(paddle)
        ids = _data(cfg)
        opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(),
                                     grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
        if shard:
            model, opt, _ = group_sharded_parallel(model, opt, level=level)
        for _ in range(2):
            for a in range(2):  # gradient accumulation
                sl = slice(a * 2, a * 2 + 2)
                loss = crit(model(paddle.Tensor(ids[sl, :-1])), paddle.Tensor(ids[sl, 1:])) * 0.5
                loss.backward()
            opt.step()
            opt.clear_grad()
        return {k: v.numpy() for k, v in model.state_dict().items()}

    ref, got = run(False), run(True)
    for k in ref:
        np.testing.assert_allclose(got[k], ref[k], rtol=1e-5, atol=1e-6, err_msg=k)


# ----------------------------------------------------------------------------- SyncBatchNorm
def _sbn_data(fmt):
    g = torch.Generator().manual_seed(21)
    shape = (4, 6, 5, 3) if fmt == "NCHW" else (4, 5, 3, 6)
    return torch.randn(*shape, generator=g) * 2 + 0.5, torch.randn(*shape, generator=g)


def _sbn_worker(rank, world, port, fmt, q):
    paddle = _setup(rank, world, port)
    x, r = _sbn_data(fmt)
    per = x.shape[0] // world
    xs = paddle.Tensor(x[rank * per:(rank + 1) * per].clone())
    xs.stop_gradient = False
    bn = paddle.nn.SyncBatchNorm(6, data_format=fmt)
    with torch.no_grad():
        bn.weight._t.copy_(torch.linspace(0.5, 1.5, 6))
        bn.bias._t.copy_(torch.linspace(-0.2, 0.3, 6))
    y = bn(xs)
    (y * paddle.Tensor(r[rank * per:(rank + 1) * per])).sum().backward()
    q.put((rank, y.numpy(), xs.grad.numpy(), bn.weight.grad.numpy(), bn.bias.grad.numpy(), bn._mean.numpy(),
           bn._variance.numpy()))
    paddle.distributed.barrier()


def _sbn_reference(fmt):
    sys.path.insert(0, ROOT)
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    x, r = _sbn_data(fmt)
    xt = paddle.Tensor(x.clone())
    xt.stop_gradient = False
    bn = paddle.nn.BatchNorm2D(6, data_format=fmt)
    with torch.no_grad():
        bn.weight._t.copy_(torch.linspace(0.5, 1.5, 6))
        bn.bias._t.copy_(torch.linspace(-0.2, 0.3, 6))
    y = bn(xt)
    (y * paddle.Tensor(r)).sum().backward()
    return y.numpy(), xt.grad.numpy(), bn.weight.grad.numpy(), bn.bias.grad.numpy(), bn._mean.numpy(), \
        bn._variance.numpy()


@pytest.mark.parametrize("fmt", ["NCHW", "NHWC"])
def test_sync_batch_norm_matches_full_batch(fmt):
    """2 ranks x half batch == BatchNorm2D on the full batch: outputs, input gradients (cross-rank
    terms included), summed weight/bias gradients and running statistics (sync_batch_norm_utils.h:575)."""
    y, dx, dw, db, rm, rv = _sbn_reference(fmt)
    res = sorted(_spawn(_sbn_worker, fmt), key=lambda t: t[0])
    np.testing.assert_allclose(np.concatenate([t[1] for t in res]), y, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(np.concatenate([t[2] for t in res]), dx, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(res[0][3] + res[1][3], dw, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(res[0][4] + res[1][4], db, rtol=1e-5, atol=1e-5)
    for t in res:
        np.testing.assert_allclose(t[5], rm, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(t[6], rv, rtol=1e-5, atol=1e-6)


def _native_engine_worker(rank, world, port, mode, q):
    """DataParallel / sharding gradient-ready hooks under FLAGS_eager_backward_engine=native: their final
    bucket flush goes through autograd.engine.queue_callback, which runs after the native backward."""
    paddle = _setup(rank, world, port)
    paddle.set_flags({"FLAGS_eager_backward_engine": "native"})
    from paddlepaddle_amd.autograd import engine
    assert engine.use_native()
    cfg, model, crit = _make_model(paddle)
    ids = _data(cfg)
    local = ids[rank * 2:(rank + 1) * 2]
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    if mode == "dp":
        model = paddle.DataParallel(model)
    else:
        from paddlepaddle_amd.distributed.sharding import group_sharded_parallel
        model, opt, _ = group_sharded_parallel(model, opt, level=mode)
    losses = _train(paddle, model, crit, opt, paddle.Tensor(local))
    sd = {k: v.numpy() for k, v in model.state_dict().items()}
    q.put((rank, losses, sd))
    paddle.distributed.barrier()


@pytest.mark.parametrize("mode", ["dp", "os_g", "p_g_os"])
def test_data_parallel_and_sharding_under_native_autograd_engine(mode):
    from paddlepaddle_amd.utils import native
    if native.module() is None or not hasattr(native.module(), "run_backward"):
        pytest.skip("native runtime extension not built")
    ref_losses, ref_sd = _reference()
    (_, l0, sd0), (_, l1, sd1) = _spawn(_native_engine_worker, mode)
    np.testing.assert_allclose((np.array(l0) + np.array(l1)) / 2, ref_losses, rtol=1e-4, atol=1e-5)
    for k in ref_sd:
        np.testing.assert_allclose(sd0[k], ref_sd[k], rtol=2e-3, atol=2e-4, err_msg=f"{mode}:{k}")
        np.testing.assert_allclose(sd1[k], sd0[k], rtol=0, atol=0, err_msg=f"{mode}:{k} replicas differ")


def _stream_worker(rank, world, port, q):
    paddle = _setup(rank, world, port)
    import paddlepaddle_amd.distributed as dist
    from paddlepaddle_amd.distributed.communication import stream as S
    assert dist.stream is S
    out = {}
    x = paddle.to_tensor([1.0 + rank, 2.0])
    task = dist.stream.all_reduce(x, sync_op=False)
    task.wait()
    out["ar_async"] = x.numpy().tolist()
    y = paddle.to_tensor([float(rank)])
    out["ar_calc"] = dist.stream.all_reduce(y, sync_op=True, use_calc_stream=True)  # None on the calc stream
    out["ar_calc_val"] = y.numpy().tolist()
    try:
        dist.stream.all_reduce(y, sync_op=False, use_calc_stream=True)
        out["bad"] = "accepted"
    except RuntimeError:
        out["bad"] = "rejected"
    g = paddle.zeros([2 * 2])
    t2 = dist.stream.all_gather(g, paddle.to_tensor([rank * 10.0, rank * 10.0 + 1]), sync_op=True)
    out["ag_tensor"] = g.numpy().tolist()
    out["ag_task_done"] = t2.is_completed()
    rs = paddle.zeros([2])
    dist.stream.reduce_scatter(rs, paddle.to_tensor([1.0, 2.0, 3.0, 4.0]), sync_op=True)
    out["rs"] = rs.numpy().tolist()
    q.put((rank, out))
    dist.barrier()


def test_stream_collectives_semantics_gloo():
    res = _spawn(_stream_worker)
    for rank, out in res:
        assert out["ar_async"] == [3.0, 4.0]
        assert out["ar_calc"] is None and out["ar_calc_val"] == [1.0]
        assert out["bad"] == "rejected"
        assert out["ag_tensor"] == [0.0, 1.0, 10.0, 11.0] and out["ag_task_done"]
    assert res[0][1]["rs"] == [2.0, 4.0] and res[1][1]["rs"] == [6.0, 8.0]


def _two_opt_worker(rank, world, port, q):
    """One DataParallel model, two optimizers over disjoint halves of it (GAN generator / discriminator):
    clearing one optimizer's grads must not wipe the other's before it steps, and
    clear_grad(set_to_zero=False) leaves .grad None."""
    paddle = _setup(rank, world, port)
    paddle.seed(3)
    net = paddle.nn.Sequential(paddle.nn.Linear(8, 8), paddle.nn.Linear(8, 4))
    dp = paddle.DataParallel(net, comm_buffer_size=1, last_comm_buffer_size=1)
    opt_a = paddle.optimizer.SGD(0.1, parameters=net[0].parameters())
    opt_b = paddle.optimizer.SGD(0.1, parameters=net[1].parameters())
    g = torch.Generator().manual_seed(7)
    x = torch.randn(4, 8, generator=g)
    out = []
    for step in range(2):
        loss = dp(paddle.Tensor(x[rank * 2:(rank + 1) * 2])).square().mean()
        loss.backward()
        opt_a.step()
        opt_a.clear_grad(set_to_zero=(step == 0))
        if step == 1:
            out.append([p.grad is None for p in net[0].parameters()])
        opt_b.step()
        opt_b.clear_grad()
    q.put((rank, {k: v.numpy() for k, v in net.state_dict().items()}, out))
    paddle.distributed.barrier()


def test_data_parallel_two_optimizers_clear_grad_keeps_other_grads():
    sys.path.insert(0, ROOT)
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    paddle.seed(3)
    net = paddle.nn.Sequential(paddle.nn.Linear(8, 8), paddle.nn.Linear(8, 4))
    g = torch.Generator().manual_seed(7)
    x = torch.randn(4, 8, generator=g)
    opt = paddle.optimizer.SGD(0.1, parameters=net.parameters())
    for _ in range(2):
        # mean over the two half-batch losses == the DP average of the per-rank gradients
        loss = (net(paddle.Tensor(x[:2])).square().mean() + net(paddle.Tensor(x[2:])).square().mean()) * 0.5
        loss.backward()
        opt.step()
        opt.clear_grad()
    ref = {k: v.numpy() for k, v in net.state_dict().items()}
    res = _spawn(_two_opt_worker)
    for _, sd, out in res:
        assert out == [[True, True]]
        for k in ref:
            np.testing.assert_allclose(sd[k], ref[k], rtol=1e-5, atol=1e-6, err_msg=k)


def _moe_exchange_worker(rank, world, port, q):
    paddle = _setup(rank, world, port)
    from paddlepaddle_amd.distributed.utils import global_gather, global_scatter
    # 2 experts per card; rank r sends local_count[j * 2 + e] rows to expert e of card j
    local = {0: [1, 2, 0, 1], 1: [2, 0, 1, 1]}
    lc = local[rank]
    # global_count[j * 2 + e] = rows card j sends to my expert e
    gc = [local[j][rank * 2 + e] for j in range(world) for e in range(2)]
    rows = sum(lc)
    x = paddle.to_tensor(np.arange(rows, dtype="float32").reshape(rows, 1) + 100 * rank)
    y = global_scatter(x, paddle.to_tensor(lc, dtype="int64"), paddle.to_tensor(gc, dtype="int64"))
    # expected: expert-major, then source card
    exp = []
    for e in range(2):
        for j in range(world):
            off = sum(local[j][:rank * 2 + e])
            exp += [100 * j + off + k for k in range(local[j][rank * 2 + e])]
    np.testing.assert_array_equal(y.numpy().ravel(), np.array(exp, "float32"))
    z = global_gather(y, paddle.to_tensor(lc, dtype="int64"), paddle.to_tensor(gc, dtype="int64"))
    np.testing.assert_array_equal(z.numpy(), x.numpy())
    q.put((rank, True))


def test_moe_global_scatter_gather_two_ranks():
    _spawn(_moe_exchange_worker)


def test_data_parallel_launch_order_interleaves_dtype_groups():
    """Bucket launch order follows expected gradient readiness (reverse registration of each bucket's earliest
    parameter) across dtype groups, so an fp32 group's buckets are not held behind the bf16 group's last one."""
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.parallel.data_parallel import DataParallel
    layers = []
    for i in range(4):
        lin = paddle.nn.Linear(8, 8)
        lin.weight._t.data = lin.weight._t.data.bfloat16()  # bf16 weights, fp32 biases: two dtype groups
        layers.append(lin)
    model = paddle.nn.Sequential(*layers)
    dp = DataParallel(model)  # world 1: no buckets yet
    dp._world = 2
    dp._build_buckets(1e-6, 1e-6)  # one parameter per bucket
    params = [p for p in model.parameters() if not p.stop_gradient]
    reg = {id(p): i for i, p in enumerate(params)}
    first = [min(reg[id(p)] for p in dp._buckets[bi].params) for bi in dp._order]
    assert first == sorted(first, reverse=True)
    dts = [dp._buckets[bi].params[0]._t.dtype for bi in dp._order]
    assert dts[:2] == [torch.float32, torch.bfloat16]  # the last layer's bias, then its weight: groups interleave
