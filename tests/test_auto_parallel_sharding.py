"""Semi-auto sharding stages (ShardingStage1/2/3 in shard_optimizer) and shard_scaler: 2 gloo ranks, data
parallel over the mesh, must match single-process training. Reference: test/auto_parallel/hybrid_strategy/
semi_auto_parallel_sharding_stage_{1,2,3}.py."""
import os
import sys

import numpy as np
import pytest

from test_distributed_cpu import ROOT, _setup, _spawn


def _net(paddle):
    paddle.seed(0)
    return paddle.nn.Sequential(paddle.nn.Linear(8, 16), paddle.nn.Tanh(), paddle.nn.Linear(16, 4))


def _data():
    rng = np.random.RandomState(3)
    return rng.randn(8, 8).astype("float32"), rng.randn(8, 4).astype("float32")


def _worker(rank, world, port, stage, q):
    paddle = _setup(rank, world, port)
    import paddlepaddle_amd.distributed as dist
    mesh = dist.ProcessMesh([0, 1], dim_names=["dp"])
    net = _net(paddle)
    dist.shard_layer(net, mesh)
    fn = {1: dist.ShardingStage1, 2: dist.ShardingStage2, 3: dist.ShardingStage3}[stage](mesh)
    opt = dist.shard_optimizer(paddle.optimizer.AdamW(0.05, parameters=net.parameters()), fn)
    scaler = dist.shard_scaler(paddle.amp.GradScaler(init_loss_scaling=1024.0))
    X, Y = _data()
    xs = dist.shard_tensor(paddle.to_tensor(X), mesh, [dist.Shard(0)])
    ys = dist.shard_tensor(paddle.to_tensor(Y), mesh, [dist.Shard(0)])
    losses = []
    for _ in range(3):
        loss = ((net(xs) - ys) ** 2).mean()
        scaler.scale(loss).backward()
        scaler.step(opt)
        scaler.update()
        opt.clear_grad()
        losses.append(float(dist.unshard_dtensor(loss).numpy()))
    w0 = net[0].weight
    q.put((rank, losses, str(w0.placements)))
    dist.barrier()


@pytest.mark.parametrize("stage", [1, 2, 3])
def test_sharding_stages_match_single_process(stage):
    sys.path.insert(0, ROOT)
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    net = _net(paddle)
    opt = paddle.optimizer.AdamW(0.05, parameters=net.parameters())
    X, Y = _data()
    ref = []
    for _ in range(3):
        loss = ((net(paddle.to_tensor(X)) - paddle.to_tensor(Y)) ** 2).mean()
        loss.backward()
        opt.step()
        opt.clear_grad()
        ref.append(float(loss))
    res = _spawn(_worker, stage)
    for rank, losses, pl in res:
        np.testing.assert_allclose(losses, ref, rtol=1e-4, atol=1e-5)
        if stage == 3:
            assert "Shard(dim=0)" in pl  # parameters live sharded
