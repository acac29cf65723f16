"""Static auto-parallel engine: a row-parallel linear WITH a bias (the bias joins the partial sum once, on the
mp group's rank 0, then the all-reduce adds the parts) next to a column-parallel one, on 2 ranks, must train
like the single process."""
import numpy as np
import torch

from test_distributed_cpu import _setup, _spawn

STEPS = 3


def _model(paddle):
    class MLP(paddle.nn.Layer):
        def __init__(self):
            super().__init__()
            self.fc1 = paddle.nn.Linear(16, 32)
            self.fc2 = paddle.nn.Linear(32, 8)

        def forward(self, x):
            return self.fc2(paddle.nn.functional.relu(self.fc1(x)))
    return MLP()


def _data():
    g = torch.Generator().manual_seed(3)
    return torch.randn(8, 16, generator=g), torch.randn(8, 8, generator=g)


def _worker(rank, world, port, q):
    paddle = _setup(rank, world, port)
    import paddlepaddle_amd.distributed as dist
    dist.auto_parallel.set_mesh(None)
    paddle.seed(7)
    model = _model(paddle)
    opt = paddle.optimizer.SGD(0.1, parameters=model.parameters())
    mesh = dist.ProcessMesh(np.arange(world).reshape(1, 1, world), dim_names=["pp", "dp", "mp"])
    plan = {"fc1": dist.ColWiseParallel(), "fc2": dist.RowWiseParallel()}
    model, opt = dist.parallelize(model, opt, mesh, dp_config={"sharding_level": 0},
                                  mp_config={"parallelize_plan": plan})
    dm = dist.to_static(model, None, paddle.nn.MSELoss(), opt, dist.Strategy())
    x, y = _data()
    losses = [float(dm(paddle.Tensor(x), paddle.Tensor(y))) for _ in range(STEPS)]
    kinds = sorted({n.name for nodes in dm._engine.stage_nodes for n in nodes})
    q.put((rank, losses, kinds))
    paddle.distributed.barrier()


def _reference():
    import os
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    paddle.distributed.auto_parallel.set_mesh(None)
    paddle.seed(7)
    model = _model(paddle)
    opt = paddle.optimizer.SGD(0.1, parameters=model.parameters())
    x, y = _data()
    out = []
    for _ in range(STEPS):
        loss = paddle.nn.MSELoss()(model(paddle.Tensor(x)), paddle.Tensor(y))
        loss.backward()
        opt.step()
        opt.clear_grad()
        out.append(float(loss))
    return out


def test_row_parallel_linear_with_bias_matches_single_process():
    ref = _reference()
    for rank, losses, kinds in _spawn(_worker, world=2):
        np.testing.assert_allclose(losses, ref, rtol=2e-5, atol=1e-6, err_msg=f"rank {rank}")
        assert "to_partial" in kinds, kinds
