"""Cross-rank collective-sequence checker (distributed/collective_check.py; reference comm_task_manager.cc:137):
clean DataParallel / sharding runs pass it, a rank that issues a different sequence (an out-of-order bucket,
a different shape) is caught at the end of the step on every rank. gloo, 2 ranks, CPU."""
import os

import pytest
import torch

from test_distributed_cpu import _data, _make_model, _setup, _spawn, _train


def _clean_worker(rank, world, port, mode, q):
    os.environ["PADDLE_AMD_CHECK_COLLECTIVES"] = "1"
    paddle = _setup(rank, world, port)
    from paddlepaddle_amd.distributed import collective_check as cc
    assert cc.enabled()
    cfg, model, crit = _make_model(paddle)
    ids = _data(cfg)[rank * 2:(rank + 1) * 2]
    opt = paddle.optimizer.AdamW(1e-2, parameters=model.parameters())
    if mode == "dp":
        model = paddle.DataParallel(model, comm_buffer_size=0.02, last_comm_buffer_size=0.01)
        assert len(model._buckets) > 2
    else:
        from paddlepaddle_amd.distributed.sharding import group_sharded_parallel
        model, opt, _ = group_sharded_parallel(model, opt, level="p_g_os")
    losses = _train(paddle, model, crit, opt, paddle.Tensor(ids))
    q.put((rank, losses, cc._STATE["checks"]))
    paddle.distributed.barrier()


@pytest.mark.parametrize("mode", ["dp", "stage3"])
def test_checker_passes_clean_runs(mode):
    (_, l0, c0), (_, l1, c1) = _spawn(_clean_worker, mode)
    assert c0 == c1 >= 3 and len(l0) == len(l1) == 3  # a check per step on both ranks, none raised


def _diverge_worker(rank, world, port, how, q):
    paddle = _setup(rank, world, port)
    import torch.distributed as tdist
    from paddlepaddle_amd.distributed import collective_check as cc
    cc.enable_collective_check()
    err = None
    if how == "shape":
        # same byte count (gloo completes it), different shape on rank 1: a different buffer
        t = torch.ones(4) if rank == 0 else torch.ones(2, 2)
        tdist.all_reduce(t)
    else:
        # two equal-sized DP buckets launched in opposite orders on the two ranks
        lin = [paddle.nn.Linear(8, 8, bias_attr=False) for _ in range(2)]
        model = paddle.DataParallel(paddle.nn.Sequential(*lin), comm_buffer_size=1e-6, last_comm_buffer_size=1e-6)
        assert len(model._buckets) == 2
        if rank == 1:
            model._order.reverse()
        try:
            model(paddle.ones([2, 8])).sum().backward()
        except cc.CollectiveMismatchError as e:
            err = str(e)
    if err is None:
        try:
            cc.check_collectives("test")
        except cc.CollectiveMismatchError as e:
            err = str(e)
    q.put((rank, err))


@pytest.mark.parametrize("how", ["shape", "bucket_order"])
def test_checker_fires_on_divergence(how):
    res = _spawn(_diverge_worker, how)
    for _, err in res:
        assert err is not None and "diverged" in err
    if how == "bucket_order":
        assert "dp bucket" in res[0][1]
