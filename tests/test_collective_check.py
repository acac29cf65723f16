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


def _trace_worker(rank, world, port, d, how, q):
    _setup(rank, world, port)
    import torch.distributed as tdist
    from paddlepaddle_amd.distributed import collective_check as cc
    cc.enable_collective_check(trace_dir=d)
    a = torch.ones(4)
    if how == "order":  # two equal-shaped buckets in opposite orders (gloo completes it; RCCL would mix them)
        names = ["bucket 0", "bucket 1"] if rank == 0 else ["bucket 1", "bucket 0"]
        for nm in names:
            with cc.label(nm):
                tdist.all_reduce(a)
    else:
        tdist.all_reduce(a)
    cc.disable_collective_check()
    q.put((rank, None))


@pytest.mark.parametrize("how", ["stop", "order"])
def test_flight_recorder_names_where_ranks_part(tmp_path, how):
    """PADDLE_AMD_COLLECTIVE_TRACE_DIR flight recorder: each rank appends every collective as it is issued; the
    offline diff (tools/collective_trace_diff.py) names the rank that stopped short of its peers (what a hang
    leaves, no end-of-step check needed) or the first entry where two ranks' sequences differ."""
    from paddlepaddle_amd.distributed.collective_check import first_divergence
    if how == "stop":  # rank 1 never issues the broadcast: gloo would hang, so rank 0 skips waiting for it
        _spawn(_trace_worker, str(tmp_path), "stop_local")
        # fabricate the hang's picture: rank 0 issued one more collective than rank 1
        with open(tmp_path / "collectives.rank0.log", "a") as f:
            f.write("coll:0-1 #2 broadcast (8,):float32\n")
    else:
        _spawn(_trace_worker, str(tmp_path), how)
    files = sorted(str(p) for p in tmp_path.glob("collectives.rank*.log"))
    assert len(files) == 2
    found = first_divergence(files)
    assert len(found) == 1, found
    if how == "stop":
        assert "ranks [1] stopped after 1 of 2 entries" in found[0], found
    else:
        assert "entry #1" in found[0] and "[bucket 0]" in found[0] and "[bucket 1]" in found[0], found
