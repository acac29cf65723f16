"""Static-graph collective data parallelism (reference: fleet.distributed_optimizer(opt).minimize(loss) in static
mode, meta_optimizers/raw_program_optimizer.py — c_allreduce_sum + 1/nranks scale of every gradient after the
backward): 2 gloo ranks on half batches train like one process on the whole batch."""
import numpy as np
import pytest

from test_distributed_cpu import _setup, _spawn

STEPS = 3


def _data():
    rs = np.random.RandomState(0)
    return rs.randn(8, 16).astype("float32"), rs.randn(8, 4).astype("float32")


def _build(paddle, fleet=None):
    paddle.enable_static()
    main, start = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, start):
        paddle.seed(9)
        x = paddle.static.data("x", [None, 16], "float32")
        y = paddle.static.data("y", [None, 4], "float32")
        h = paddle.nn.functional.relu(paddle.nn.Linear(16, 32)(x))
        out = paddle.nn.Linear(32, 4)(h)
        loss = paddle.mean((out - y) ** 2)
        opt = paddle.optimizer.Momentum(0.1, momentum=0.9)
        if fleet is not None:
            opt = fleet.distributed_optimizer(opt)
        opt.minimize(loss)
    return main, loss


def _worker(rank, world, port, native, q):
    paddle = _setup(rank, world, port)
    overlap = native == "overlap"
    native = native is True
    paddle.set_flags({"FLAGS_static_native_executor": "force" if native else "off"})
    from paddlepaddle_amd.distributed import fleet
    fleet.init(is_collective=True)
    main, loss = _build(paddle, fleet)
    assert main._dp_sync is not None
    if overlap:  # auto_parallel_data_parallel_optimization: 2 KiB buckets -> several all-reduces from backward
        from paddlepaddle_amd.distributed.passes import new_pass
        new_pass("auto_parallel_data_parallel_optimization", {"bucket_size_mb": 2.0 / 1024}).apply(main, None)
    exe = paddle.static.Executor(paddle.CPUPlace())
    xs, ys = _data()
    half = slice(rank * 4, rank * 4 + 4)
    losses = []
    for _ in range(STEPS):
        lv, = exe.run(main, feed={"x": xs[half], "y": ys[half]}, fetch_list=[loss])
        losses.append(float(lv))
    params = [p.numpy().copy() for p in main.all_parameters()]
    runners = [r for r in main.__dict__.get("_native_runners", {}).values() if r is not None]
    assert bool(runners) == native, (native, main.__dict__.get("_native_reason"))
    if overlap:
        from paddlepaddle_amd.static.executor import DP_OVERLAP_STATS
        assert DP_OVERLAP_STATS["launched_in_backward"] >= 2 * STEPS
    paddle.disable_static()
    q.put((rank, losses, params))
    paddle.distributed.barrier()


@pytest.mark.parametrize("native", [False, True, "overlap"])
def test_static_collective_dp_matches_whole_batch(native):
    """Python replay and the native training executor (_C_train: the all-reduce as its gradient hook between the
    backward and the fused update)."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["PADDLE_AMD_FORCE_CPU"] = "1"
    import paddlepaddle_amd as paddle
    main, loss = _build(paddle)
    exe = paddle.static.Executor(paddle.CPUPlace())
    xs, ys = _data()
    ref = [float(exe.run(main, feed={"x": xs, "y": ys}, fetch_list=[loss])[0]) for _ in range(STEPS)]
    ref_params = [p.numpy().copy() for p in main.all_parameters()]
    paddle.disable_static()
    res = sorted(_spawn(_worker, native, world=2))
    (_, l0, p0), (_, l1, p1) = res
    # the mean of the ranks' half-batch losses is the whole-batch loss; parameters stay identical on both ranks
    np.testing.assert_allclose((np.array(l0) + np.array(l1)) / 2, ref, rtol=1e-5, atol=1e-6)
    for a, b, r in zip(p0, p1, ref_params):
        np.testing.assert_allclose(a, b, rtol=0, atol=0)
        np.testing.assert_allclose(a, r, rtol=1e-5, atol=1e-6)
