"""Static-graph control flow as sub-block nodes (cond / while_loop / case / switch_case), executed by the
interpreter on device values; collectives recorded as comm nodes. Reference: python/paddle/static/nn/
control_flow.py:755 (while_loop), :1620 (cond); test/legacy_test/test_while_loop_op.py, test_cond.py."""
import json
import os
import sys

import numpy as np
import pytest

import paddlepaddle_amd as paddle
from paddlepaddle_amd.static.program import CFNode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def static():
    paddle.enable_static()
    yield
    paddle.disable_static()


def test_cond_runs_only_the_taken_branch(static):
    main, start = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, start):
        x = paddle.static.data("x", [4], "float32")
        flag = paddle.static.data("flag", [1], "bool")
        out = paddle.static.nn.cond(flag, lambda: x * 2.0 + 1.0, lambda: x.exp() - 3.0)
    assert any(isinstance(n, CFNode) for n in main.nodes) and main.num_blocks == 3
    exe = paddle.static.Executor()
    xv = np.arange(4, dtype="float32")
    t, = exe.run(main, feed={"x": xv, "flag": np.array([True])}, fetch_list=[out])
    f, = exe.run(main, feed={"x": xv, "flag": np.array([False])}, fetch_list=[out])
    np.testing.assert_allclose(t, xv * 2 + 1)
    np.testing.assert_allclose(f, np.exp(xv) - 3, rtol=1e-6)


def test_while_loop_data_dependent_trip_count(static):
    main, start = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, start):
        limit = paddle.static.data("limit", [1], "int64")
        i = paddle.full([1], 0, "int64")
        acc = paddle.full([1], 0.0, "float32")
        i_out, acc_out = paddle.static.nn.while_loop(lambda i, a: i < limit,
                                                     lambda i, a: [i + 1, a + i.astype("float32") * 0.5],
                                                     [i, acc])
    exe = paddle.static.Executor()
    for n in (0, 3, 7):
        iv, av = exe.run(main, feed={"limit": np.array([n], "int64")}, fetch_list=[i_out, acc_out])
        assert int(iv[0]) == n
        np.testing.assert_allclose(av[0], 0.5 * sum(range(n)))


def test_nested_cond_in_while_and_gradient(static):
    main, start = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, start):
        x = paddle.static.data("x", [3], "float32")
        x.stop_gradient = False
        k = paddle.full([1], 0, "int64")

        def body(k, y):
            y2 = paddle.static.nn.cond(k % 2 == 0, lambda: y * 2.0, lambda: y + 1.0)
            return [k + 1, y2]
        _, y = paddle.static.nn.while_loop(lambda k, y: k < 3, body, [k, x])
        loss = y.sum()
        g, = paddle.static.gradients([loss], [x])
    exe = paddle.static.Executor()
    xv = np.array([1.0, 2.0, 3.0], "float32")
    yv, gv = exe.run(main, feed={"x": xv}, fetch_list=[y, g])
    np.testing.assert_allclose(yv, (xv * 2 + 1) * 2)  # k = 0: *2, k = 1: +1, k = 2: *2
    np.testing.assert_allclose(gv, np.full(3, 4.0))


def test_switch_case_and_case(static):
    main, start = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, start):
        idx = paddle.static.data("idx", [1], "int32")
        x = paddle.static.data("x", [2], "float32")
        out = paddle.static.nn.switch_case(idx, {0: lambda: x + 10.0, 1: lambda: x * 0.0, 2: lambda: -x})
        c = paddle.static.nn.case([(x.sum() > 100.0, lambda: x * 0.0)], default=lambda: x + 1.0)
    exe = paddle.static.Executor()
    xv = np.array([1.0, -2.0], "float32")
    for i, ref in [(0, xv + 10), (1, xv * 0), (2, -xv), (7, -xv)]:
        o, cv = exe.run(main, feed={"idx": np.array([i], "int32"), "x": xv}, fetch_list=[out, c])
        np.testing.assert_allclose(o, ref)
        np.testing.assert_allclose(cv, xv + 1)


def test_control_flow_program_serializes(static, tmp_path):
    main, start = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, start):
        x = paddle.static.data("x", [2, 3], "float32")
        lin = paddle.nn.Linear(3, 3)
        h = lin(x)
        out = paddle.static.nn.cond(h.mean() > 0, lambda: paddle.nn.functional.relu(h), lambda: h * -1.0)
    exe = paddle.static.Executor()
    xv = np.random.RandomState(0).randn(2, 3).astype("float32")
    ref, = exe.run(main, feed={"x": xv}, fetch_list=[out])
    prefix = str(tmp_path / "m")
    paddle.static.save_inference_model(prefix, [x], [out], exe, program=main)
    prog, feeds, fetches = paddle.static.load_inference_model(prefix, exe)
    got, = exe.run(prog, feed={feeds[0]: xv}, fetch_list=fetches)
    np.testing.assert_allclose(got, ref, rtol=1e-6)


def _comm_worker(rank, world, port, q):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_distributed_cpu import _setup
    paddle = _setup(rank, world, port)
    paddle.enable_static()
    main, start = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, start):
        x = paddle.static.data("x", [4], "float32")
        y = x * 2.0
        paddle.distributed.all_reduce(y)
        z = x + 1.0  # independent of the collective: may overlap it
        out = y + z
    exe = paddle.static.Executor()
    o, = exe.run(main, feed={"x": np.full(4, rank + 1.0, "float32")}, fetch_list=[out])
    kinds = [n.kind for n in main.nodes]
    paddle.disable_static()
    q.put((rank, o.tolist(), kinds))
    paddle.distributed.barrier()


def test_static_program_collective_node_gloo():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_distributed_cpu import _spawn
    res = _spawn(_comm_worker)
    for rank, o, kinds in res:
        assert "comm" in kinds
        # all_reduce(2 * x) = 2 * (1 + 2) = 6, plus x + 1
        np.testing.assert_allclose(o, [6.0 + rank + 2.0] * 4)
