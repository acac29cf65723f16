"""Static Executor with BuildStrategy.allow_cuda_graph_capture (reference base/executor.py:993): after two eager
warm-up runs the whole run — program replay, backward, optimizer update — is captured into one hipGraph and
replayed; training must follow the eager run step for step."""
import numpy as np
import pytest

import paddlepaddle_amd as paddle


def _train(use_graph, steps=8):
    paddle.enable_static()
    try:
        main, start = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, start):
            paddle.seed(3)
            x = paddle.static.data("x", [32, 16], "float32")
            t = paddle.static.data("t", [32, 1], "float32")
            h = paddle.nn.functional.gelu(paddle.nn.Linear(16, 64)(x))
            y = paddle.nn.Linear(64, 1)(h)
            loss = ((y - t) ** 2).mean()
            paddle.optimizer.AdamW(learning_rate=0.01, weight_decay=0.01).minimize(loss)
        exe = paddle.static.Executor(paddle.CUDAPlace(0))
        prog = main
        if use_graph:
            bs = paddle.static.BuildStrategy()
            bs.allow_cuda_graph_capture = True
            prog = paddle.static.CompiledProgram(main, build_strategy=bs)
        rng = np.random.RandomState(0)
        losses = []
        for _ in range(steps):
            xs = rng.rand(32, 16).astype("float32")
            ts = xs.sum(1, keepdims=True).astype("float32") * 0.1
            losses.append(float(exe.run(prog, feed={"x": xs, "t": ts}, fetch_list=[loss])[0]))
        return losses
    finally:
        paddle.disable_static()


@pytest.mark.gpu
def test_captured_static_training_matches_eager():
    from paddlepaddle_amd.static import executor as E
    paddle.set_device("gpu:0")
    eager = _train(False)
    before = dict(E._GRAPH_STATS)
    graph = _train(True)
    assert E._GRAPH_STATS["captured"] == before["captured"] + 1
    assert E._GRAPH_STATS["replayed"] >= before["replayed"] + 6
    np.testing.assert_allclose(graph, eager, rtol=2e-4, atol=1e-6)
    assert graph[-1] < graph[0]


def test_cpu_program_with_capture_flag_runs_eagerly():
    """CPU place: the flag is accepted and the program runs eagerly (no hipGraph on the host)."""
    paddle.set_device("cpu")
    paddle.enable_static()
    try:
        main, start = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, start):
            x = paddle.static.data("x", [4, 2], "float32")
            y = paddle.nn.Linear(2, 1)(x)
        bs = paddle.static.BuildStrategy()
        bs.allow_cuda_graph_capture = True
        exe = paddle.static.Executor(paddle.CPUPlace())
        out = exe.run(paddle.static.CompiledProgram(main, build_strategy=bs), feed={"x": np.ones((4, 2), "float32")},
                      fetch_list=[y])
        assert out[0].shape == (4, 1)
    finally:
        paddle.disable_static()


def test_static_print_is_an_op_of_the_program(capsys):
    """paddle.static.Print prints when the program runs (every run, first_n bounded), not at build time."""
    import numpy as np
    paddle.set_device("cpu")
    paddle.enable_static()
    try:
        main, start = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, start):
            x = paddle.static.data("x", [2, 2], "float32")
            y = paddle.static.Print(x * 3, message="tripled", first_n=2)
            z = y + 1
        assert capsys.readouterr().out == ""          # nothing printed while building
        exe = paddle.static.Executor(paddle.CPUPlace())
        for _ in range(3):
            out = exe.run(main, feed={"x": np.ones((2, 2), "float32")}, fetch_list=[z])[0]
        np.testing.assert_array_equal(out, np.full((2, 2), 4.0, "float32"))
        printed = capsys.readouterr().out
        assert printed.count("tripled") == 2 and "[3.0, 3.0, 3.0, 3.0]" in printed
    finally:
        paddle.disable_static()


def _train_opt(make_opt, use_graph, steps=6, on_step=None):
    paddle.enable_static()
    try:
        main, start = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, start):
            paddle.seed(5)
            x = paddle.static.data("x", [16, 8], "float32")
            y = paddle.nn.Linear(8, 1)(x)
            loss = (y ** 2).mean()
            opt = make_opt()
            opt.minimize(loss)
        exe = paddle.static.Executor(paddle.CUDAPlace(0))
        prog = main
        if use_graph:
            bs = paddle.static.BuildStrategy()
            bs.allow_cuda_graph_capture = True
            prog = paddle.static.CompiledProgram(main, build_strategy=bs)
        rng = np.random.RandomState(1)
        losses = []
        for i in range(steps):
            if on_step is not None:
                on_step(i, opt)
            xs = rng.rand(16, 8).astype("float32")
            losses.append(float(exe.run(prog, feed={"x": xs}, fetch_list=[loss])[0]))
        return losses, opt
    finally:
        paddle.disable_static()


@pytest.mark.gpu
def test_replayed_adam_keeps_host_step_counters():
    """the host step counters advance with every replay, so state_dict() after replays holds the
    beta powers of the true step and a later eager step applies the right bias correction."""
    paddle.set_device("gpu:0")
    mk = lambda: paddle.optimizer.Adam(learning_rate=0.01)  # noqa: E731
    eager, oe = _train_opt(mk, False, steps=7)
    graph, og = _train_opt(mk, True, steps=7)
    np.testing.assert_allclose(graph, eager, rtol=2e-4, atol=1e-6)
    for sd in (oe.state_dict(), og.state_dict()):  # parameter names differ between the two programs
        pows = [v for k, v in sd.items() if k.endswith("beta1_pow_acc_0")]
        assert pows and sd["@step"] == 7
        for v in pows:
            np.testing.assert_allclose(v.numpy(), 0.9 ** 7, rtol=1e-6)


@pytest.mark.gpu
def test_momentum_lr_change_recaptures_and_scheduler_stays_eager():
    from paddlepaddle_amd.static import executor as E
    paddle.set_device("gpu:0")

    def bump(i, opt):
        if i == 4:
            opt.set_lr(0.05)
    mk = lambda: paddle.optimizer.Momentum(learning_rate=0.1, momentum=0.9)  # noqa: E731
    eager, _ = _train_opt(mk, False, steps=8, on_step=bump)
    before = dict(E._GRAPH_STATS)
    graph, _ = _train_opt(mk, True, steps=8, on_step=bump)
    np.testing.assert_allclose(graph, eager, rtol=2e-4, atol=1e-6)
    assert E._GRAPH_STATS["captured"] == before["captured"] + 2  # re-captured after set_lr
    # an LR scheduler feeds Momentum a host float every step: never captured, still matches eager
    mk2 = lambda: paddle.optimizer.Momentum(learning_rate=paddle.optimizer.lr.StepDecay(0.1, 2), momentum=0.9)  # noqa
    sched = lambda i, opt: opt._learning_rate.step() if i else None  # noqa: E731
    eager2, _ = _train_opt(mk2, False, steps=6, on_step=sched)
    before = dict(E._GRAPH_STATS)
    graph2, _ = _train_opt(mk2, True, steps=6, on_step=sched)
    np.testing.assert_allclose(graph2, eager2, rtol=2e-4, atol=1e-6)
    assert E._GRAPH_STATS["captured"] == before["captured"]
