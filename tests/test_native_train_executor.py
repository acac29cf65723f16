"""Native training executor (csrc/interpreter/train_interp.cpp via static/native_train.py): a static training
program's forward, backward and optimizer update run as one C++ call. Reference behaviour:
paddle/fluid/framework/new_executor/pir_interpreter.cc (instructions + dependency / GC plan).

CPU: with FLAGS_static_native_executor=force every op is an ATen dispatcher instruction (the backward is the C++
autograd engine) and the losses equal the Python replay's exactly. GPU: the hot ops run the hand-written kernels
(MFMA GEMM, LayerNorm, flash attention fwd/bwd, softmax-CE, implicit-GEMM conv, NHWC batch norm) and the fused
optimizer kernels; losses track the Python replay and the kernel counters prove the native path ran."""
import numpy as np
import pytest

import paddlepaddle_amd as paddle
from paddlepaddle_amd.static import native_train as NT


def _runners(main):
    return [r for r in main.__dict__.get("_native_runners", {}).values() if r is not None]


def _run(build, feeds_fn, mode, steps=3):
    paddle.set_flags({"FLAGS_static_native_executor": mode})
    paddle.enable_static()
    try:
        main, start = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, start):
            paddle.seed(3)
            loss = build()
        exe = paddle.static.Executor()
        rng = np.random.RandomState(0)
        out = [float(exe.run(main, feed=feeds_fn(rng), fetch_list=[loss])[0]) for _ in range(steps)]
        return out, main
    finally:
        paddle.disable_static()
        paddle.set_flags({"FLAGS_static_native_executor": "auto"})


def _mlp():
    x = paddle.static.data("x", [32, 16], "float32")
    t = paddle.static.data("t", [32, 1], "float32")
    h = paddle.nn.functional.gelu(paddle.nn.Linear(16, 64)(x))
    loss = ((paddle.nn.Linear(64, 1)(h) - t) ** 2).mean()
    paddle.optimizer.AdamW(learning_rate=0.01, weight_decay=0.01).minimize(loss)
    return loss


def _mlp_feeds(rng):
    xs = rng.rand(32, 16).astype("float32")
    return {"x": xs, "t": xs.sum(1, keepdims=True).astype("float32") * 0.1}


def _gpt(dtype="float32"):
    def build():
        from paddlepaddle_amd.models.gpt import GPTConfig, GPTForPretraining
        cfg = GPTConfig.tiny(attention_probs_dropout_prob=0.0)
        if dtype != "float32":
            paddle.set_default_dtype(dtype)
        m = GPTForPretraining(cfg)
        paddle.set_default_dtype("float32")
        ids = paddle.static.data("ids", [2, 64], "int64")
        lab = paddle.static.data("lab", [2, 64], "int64")
        loss = m(ids, labels=lab)
        paddle.optimizer.AdamW(1e-3, parameters=m.parameters(), multi_precision=dtype != "float32",
                               grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0)).minimize(loss)
        return loss
    return build


def _gpt_feeds(rng):
    d = rng.randint(0, 512, (2, 65))
    return {"ids": d[:, :-1], "lab": d[:, 1:]}


def _resnet():
    from paddlepaddle_amd.vision.models import resnet18
    m = resnet18(num_classes=10, data_format="NHWC")
    x = paddle.static.data("x", [2, 32, 32, 3], "float32")
    lab = paddle.static.data("lab", [2], "int64")
    loss = paddle.nn.functional.cross_entropy(m(x), lab)
    paddle.optimizer.Momentum(0.01, parameters=m.parameters(), weight_decay=1e-4).minimize(loss)
    return loss


def _resnet_feeds(rng):
    return {"x": rng.rand(2, 32, 32, 3).astype("float32"), "lab": rng.randint(0, 10, (2,))}


@pytest.mark.parametrize("case", ["mlp", "gpt", "resnet"])
def test_native_executor_matches_python_replay_cpu(case):
    build, feeds = {"mlp": (_mlp, _mlp_feeds), "gpt": (_gpt(), _gpt_feeds), "resnet": (_resnet, _resnet_feeds)}[case]
    ref, _ = _run(build, feeds, "off")
    got, main = _run(build, feeds, "force")
    assert getattr(main, "_native_reason", "unset") is None, main._native_reason
    rs = _runners(main)
    assert len(rs) == 1 and rs[0].num_instructions > 10
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)


def test_native_executor_falls_back_with_reason():
    """A gradient-merge program keeps the Python replay and records why."""
    from paddlepaddle_amd.static import program as P
    paddle.set_flags({"FLAGS_static_native_executor": "force"})
    paddle.enable_static()
    try:
        main, start = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, start):
            loss = _mlp()
        main._grad_merge = (2, True)
        main._gm_count = 0
        exe = paddle.static.Executor()
        exe.run(main, feed=_mlp_feeds(np.random.RandomState(0)), fetch_list=[loss])
        assert "gradient merge" in main._native_reason
        assert not _runners(main)
        del P
    finally:
        paddle.disable_static()
        paddle.set_flags({"FLAGS_static_native_executor": "auto"})


@pytest.mark.gpu
def test_native_executor_gpt_bf16_kernels():
    paddle.set_device("gpu:0")
    NT.reset_kernel_calls()
    got, main = _run(_gpt("bfloat16"), _gpt_feeds, "auto", steps=4)
    assert main._native_reason is None, main._native_reason
    calls = NT.kernel_calls()
    for k in ("gemm", "layer_norm", "flash_attn", "flash_attn_bwd", "softmax_ce", "adamw"):
        assert calls.get(k, 0) > 0, (k, calls)
    r = _runners(main)[0]
    assert r.num_native > 10 and r.scalars_fn is not None  # the optimizer update ran natively
    ref, _ = _run(_gpt("bfloat16"), _gpt_feeds, "off", steps=4)
    np.testing.assert_allclose(got, ref, rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
def test_native_executor_conv_bn_block_bf16():
    """NHWC conv (implicit GEMM fwd / flipped-filter dgrad / split-K wgrad) + fused BN(+ReLU) + Momentum."""
    paddle.set_device("gpu:0")

    def build():
        paddle.set_default_dtype("bfloat16")
        c1 = paddle.nn.Conv2D(64, 64, 3, padding=1, data_format="NHWC", bias_attr=False)
        c2 = paddle.nn.Conv2D(64, 64, 3, padding=1, data_format="NHWC", bias_attr=False)
        head = paddle.nn.Linear(64, 10)
        paddle.set_default_dtype("float32")
        b1 = paddle.nn.BatchNorm2D(64, data_format="NHWC")
        b2 = paddle.nn.BatchNorm2D(64, data_format="NHWC")
        x = paddle.static.data("x", [8, 16, 16, 64], "bfloat16")
        lab = paddle.static.data("lab", [8], "int64")
        h = paddle.nn.functional.relu(b1(c1(x)))
        h = paddle.nn.functional.relu(b2(c2(h)) + x)
        logits = head(h.mean(axis=[1, 2]))
        loss = paddle.nn.functional.cross_entropy(logits.astype("float32"), lab)
        params = [p for l in (c1, c2, head, b1, b2) for p in l.parameters()]
        paddle.optimizer.Momentum(0.01, parameters=params, multi_precision=True).minimize(loss)
        return loss

    def feeds(rng):
        return {"x": rng.rand(8, 16, 16, 64).astype("float32"), "lab": rng.randint(0, 10, (8,))}
    NT.reset_kernel_calls()
    got, main = _run(build, feeds, "auto", steps=3)
    assert main._native_reason is None, main._native_reason
    calls = NT.kernel_calls()
    for k in ("conv2d", "conv2d_wgrad", "batch_norm", "batch_norm_bwd", "momentum"):
        assert calls.get(k, 0) > 0, (k, calls)
    ref, _ = _run(build, feeds, "off", steps=3)
    np.testing.assert_allclose(got, ref, rtol=3e-2, atol=3e-2)


@pytest.mark.gpu
def test_native_executor_dp_gradient_hook_gpu(monkeypatch):
    """Static collective DP on the native update: the executor's gradient hook (the data-parallel all-reduce) runs
    once per step between the C++ backward and the fused AdamW kernel, on the gradients of every parameter."""
    from paddlepaddle_amd.static import executor as EX
    seen = []

    def fake(grads, pg):
        seen.append((len(grads), pg))
    monkeypatch.setattr(EX, "_allreduce_mean", fake)
    paddle.set_device("gpu:0")
    paddle.set_flags({"FLAGS_static_native_executor": "auto"})
    paddle.enable_static()
    try:
        main, start = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, start):
            paddle.seed(3)
            loss = _mlp()
        main._dp_sync = "dp-group"
        exe = paddle.static.Executor()
        rng = np.random.RandomState(0)
        for _ in range(3):
            exe.run(main, feed=_mlp_feeds(rng), fetch_list=[loss])
        r = _runners(main)
        assert r and r[0].scalars_fn is not None, main._native_reason  # the update ran natively
        assert seen == [(4, "dp-group")] * 3, seen
    finally:
        paddle.disable_static()


def test_native_executor_replay_only_before_side_effects():
    """A failed native step may be replayed by the Python executor only when it stopped in the forward before any
    instruction writing persistent state (BN statistics, in-place ops) had run."""
    assert NT._mutates(("native", "batch_norm_act", [], [], [], []))
    assert not NT._mutates(("native", "linear", [], [], [], []))
    assert NT._mutates(("aten", "add_", "Tensor", [], [0]))
    assert not NT._mutates(("aten", "add", "Tensor", [], [0]))

    class TP:
        def __init__(self, phase, done):
            self.phase, self.done = phase, done

    class Low:
        instrs = [("aten", "mm", "default", [], [0]), ("native", "batch_norm_act", [], [], [], []),
                  ("aten", "relu", "default", [], [0])]

    r = NT.NativeTrainRunner.__new__(NT.NativeTrainRunner)
    r._lowering = Low()
    for phase, done, ok in [(0, 0, True), (0, 1, False), (0, 2, False), (1, 3, False), (3, 3, False)]:
        r.tp = TP(phase, done)
        assert r.replayable() is ok, (phase, done)


def _comm_build(fn=None):
    def build():
        from paddlepaddle_amd.distributed.collective import _static_comm
        x = paddle.static.data("x", [32, 16], "float32")
        t = paddle.static.data("t", [32, 1], "float32")
        h = paddle.nn.Linear(16, 64)(x)
        if fn is None:
            paddle.distributed.all_reduce(h)  # a c:all_reduce node of the program
        else:
            assert _static_comm(h, "scale", fn)
        side = paddle.nn.Linear(16, 64)(x)  # independent of the collective: overlaps it on the compute stream
        loss = ((paddle.nn.Linear(64, 1)(paddle.nn.functional.relu(h) + side) - t) ** 2).mean()
        paddle.optimizer.AdamW(learning_rate=0.01).minimize(loss)
        return loss
    return build


def _comm_worker(rank, world, port, q):
    from test_distributed_cpu import _setup
    _setup(rank, world, port)
    out = {}
    for mode in ("off", "force"):
        losses, main = _run(_comm_build(), _mlp_feeds, mode)
        rs = _runners(main)
        out[mode] = (losses, [r.num_comm for r in rs])
    q.put((rank, out))


def test_native_executor_collective_instructions_gloo():
    """A program with an all_reduce node lowers onto the native executor as a communication instruction (2 gloo
    ranks): same losses as the Python replay on both ranks."""
    from test_distributed_cpu import _spawn
    for rank, out in _spawn(_comm_worker, world=2):
        ref, _ = out["off"]
        got, ncomm = out["force"]
        assert ncomm == [1], ncomm
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_native_executor_comm_stream_gpu():
    """GPU: the communication instruction runs on the executor's own stream (not the compute stream), and the
    instruction reading what it wrote waits for it through an event: same losses as the Python replay (which
    runs collectives on its own comm stream too)."""
    import torch
    seen = []

    def scale(x):  # an in-place "collective" on the current (communication) stream
        seen.append(torch.cuda.current_stream().cuda_stream)
        x.mul_(0.5)

    NT.reset_kernel_calls()
    ref, _ = _run(_comm_build(scale), _mlp_feeds, "off")
    seen.clear()
    got, main = _run(_comm_build(scale), _mlp_feeds, "on")
    rs = _runners(main)
    assert len(rs) == 1 and rs[0].num_comm == 1, main.__dict__.get("_native_reason")
    assert NT.kernel_calls().get("comm", 0) == 3
    assert seen and all(s != torch.cuda.default_stream().cuda_stream for s in seen), seen
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)
