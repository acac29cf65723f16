"""Static graph (Program/Executor), jit (to_static/save/load) and inference predictor.
Reference test strategy: test/legacy_test/test_executor_*.py, test/dygraph_to_static/*, test/inference:
the static / translated program must reproduce dygraph numerics."""
import json
import os

import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle
import paddlepaddle_amd.nn.functional as F
from paddlepaddle_amd.static import InputSpec


@pytest.fixture
def static_mode():
    paddle.enable_static()
    yield
    paddle.disable_static()


def _mlp_prog():
    main, startup = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, startup):
        x = paddle.static.data("x", [None, 16], "float32")
        y = paddle.static.data("y", [None, 1], "int64")
        h = paddle.static.nn.fc(x, 32, activation="relu")
        out = paddle.static.nn.fc(h, 4)
        loss = paddle.mean(F.cross_entropy(out, y))
    return main, startup, x, y, out, loss


def test_static_train_and_inference_roundtrip(static_mode, tmp_path):
    paddle.seed(1)
    main, startup, x, y, out, loss = _mlp_prog()
    with paddle.static.program_guard(main, startup):
        paddle.optimizer.Adam(0.01).minimize(loss)
    # op list: HIP ops recorded whole (fused_linear / softmax_cross_entropy), no decompositions
    names = [n.name for n in main.global_block().ops]
    assert sum("fused_linear" in n for n in names) == 2 and any("softmax_cross_entropy" in n for n in names)
    exe = paddle.static.Executor(paddle.CPUPlace())
    exe.run(startup)
    rng = np.random.RandomState(0)
    xs = rng.randn(64, 16).astype("float32")
    ys = xs[:, :4].argmax(1).reshape(-1, 1).astype("int64")
    losses = [float(exe.run(main, feed={"x": xs, "y": ys}, fetch_list=[loss])[0]) for _ in range(40)]
    assert losses[-1] < 0.3 * losses[0]
    test = main.clone(for_test=True)
    o1, = exe.run(test, feed={"x": xs[:8]}, fetch_list=[out])
    o1b, = exe.run(test, feed={"x": xs[:8]}, fetch_list=[out])
    np.testing.assert_array_equal(o1, o1b)  # for_test program does not train
    prefix = str(tmp_path / "mlp")
    paddle.static.save_inference_model(prefix, [x], [out], exe, program=main)
    prog, feeds, fetches = paddle.static.load_inference_model(prefix, exe)
    o2, = exe.run(prog, feed={feeds[0]: xs[:8]}, fetch_list=fetches)
    np.testing.assert_allclose(o2, o1, rtol=1e-6, atol=1e-6)
    # static.save / load restore parameters
    paddle.static.save(main, str(tmp_path / "ckpt"))
    w = main.all_parameters()[0]
    before = w.numpy().copy()
    exe.run(main, feed={"x": xs, "y": ys}, fetch_list=[loss])
    assert not np.allclose(w.numpy(), before)
    paddle.static.load(main, str(tmp_path / "ckpt"))
    np.testing.assert_array_equal(w.numpy(), before)


def test_static_matches_dygraph(static_mode):
    paddle.seed(5)
    main, startup = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, startup):
        x = paddle.static.data("x", [4, 8], "float32")
        lin = paddle.nn.Linear(8, 8)
        ln = paddle.nn.LayerNorm(8)
        out = paddle.tanh(ln(lin(x))).sum(axis=-1)
    xs = np.random.RandomState(1).randn(4, 8).astype("float32")
    got, = paddle.static.Executor().run(main, feed={"x": xs}, fetch_list=[out])
    paddle.disable_static()
    ref = paddle.tanh(ln(lin(paddle.to_tensor(xs)))).sum(axis=-1).numpy()
    paddle.enable_static()
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)


def test_static_gradients_and_append_backward(static_mode):
    main = paddle.static.Program()
    with paddle.static.program_guard(main):
        x = paddle.static.data("x", [3, 4], "float32")
        lin = paddle.nn.Linear(4, 2)
        y = (x * x).sum()
        gx, = paddle.static.gradients([y], [x])
        loss = lin(x).sum()
        pg = paddle.static.append_backward(loss)
    xs = np.arange(12, dtype="float32").reshape(3, 4)
    exe = paddle.static.Executor()
    g, gw = exe.run(main, feed={"x": xs}, fetch_list=[gx, pg[0][1]])
    np.testing.assert_allclose(g, 2 * xs)
    # d(sum(x W + b))/dW = x^T 1
    np.testing.assert_allclose(gw, xs.sum(0)[:, None].repeat(2, 1), rtol=1e-6)


def test_program_file_refuses_foreign_callables(tmp_path):
    from paddlepaddle_amd.static.program import Program
    d = {"format": "paddlepaddle_amd.program", "version": 1, "n_slots": 1, "slot_meta": [[[1], "float32"]],
         "feeds": [], "fetch": [0], "nodes": [{"f": "f:os:system", "a": ["echo hi"], "k": {}, "o": {"r": 0}}]}
    with pytest.raises(ValueError):
        Program.from_dict(json.loads(json.dumps(d)), {})
    d["nodes"][0]["f"] = "o:subprocess:run"
    with pytest.raises(ValueError):
        Program.from_dict(d, {})


class _Net(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.l1 = paddle.nn.Linear(8, 16)
        self.l2 = paddle.nn.Linear(16, 4)
        self.ln = paddle.nn.LayerNorm(16)

    def forward(self, x):
        h = F.gelu(self.ln(self.l1(x)))
        b = x.shape[0]
        h = h.reshape([b, 4, 4]).transpose([0, 2, 1]).reshape([b, 16])
        return self.l2(h)


def test_to_static_forward_backward_and_jit_save_load_dynamic_batch(tmp_path):
    paddle.seed(3)
    net = _Net()
    x = paddle.randn([5, 8])
    ref = net(x)
    snet = paddle.jit.to_static(net)
    np.testing.assert_array_equal(snet(x).numpy(), ref.numpy())
    assert len(net.forward.program_cache) == 1
    # gradients flow through the replay into the real parameters
    loss = (snet(x) ** 2).mean()
    loss.backward()
    g_static = net.l1.weight.grad.numpy().copy()
    net.clear_gradients()
    loss = (_Net.forward(net, x) ** 2).mean()
    loss.backward()
    np.testing.assert_allclose(g_static, net.l1.weight.grad.numpy(), rtol=1e-5, atol=1e-7)
    path = str(tmp_path / "net")
    paddle.jit.save(net, path, input_spec=[InputSpec([None, 8], "float32", "x")])
    tl = paddle.jit.load(path)
    net.eval()
    for n in (5, 7, 1):
        xi = paddle.randn([n, 8])
        np.testing.assert_allclose(tl(xi).numpy(), _Net.forward(net, xi).numpy(), rtol=1e-6, atol=1e-6)
    assert len(tl.parameters()) == 6
    # predictor over the same files (handle API and list API)
    cfg = paddle.inference.Config(path + ".pdmodel", path + ".pdiparams")
    cfg.disable_gpu()
    pred = paddle.inference.create_predictor(cfg)
    xi = np.random.RandomState(0).randn(3, 8).astype("float32")
    h = pred.get_input_handle(pred.get_input_names()[0])
    h.reshape(xi.shape)
    h.copy_from_cpu(xi)
    pred.run()
    out = pred.get_output_handle(pred.get_output_names()[0]).copy_to_cpu()
    np.testing.assert_allclose(out, _Net.forward(net, paddle.to_tensor(xi)).numpy(), rtol=1e-6, atol=1e-6)
    out2 = pred.run([xi])[0].numpy()
    np.testing.assert_array_equal(out, out2)


def test_to_static_value_dependent_control_flow_is_guarded():
    """float(x.sum()) is a graph break: the function is traced with a guard on that value instead of
    falling back to eager (tests/test_jit_guards.py covers the variants)."""
    @paddle.jit.to_static
    def f(x):
        if float(x.sum()) > 0:
            return x * 2
        return x * 3
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # no eager-fallback warning
        y = f(paddle.ones([3]))
        z = f(-paddle.ones([3]))
    np.testing.assert_array_equal(y.numpy(), [2, 2, 2])
    np.testing.assert_array_equal(z.numpy(), [-3, -3, -3])
    assert all(cp.guarded for cp in f.variants(paddle.ones([3])))


def test_native_scheduler_frees_intermediates():
    from paddlepaddle_amd.static import program as P
    from paddlepaddle_amd.jit import trace_program
    prog, feeds, tmpl, fetch = trace_program(lambda a: ((a + 1) * 2 - 3).exp(), (InputSpec([4], "float32"),), {})
    plan = P.build_plan(prog, fetch)
    freed = sorted(s for v in plan.free_after.values() for s in v)
    assert len(plan.order) == 4 and len(freed) == 3  # every intermediate is released after its last use


@pytest.mark.gpu
def test_to_static_gpt_replays_hip_ops_and_predictor_hipgraph(tmp_path):
    from paddlepaddle_amd.models.gpt import GPTConfig, GPTForPretraining
    paddle.set_device("gpu")
    paddle.seed(0)
    paddle.set_default_dtype("bfloat16")
    try:
        cfg = GPTConfig.tiny(num_hidden_layers=2)
        model = GPTForPretraining(cfg)
        model.eval()
        ids = paddle.randint(0, cfg.vocab_size, [2, 64])
        with paddle.no_grad():
            ref = model(ids)
            sm = paddle.jit.to_static(model)
            out = sm(ids)
        np.testing.assert_allclose(out.astype("float32").numpy(), ref.astype("float32").numpy(), rtol=0, atol=0)
        prog = next(iter(model.forward.program_cache.values())).program
        names = [n.name for n in prog.nodes]
        assert any("flash_attention" in n for n in names) and any("layer_norm" in n for n in names)
        path = str(tmp_path / "gpt")
        paddle.jit.save(model, path, input_spec=[InputSpec([None, 64], "int64", "ids")])
        cfgi = paddle.inference.Config(path + ".pdmodel", path + ".pdiparams")
        cfgi.enable_use_gpu(100, 0)
        cfgi.enable_hip_graph()
        pred = paddle.inference.create_predictor(cfgi)
        for _ in range(2):
            o = pred.run([ids.numpy()])[0]
        np.testing.assert_allclose(o.astype("float32").numpy(), ref.astype("float32").numpy(), rtol=0, atol=0)
    finally:
        paddle.set_default_dtype("float32")
