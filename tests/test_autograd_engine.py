"""Native eager backward engine (csrc/runtime/autograd_engine.cpp, FLAGS_eager_backward_engine=native) against
PyTorch's engine on the same grad nodes. Reference semantics: paddle/fluid/eager/backward.cc:105 (RunBackward),
python/paddle/autograd/backward_mode.py, general_grad.h (paddle.grad)."""
import contextlib

import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle
from paddlepaddle_amd.autograd import engine
from paddlepaddle_amd.utils import native

pytestmark = pytest.mark.skipif(not native.available(), reason="_C_runtime not built")


@contextlib.contextmanager
def eng(name):
    old = paddle.get_flags("FLAGS_eager_backward_engine")["FLAGS_eager_backward_engine"]
    paddle.set_flags({"FLAGS_eager_backward_engine": name})
    try:
        yield
    finally:
        paddle.set_flags({"FLAGS_eager_backward_engine": old})


def test_native_engine_selected():
    with eng("native"):
        assert engine.use_native()
    with eng("torch"):
        assert not engine.use_native()


def test_mlp_parity():
    # the same weights in both runs (seeded build); compare all parameter gradients
    res = {}
    for name in ("torch", "native"):
        with eng(name):
            paddle.seed(11)
            net = paddle.nn.Sequential(paddle.nn.Linear(8, 16), paddle.nn.GELU(), paddle.nn.Linear(16, 4))
            x = paddle.randn([5, 8])
            (net(x) ** 2).mean().backward()
            res[name] = [p.grad.numpy() for p in net.parameters()]
    for a, b in zip(res["torch"], res["native"]):
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7)


def test_conv_bn_parity():
    res = {}
    for name in ("torch", "native"):
        with eng(name):
            paddle.seed(3)
            net = paddle.nn.Sequential(paddle.nn.Conv2D(3, 8, 3, padding=1), paddle.nn.BatchNorm2D(8),
                                       paddle.nn.ReLU(), paddle.nn.AdaptiveAvgPool2D(1), paddle.nn.Flatten(),
                                       paddle.nn.Linear(8, 10))
            x = paddle.randn([4, 3, 8, 8])
            y = paddle.randint(0, 10, [4])
            paddle.nn.functional.cross_entropy(net(x), y).backward()
            res[name] = [p.grad.numpy() for p in net.parameters() if p.grad is not None]
    assert len(res["torch"]) == len(res["native"])
    for a, b in zip(res["torch"], res["native"]):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)


def test_gpt_tiny_parity_and_accumulation():
    from paddlepaddle_amd.models.gpt import GPTConfig, GPTForPretraining, GPTPretrainingCriterion
    res = {}
    for name in ("torch", "native"):
        with eng(name):
            paddle.seed(7)
            cfg = GPTConfig.tiny(hidden_size=64, num_attention_heads=4, intermediate_size=128, num_hidden_layers=2,
                                 vocab_size=97, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
            model = GPTForPretraining(cfg)
            crit = GPTPretrainingCriterion(cfg)
            ids = paddle.randint(0, 97, [2, 17])
            for _ in range(2):  # two micro-batches: leaf gradients accumulate
                crit(model(ids[:, :-1]), ids[:, 1:]).backward()
            res[name] = {n: p.grad.numpy() for n, p in model.named_parameters() if p.grad is not None}
    assert res["torch"].keys() == res["native"].keys() and len(res["torch"]) > 10
    for k in res["torch"]:
        np.testing.assert_allclose(res["torch"][k], res["native"][k], rtol=1e-5, atol=1e-6, err_msg=k)


def test_hooks_retain_grads_and_multi_output():
    with eng("native"):
        x = paddle.to_tensor(np.arange(6, dtype="float32"), stop_gradient=False)
        a, b = paddle.split(x * 1.0, 2)
        a.retain_grads()
        calls = []
        h = a.register_hook(lambda g: (calls.append(1), g * 10)[1])
        loss = (a * 2).sum() + (b * b).sum() * 0  # b's slot contributes a zero gradient
        loss.backward()
        np.testing.assert_allclose(x.grad.numpy(), [20, 20, 20, 0, 0, 0])
        np.testing.assert_allclose(a.grad.numpy(), [2, 2, 2])  # retained before the hook ran, like paddle
        assert calls == [1]
        assert h.remove()
        # leaf hook: applied to the leaf's summed gradient before accumulation
        w = paddle.to_tensor([1.0, 2.0], stop_gradient=False)
        w.register_hook(lambda g: g + 1)
        ((w * 3).sum() + (w * 4).sum()).backward()
        np.testing.assert_allclose(w.grad.numpy(), [8, 8])


def test_pylayer_and_unused_slot_zero_fill():
    class TwoOut(paddle.autograd.PyLayer):
        @staticmethod
        def forward(ctx, x):
            return x * 2, x * 3

        @staticmethod
        def backward(ctx, g1, g2):
            return g1 * 2 + g2 * 3

    with eng("native"):
        x = paddle.to_tensor([1.0, -1.0], stop_gradient=False)
        p, q = TwoOut.apply(x)
        p.sum().backward()  # q's gradient slot is undefined -> zeros for the Python backward
        np.testing.assert_allclose(x.grad.numpy(), [2, 2])


def test_paddle_grad_prune_capture_and_double_backward():
    with eng("native"):
        a = paddle.to_tensor([1.0, 2.0, 3.0], stop_gradient=False)
        c = paddle.to_tensor([5.0], stop_gradient=False)
        u = paddle.to_tensor([1.0], stop_gradient=False)
        out = (a ** 3).sum() + c.sum() * 2
        ga, gc, gu = paddle.grad(out, [a, c, u], create_graph=True, allow_unused=True)
        np.testing.assert_allclose(ga.numpy(), [3, 12, 27])
        np.testing.assert_allclose(gc.numpy(), [2])
        assert gu is None
        assert a.grad is None and c.grad is None  # paddle.grad captures, does not accumulate
        (gga,) = paddle.grad(ga.sum(), a)
        np.testing.assert_allclose(gga.numpy(), [6, 12, 18])
        with pytest.raises(RuntimeError):
            paddle.grad((a * 2).sum(), [u])


def test_amp_dtype_mixing():
    res = {}
    for name in ("torch", "native"):
        with eng(name):
            paddle.seed(2)
            lin = paddle.nn.Linear(8, 8)
            x = paddle.randn([4, 8])
            y = lin(x).astype("bfloat16")
            (y.astype("float32") * 3).sum().backward()
            res[name] = lin.weight.grad.numpy()
    np.testing.assert_allclose(res["torch"], res["native"], rtol=1e-6)


def test_post_accumulate_hooks_fire():
    # DataParallel / sharding grad-ready hooks ride on the leaf accumulation node
    with eng("native"):
        w = paddle.to_tensor([1.0, 2.0], stop_gradient=False)
        seen = []
        w._t.register_post_accumulate_grad_hook(lambda t: seen.append(t.grad.clone()))
        (w * w).sum().backward()
        assert len(seen) == 1
        np.testing.assert_allclose(seen[0].numpy(), [2, 4])


@pytest.mark.gpu
def test_gpt_tiny_hip_kernels_native_engine():
    from paddlepaddle_amd.models.gpt import GPTConfig, GPTForPretraining, GPTPretrainingCriterion
    from paddlepaddle_amd.ops import _loader
    assert torch.cuda.is_available()
    paddle.set_device("gpu:0")
    res = {}
    for name in ("torch", "native"):
        with eng(name):
            paddle.seed(7)
            cfg = GPTConfig.tiny(hidden_size=256, num_attention_heads=2, intermediate_size=1024,
                                 hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
            paddle.set_default_dtype("bfloat16")
            model = GPTForPretraining(cfg)
            paddle.set_default_dtype("float32")
            crit = GPTPretrainingCriterion(cfg)
            ids = paddle.randint(0, cfg.vocab_size, [2, 129])
            crit(model(ids[:, :-1]), ids[:, 1:]).backward()
            torch.cuda.synchronize()
            res[name] = {n: p.grad.astype("float32").numpy() for n, p in model.named_parameters()
                         if p.grad is not None}
    assert _loader._LIB is not None, "HIP kernel library was not loaded"
    assert res["torch"].keys() == res["native"].keys()
    for k in res["torch"]:
        np.testing.assert_allclose(res["torch"][k], res["native"][k], rtol=2e-2, atol=2e-3, err_msg=k)


def test_torch_api_hooks_fire_once_under_native_engine():
    """hooks registered through torch's own API (Tensor.register_hook on the torch tensor, Module
    full-backward hooks) fire under the native executor; hooks registered through paddle fire exactly once."""
    with eng("native"):
        assert engine.runs_tensor_hooks()
        x = paddle.to_tensor([1.0, 2.0, 3.0], stop_gradient=False)
        y = x * 2
        seen_t, seen_p = [], []
        y._t.register_hook(lambda g: seen_t.append(g.clone()))
        y.register_hook(lambda g: (seen_p.append(1), g * 3)[1])
        x._t.register_hook(lambda g: g + 1)  # leaf hook through torch
        y.sum().backward()
        assert len(seen_t) == 1 and seen_p == [1]
        np.testing.assert_allclose(x.grad.numpy(), [7, 7, 7])
        # torch.nn.Module full-backward hooks are tensor pre-hooks on the module's output grad nodes
        lin = torch.nn.Linear(4, 2)
        got = []
        lin.register_full_backward_hook(lambda m, gi, go: got.append((gi[0].shape, go[0].shape)))
        inp = paddle.to_tensor(np.ones((3, 4), "float32"), stop_gradient=False)
        out = paddle.Tensor(lin(inp._t))
        out.sum().backward()
        assert got == [(torch.Size([3, 4]), torch.Size([3, 2]))]
        # torch retain_grad on a non-leaf
        z = x * 5
        z._t.retain_grad()
        (z * z).sum().backward()
        np.testing.assert_allclose(z._t.grad.numpy(), (2 * z).numpy())


def test_failed_backward_drops_queued_callbacks():
    with eng("native"):
        class Owner:
            _queued = True

            def cb(self):
                raise AssertionError("stale callback fired")
        o = Owner()

        class Boom(paddle.autograd.PyLayer):
            @staticmethod
            def forward(ctx, x):
                return x * 1

            @staticmethod
            def backward(ctx, g):
                engine.queue_callback(o.cb)
                raise ValueError("boom")
        x = paddle.to_tensor([1.0], stop_gradient=False)
        with pytest.raises(Exception):
            Boom.apply(x).sum().backward()
        assert not o._queued and not engine._FINAL
        (x * 2).sum().backward()  # an unrelated backward runs no stale callback


@pytest.mark.gpu
def test_side_stream_forward_native_engine():
    """A forward run on a side stream: each grad node runs on its forward's stream, gradients crossing streams
    are event-ordered and the caller's stream waits for the backward."""
    assert torch.cuda.is_available()
    paddle.set_device("gpu:0")
    res = {}
    for name in ("torch", "native"):
        with eng(name):
            torch.manual_seed(0)
            w = torch.randn(2048, 2048, device="cuda", requires_grad=True)
            x = torch.randn(4096, 2048, device="cuda")
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                h = x
                for _ in range(6):
                    h = torch.tanh(h @ w)
            torch.cuda.current_stream().wait_stream(side)
            loss = paddle.Tensor(h).square().sum()
            loss.backward()
            res[name] = w.grad.clone()  # read on the caller's stream right after backward
    torch.cuda.synchronize()
    torch.testing.assert_close(res["native"], res["torch"], rtol=1e-3, atol=1e-3)
