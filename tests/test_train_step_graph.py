"""A whole ResNet training step (forward, backward, Momentum multi-tensor update) captured into a hipGraph
and replayed must train exactly like the eager step (bench.py --resnet-graph). Guards the pointer tables
the multi-tensor optimizers copy to the device: a captured copy reads its host buffer on every replay."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _make(paddle):
    from paddlepaddle_amd.vision.models import resnet50
    paddle.seed(7)
    model = resnet50(num_classes=16, data_format="NHWC")
    opt = paddle.optimizer.Momentum(learning_rate=0.002, momentum=0.9, parameters=model.parameters(),
                                    weight_decay=1e-4, multi_precision=True)
    model, opt = paddle.amp.decorate(model, opt, level="O2", dtype="bfloat16")
    return model, opt


def test_captured_resnet_step_matches_eager():
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.device.cuda.graphs import CUDAGraph
    paddle.set_device("gpu")
    g = torch.Generator(device="cuda").manual_seed(3)
    x = paddle.Tensor(torch.randn(16, 64, 64, 3, device="cuda", dtype=torch.bfloat16, generator=g))
    y = paddle.Tensor(torch.randint(0, 16, (16,), device="cuda", generator=g))
    runs = []
    for use_graph in (False, True):
        model, opt = _make(paddle)

        def step():
            with paddle.amp.auto_cast(level="O2", dtype="bfloat16"):
                out = model(x)
            loss = paddle.nn.functional.cross_entropy(out.astype("float32"), y)
            loss.backward()
            opt.step()
            opt.clear_grad(set_to_zero=False)
            return loss
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        if use_graph:
            cg = CUDAGraph()
            cg.capture_begin()
            step()
            cg.capture_end()
            for _ in range(2):
                cg.replay()
        else:
            for _ in range(2):
                step()
        torch.cuda.synchronize()
        runs.append([p._t.detach().float().clone() for p in model.parameters()])
    # bf16 training with nondeterministic reductions: two eager runs differ by ~0.1 after five steps (max
    # |param| ~1), a broken replay (stale pointer table, lost update) diverges to inf / nan
    worst = max((a - b).abs().max().item() for a, b in zip(*runs))
    assert worst < 0.3, worst
    assert all(torch.isfinite(b).all() for b in runs[1])


def test_captured_adamw_follows_lr_schedule_and_bias_correction():
    """A captured AdamW step reads lr and the beta powers from device memory: replays advance the bias
    correction in-graph and follow the LR scheduler (frozen host floats ignored the schedule)."""
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.device.cuda.graphs import CUDAGraph
    paddle.set_device("gpu")
    g = torch.Generator(device="cuda").manual_seed(5)
    x = paddle.Tensor(torch.randn(32, 64, device="cuda", generator=g))
    runs = []
    for use_graph in (False, True):
        paddle.seed(11)
        net = paddle.nn.Sequential(paddle.nn.Linear(64, 128), paddle.nn.Tanh(), paddle.nn.Linear(128, 64))
        sched = paddle.optimizer.lr.StepDecay(learning_rate=1e-2, step_size=1, gamma=0.5)
        opt = paddle.optimizer.AdamW(learning_rate=sched, parameters=net.parameters(), weight_decay=0.01)

        def step():
            loss = (net(x) ** 2).mean()
            loss.backward()
            opt.step()
            opt.clear_grad(set_to_zero=False)
        for _ in range(3):
            step()
            sched.step()
        torch.cuda.synchronize()
        if use_graph:
            cg = CUDAGraph()
            cg.capture_begin()
            step()
            cg.capture_end()
            for _ in range(3):
                cg.replay()
                sched.step()
        else:
            for _ in range(3):
                step()
                sched.step()
        torch.cuda.synchronize()
        runs.append([p._t.detach().clone() for p in net.parameters()])
    worst = max((a - b).abs().max().item() for a, b in zip(*runs))
    assert worst < 1e-5, worst
