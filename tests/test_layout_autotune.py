"""Layout autotune (framework/layout_autotune.py; reference: paddle/fluid/imperative/layout_autotune.cc,
eager/eager_layout_auto_tune.h:127): with FLAGS_layout_autotune on, an NCHW model runs the NHWC HIP conv / BN /
max-pool kernels on channels-last views; shapes and results are those of the NCHW model."""
import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle
from paddlepaddle_amd.framework import layout_autotune as LA


def test_set_config_drives_the_flag_that_the_dispatch_reads():
    from paddlepaddle_amd.incubate import autotune
    try:
        autotune.set_config({"layout": {"enable": True}})
        assert LA.enabled()
        # CPU tensors never take the channels-last path (the NHWC kernels are device kernels)
        assert not LA.applies(torch.zeros(1, 3, 8, 8))
        conv = paddle.nn.Conv2D(3, 4, 3, padding=1)
        x = paddle.randn([2, 3, 8, 8])
        y = conv(x)
        assert y.shape == [2, 4, 8, 8]
    finally:
        autotune.set_config({"layout": {"enable": False}})
    assert not LA.enabled()


def test_views_round_trip():
    t = torch.randn(2, 3, 4, 5)
    v = LA.to_nhwc_view(t)
    assert v.shape == (2, 4, 5, 3) and v.is_contiguous()
    back = LA.to_nchw_view(v)
    assert back.shape == t.shape and torch.equal(back, t) and back.is_contiguous(memory_format=torch.channels_last)


def _resnet(fmt):
    from paddlepaddle_amd.vision.models import resnet50
    paddle.seed(5)
    m = resnet50(num_classes=10, data_format=fmt)
    opt = paddle.optimizer.Momentum(learning_rate=0.1, momentum=0.9, parameters=m.parameters(), multi_precision=True)
    m, opt = paddle.amp.decorate(m, opt, level="O2", dtype="bfloat16")
    return m


@pytest.mark.gpu
def test_nchw_resnet50_with_autotune_runs_the_nhwc_kernels_and_matches():
    from paddlepaddle_amd.ops import _loader as L
    paddle.set_device("gpu:0")
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(8, 3, 64, 64, device="cuda", generator=g).bfloat16()
    y = torch.randint(0, 10, (8,), device="cuda", generator=g)
    res = {}
    # a first NHWC pass settles the per-shape backend choices (ops/gemm.py choose() times candidates on first
    # use); the compared runs then take the same kernels
    for name in ("warmup", "nhwc", "nchw_autotune"):
        m = _resnet("NCHW" if name == "nchw_autotune" else "NHWC")
        paddle.set_flags({"FLAGS_layout_autotune": name == "nchw_autotune"})
        L.reset_calls()
        try:
            inp = paddle.Tensor(x if name == "nchw_autotune" else x.permute(0, 2, 3, 1).contiguous())
            with paddle.amp.auto_cast(level="O2", dtype="bfloat16"):
                out = m(inp)
            loss = paddle.nn.functional.cross_entropy(out.astype("float32"), paddle.Tensor(y))
            loss.backward()
            torch.cuda.synchronize()
        finally:
            paddle.set_flags({"FLAGS_layout_autotune": False})
        res[name] = (out.astype("float32").numpy(), float(loss), m.conv1.weight.grad.astype("float32").numpy(),
                     m.fc.weight.grad.astype("float32").numpy(), dict(L.CALLS))
    (o1, l1, g1, f1, c1), (o2, l2, g2, f2, c2) = res["nhwc"], res["nchw_autotune"]
    assert o2.shape == (8, 10)
    np.testing.assert_allclose(o2, o1, rtol=2e-2, atol=2e-2)
    assert abs(l1 - l2) < 1e-2 * max(1.0, abs(l1))
    # conv1's weight gradient: the NCHW stem weight [64, 3, 7, 7] in both models
    np.testing.assert_allclose(g2, g1, rtol=5e-2, atol=5e-2 * np.abs(g1).max())
    np.testing.assert_allclose(f2, f1, rtol=5e-2, atol=5e-2 * np.abs(f1).max())
    # the same hand-written launchers ran in both models (NHWC conv GEMMs / skinny kernels, BN, max-pool)
    hip = lambda c, key: sum(v for k, v in c.items() if key in k)  # noqa: E731
    for key in ("bn", "gemm", "pool"):
        assert hip(c2, key) > 0, (key, sorted(c2))
        assert hip(c2, key) == hip(c1, key), (key, hip(c1, key), hip(c2, key))


class _SlowDS(paddle.io.Dataset):
    """Each sample costs ~4 ms of host time (decode-like), so worker processes pay off."""

    def __len__(self):
        return 64

    def __getitem__(self, i):
        import time
        time.sleep(0.004)
        return np.full([4], i, "float32"), np.int64(i % 3)


def test_dataloader_autotune_picks_workers_and_keeps_the_data():
    from paddlepaddle_amd.incubate import autotune
    try:
        autotune.set_config({"dataloader": {"enable": True, "tuning_steps": 3}})
        dl = paddle.io.DataLoader(_SlowDS(), batch_size=8)
        assert dl.autotuned_num_workers is not None and dl.num_workers == dl.autotuned_num_workers
        xs = [x.numpy() for x, _ in dl]
        assert len(xs) == 8 and np.array_equal(np.concatenate(xs)[:, 0], np.arange(64, dtype="float32"))
        # a loader the user configured explicitly is left alone
        assert paddle.io.DataLoader(_SlowDS(), batch_size=8, num_workers=1).autotuned_num_workers is None
    finally:
        autotune.set_config({"dataloader": {"enable": False}})
    assert paddle.io.DataLoader(_SlowDS(), batch_size=8).autotuned_num_workers is None
