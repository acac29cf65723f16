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
    """Same weights, same input: the autotuned NCHW model equals the NHWC model bit for bit through stage 1 and
    stays within the run-to-run spread of two NHWC models at the logits (split-K partial sums and atomics make
    deep layers differ in the last bits between any two runs, amplified by small-batch BN:
    profiles/layout_autotune_stage_diff_r4.log), and launches exactly the same hand-written kernels."""
    from paddlepaddle_amd.ops import _loader as L
    paddle.set_device("gpu:0")
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(8, 3, 64, 64, device="cuda", generator=g).bfloat16()
    y = torch.randint(0, 10, (8,), device="cuda", generator=g)
    res = {}
    # a first NHWC pass settles the per-shape backend choices (ops/gemm.py choose() times candidates on first
    # use); the compared runs then take the same kernels
    # the conv -> BN statistics fusion is learned per shape during the first passes; the layout comparison runs
    # with it off so every pass takes one path (tests/test_conv_bn_fusion_gpu.py covers the fusion)
    paddle.set_flags({"FLAGS_conv_bn_fusion": False})
    for name in ("warmup", "nhwc", "nhwc2", "nhwc3", "nchw_autotune"):
        m = _resnet("NCHW" if name == "nchw_autotune" else "NHWC")
        stage1 = []
        h = m.layer1.register_forward_post_hook(lambda l, i, o: stage1.append(o._t.detach().float()))
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
            h.remove()
        s1 = stage1[0] if name == "nchw_autotune" else stage1[0].permute(0, 3, 1, 2)
        res[name] = (out.astype("float32").numpy(), float(loss), s1, dict(L.CALLS))
    paddle.set_flags({"FLAGS_conv_bn_fusion": True})
    (o1, l1, s1, c1), (o2, l2, _, _), (o3, l3, s3, c3) = res["nhwc"], res["nhwc2"], res["nchw_autotune"]
    assert o3.shape == (8, 10)
    assert torch.equal(s3, s1), "stage-1 outputs differ"
    # run-to-run spread from three NHWC runs (one pair alone can land unusually close and under-state it)
    refs = [o1, o2, res["nhwc3"][0]]
    spread = max(np.abs(a - b).max() for i, a in enumerate(refs) for b in refs[i + 1:])
    dist_ = min(np.abs(o3 - r).max() for r in refs)
    assert dist_ <= 3 * spread + 2e-2, (dist_, spread)
    hip = lambda c, key: sum(v for k, v in c.items() if key in k)  # noqa: E731
    for key in ("bn", "gemm", "pool"):
        assert hip(c3, key) > 0, (key, sorted(c3))
        assert hip(c3, key) == hip(c1, key), (key, hip(c1, key), hip(c3, key))


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
