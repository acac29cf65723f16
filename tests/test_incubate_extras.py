"""paddle.incubate submodules: operators.ResNetUnit, layers (correlation, partial_*, batch_fc, shuffle_batch,
pow2 decay), framework RNG index registry, checkpoint.auto_checkpoint, jit.inference, multiprocessing, tensor,
xpu.ResNetBasicBlock, optimizers (LARS, gradient merge, DistributedFusedLamb). CPU; fp32 references."""
import os

import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle
from paddlepaddle_amd import incubate


def _np(t):
    return t.numpy() if hasattr(t, "numpy") else np.asarray(t)


def test_resnet_unit_matches_conv_bn_relu_composition():
    paddle.seed(1)
    unit = incubate.operators.ResNetUnit(8, 16, 3, stride=1, data_format="NHWC", has_shortcut=True,
                                         num_channels_z=8, stride_z=1)
    x = paddle.randn([2, 6, 6, 8])
    z = paddle.randn([2, 6, 6, 8])
    out = unit(x, z)
    xt, zt = x._t.permute(0, 3, 1, 2), z._t.permute(0, 3, 1, 2)

    def cbn(inp, f, pad):
        y = torch.nn.functional.conv2d(inp, f._t.permute(0, 3, 1, 2), None, 1, pad)
        m, v = y.mean((0, 2, 3), keepdim=True), y.var((0, 2, 3), unbiased=False, keepdim=True)
        return (y - m) / torch.sqrt(v + 1e-5)
    ref = torch.relu(cbn(xt, unit.filter_x, 1) + cbn(zt, unit.filter_z, 1)).permute(0, 2, 3, 1)
    np.testing.assert_allclose(_np(out), ref.detach().numpy(), rtol=1e-4, atol=1e-4)
    # running statistics moved towards the batch statistics
    assert float(unit.mean_x._t.abs().sum()) > 0
    out.sum().backward()
    assert unit.filter_x.grad is not None and unit.scale_z.grad is not None


def test_resnet_basic_block_nchw_runs_and_trains():
    paddle.seed(2)
    blk = incubate.xpu.ResNetBasicBlock(4, 4, 3, 4, 4, 3, 4, 4, 1, padding1=1, padding2=1, data_format="NCHW")
    x = paddle.randn([2, 4, 5, 5])
    x.stop_gradient = False
    y = blk(x)
    assert tuple(y.shape) == (2, 4, 5, 5) and float(y._t.min()) >= 0
    y.mean().backward()
    assert x.grad is not None


def test_correlation_matches_direct_loop():
    rng = np.random.RandomState(0)
    a = rng.randn(1, 3, 7, 7).astype("float32")
    b = rng.randn(1, 3, 7, 7).astype("float32")
    pad, k, md, s1, s2 = 2, 3, 2, 1, 1
    out = _np(incubate.layers.correlation(paddle.to_tensor(a), paddle.to_tensor(b), pad, k, md, s1, s2))
    pa = np.pad(a, ((0, 0), (0, 0), (pad, pad), (pad, pad)))
    pb = np.pad(b, ((0, 0), (0, 0), (pad, pad), (pad, pad)))
    kr, dr = 1, md // s2
    D = 2 * dr + 1
    OH = out.shape[2]
    ref = np.zeros_like(out)
    for oy in range(OH):
        for ox in range(out.shape[3]):
            h1, w1 = oy * s1 + md, ox * s1 + md
            for tj in range(-dr, dr + 1):
                for ti in range(-dr, dr + 1):
                    acc = 0.0
                    for j in range(-kr, kr + 1):
                        for i in range(-kr, kr + 1):
                            acc += (pa[0, :, h1 + j, w1 + i] * pb[0, :, h1 + tj * s2 + j, w1 + ti * s2 + i]).sum()
                    ref[0, (tj + dr) * D + ti + dr, oy, ox] = acc / (k * k * 3)
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-5)


def test_partial_ops_batch_fc_shuffle_and_pow2_decay():
    x = paddle.to_tensor(np.array([[0, 1, 2], [3, 4, 5]], "float32"))
    y = paddle.to_tensor(np.array([[6, 7, 8], [9, 10, 11]], "float32"))
    np.testing.assert_array_equal(_np(incubate.layers.partial_concat([x, y], 0, 2)),
                                  [[0, 1, 6, 7], [3, 4, 9, 10]])
    np.testing.assert_array_equal(_np(incubate.layers.partial_sum([x, y], 1, 2)), [[8, 10], [14, 16]])
    inp = paddle.randn([3, 4, 5])
    out = incubate.layers.batch_fc(inp, [3, 5, 2], None, [3, 2], None, act="relu")
    assert tuple(out.shape) == (3, 4, 2) and float(out._t.min()) >= 0
    s = incubate.layers.shuffle_batch(paddle.to_tensor(np.arange(20, dtype="float32").reshape(10, 2)), seed=3)
    rows = sorted(map(tuple, _np(s).tolist()))
    assert rows == [(2.0 * i, 2.0 * i + 1) for i in range(10)]
    lr = incubate.layers.pow2_decay_with_linear_warmup(2, 6, 1.0, 0.1)
    vals = [lr.step() for _ in range(7)]
    np.testing.assert_allclose(vals, [0.5, 1.0, 0.1 + 0.9 * 0.75 ** 2, 0.1 + 0.9 * 0.25, 0.1 + 0.9 * 0.0625, 0.1,
                                      0.1], rtol=1e-6)
    with pytest.raises(NotImplementedError):
        incubate.layers.tdm_child(x, None, None)


def test_rng_state_index_registry():
    paddle.seed(5)
    idx = incubate.register_rng_state_as_index(device="cpu")
    a = paddle.rand([3]).numpy()
    incubate.set_rng_state(idx, device="cpu", use_index=True)
    b = paddle.rand([3]).numpy()
    np.testing.assert_array_equal(a, b)
    st = incubate.get_rng_state(device="cpu")
    c = paddle.rand([3]).numpy()
    incubate.set_rng_state(st, device="cpu")
    np.testing.assert_array_equal(c, paddle.rand([3]).numpy())


def test_auto_checkpoint_resumes_after_interruption(tmp_path, monkeypatch):
    from paddlepaddle_amd.incubate.checkpoint import auto_checkpoint as acp
    monkeypatch.setenv("PADDLE_RUNNING_ENV", "PADDLE_EDL_AUTO_CHECKPOINT")
    monkeypatch.setenv("PADDLE_EDL_HDFS_CHECKPOINT_PATH", str(tmp_path))
    monkeypatch.setenv("PADDLE_JOB_ID", "job_a")
    lin = paddle.nn.Linear(2, 2)
    acp._REGISTERED.clear()
    acp.register("model", lin)
    seen = []
    for ep in acp.train_epoch_range(5, save_checkpoint_inter=0):
        seen.append(ep)
        lin.weight.set_value(np.full((2, 2), float(ep), "float32"))
        if ep == 2:
            break                    # "killed" inside epoch 2: epochs 0, 1 were saved
    lin.weight.set_value(np.zeros((2, 2), "float32"))
    resumed = list(acp.train_epoch_range(5, save_checkpoint_inter=0))
    assert seen == [0, 1, 2] and resumed == [2, 3, 4]
    acp._REGISTERED.clear()


def test_jit_inference_decorator_matches_eager(tmp_path):
    paddle.seed(0)
    lin = paddle.nn.Linear(4, 3)
    x = paddle.randn([2, 4])
    ref = lin(x).numpy()
    fast = incubate.jit.inference(lin, save_model_dir=str(tmp_path))
    assert incubate.jit.is_inference_mode(fast)
    np.testing.assert_allclose(fast(x).numpy(), ref, rtol=1e-5, atol=1e-5)


def test_multiprocessing_shares_tensors():
    import pickle
    from multiprocessing.reduction import ForkingPickler
    from paddlepaddle_amd.incubate import multiprocessing as mp  # noqa: F401
    t = paddle.to_tensor(np.arange(4, dtype="float32"))
    buf = ForkingPickler.dumps(t)
    back = pickle.loads(buf)
    np.testing.assert_array_equal(back.numpy(), t.numpy())


def test_async_offload_reload_roundtrip():
    from paddlepaddle_amd.incubate import tensor as it
    ld = it.create_async_load()
    x = paddle.randn([3, 3])
    h, task = it.async_offload(x, ld)
    task.cpu_wait()
    back, task2 = it.async_reload(h, ld)
    task2.wait()
    np.testing.assert_array_equal(back.numpy(), x.numpy())
    assert it._npu_identity(x) is x


def test_lars_momentum_update_matches_formula():
    from paddlepaddle_amd.incubate.optimizer import LarsMomentumOptimizer
    lin = paddle.nn.Linear(3, 2, bias_attr=False)
    w0 = lin.weight.numpy().copy()
    opt = LarsMomentumOptimizer(0.1, 0.9, lars_coeff=0.01, lars_weight_decay=0.001, parameter_list=lin.parameters())
    x = paddle.randn([4, 3])
    lin(x).sum().backward()
    g = lin.weight.grad.numpy()
    opt.step()
    pn, gn = np.linalg.norm(w0), np.linalg.norm(g)
    local = 0.1 * 0.01 * pn / (0.001 * pn + gn)
    np.testing.assert_allclose(lin.weight.numpy(), w0 - local * (g + 0.001 * w0), rtol=1e-5, atol=1e-6)


def test_gradient_merge_applies_every_k_steps_with_average():
    from paddlepaddle_amd.incubate.optimizer import GradientMergeOptimizer
    lin = paddle.nn.Linear(2, 1, bias_attr=False)
    w0 = lin.weight.numpy().copy()
    opt = GradientMergeOptimizer(paddle.optimizer.SGD(1.0, parameters=lin.parameters()), k_steps=2, avg=True)
    xs = [paddle.to_tensor(np.array([[1.0, 0.0]], "float32")), paddle.to_tensor(np.array([[0.0, 3.0]], "float32"))]
    lin(xs[0]).sum().backward()
    opt.step()
    opt.clear_grad()
    np.testing.assert_array_equal(lin.weight.numpy(), w0)       # not applied yet, gradient kept
    lin(xs[1]).sum().backward()
    opt.step()
    opt.clear_grad()
    np.testing.assert_allclose(lin.weight.numpy(), w0 - np.array([[0.5], [1.5]], "float32"), rtol=1e-6)
    assert lin.weight.grad is None or float(np.abs(lin.weight.grad.numpy()).sum()) == 0.0


def test_fuse_resnet_unit_pass_enables_runtime_fusion():
    from paddlepaddle_amd.framework import flags
    flags.set_flags({"FLAGS_conv_bn_fusion": False})
    incubate.fuse_resnet_unit_pass.fuse_resnet_unit()
    assert flags.flag("FLAGS_conv_bn_fusion") is True
    assert os.path.basename(incubate.passes.__file__) == "__init__.py"
