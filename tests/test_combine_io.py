"""``.pdiparams`` in the reference save_combine layout (dense_tensor_serialize.cc): byte-level checks of a
hand-assembled record, round trips for every dtype, and save/load_inference_model on top of it.
Parity with files written by PaddlePaddle itself is unpinned (no such file ships with the reference)."""
import struct

import numpy as np
import torch

import paddlepaddle_amd as paddle
from paddlepaddle_amd.framework import combine_io as C


def test_record_bytes_match_the_reference_layout(tmp_path):
    p = str(tmp_path / "x.pdiparams")
    C.write_combined(p, [torch.tensor([[1.0, 2.0, 3.0]], dtype=torch.float32)])
    raw = open(p, "rb").read()
    # version, lod_level, version, desc size, desc {1: FP32 (5), 2: 1, 2: 3}, 12 data bytes
    desc = bytes([0x08, 5, 0x10, 1, 0x10, 3])
    want = struct.pack("<IQIi", 0, 0, 0, len(desc)) + desc + struct.pack("<3f", 1, 2, 3)
    assert raw == want


def test_packed_dims_and_lod_levels_are_read(tmp_path):
    desc = bytes([0x08, 3, 0x12, 2, 2, 2])  # INT64, packed dims [2, 2]
    rec = struct.pack("<IQ", 0, 1) + struct.pack("<Q", 8) + b"\x00" * 8  # one lod level of 8 bytes
    rec += struct.pack("<Ii", 0, len(desc)) + desc + struct.pack("<4q", 1, 2, 3, 4)
    p = tmp_path / "y.pdiparams"
    p.write_bytes(rec)
    (t,) = C.read_combined(str(p))
    assert t.dtype == torch.int64 and t.tolist() == [[1, 2], [3, 4]]


def test_roundtrip_dtypes(tmp_path):
    ts = [torch.randn(3, 4), torch.randn(2).double(), torch.arange(5, dtype=torch.int32),
          torch.randn(2, 2).bfloat16(), torch.randn(3).half(), torch.tensor([True, False]), torch.zeros(0, 4)]
    p = str(tmp_path / "z.pdiparams")
    C.write_combined(p, ts)
    got = C.read_combined(p)
    assert C.is_combined(p)
    for a, b in zip(ts, got):
        assert a.dtype == b.dtype and a.shape == b.shape and torch.equal(a, b)


def test_inference_model_uses_the_combined_layout(tmp_path):
    paddle.enable_static()
    try:
        main, start = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, start):
            x = paddle.static.data("x", [2, 4], "float32")
            y = paddle.nn.Linear(4, 3)(x)
        exe = paddle.static.Executor()
        xv = np.random.RandomState(0).randn(2, 4).astype("float32")
        ref, = exe.run(main, feed={"x": xv}, fetch_list=[y])
        prefix = str(tmp_path / "m")
        paddle.static.save_inference_model(prefix, [x], [y], exe, program=main)
        assert C.is_combined(prefix + ".pdiparams") and len(C.read_combined(prefix + ".pdiparams")) == 2
        prog, feeds, fetches = paddle.static.load_inference_model(prefix, exe)
        got, = exe.run(prog, feed={feeds[0]: xv}, fetch_list=fetches)
        np.testing.assert_allclose(got, ref, rtol=1e-6)
    finally:
        paddle.disable_static()


def test_bf16_model_jit_save_and_predictor(tmp_path):
    """bf16 parameters come back from the combined file as bf16 torch tensors (no numpy hop)."""
    from paddlepaddle_amd.static import InputSpec
    paddle.seed(0)
    paddle.set_default_dtype("bfloat16")
    try:
        net = paddle.nn.Linear(8, 4)
        x = paddle.randn([2, 8]).astype("bfloat16")
        ref = net(x)
        prefix = str(tmp_path / "lin")
        paddle.jit.save(net, prefix, input_spec=[InputSpec([None, 8], "bfloat16", "x")])
    finally:
        paddle.set_default_dtype("float32")
    cfg = paddle.inference.Config(prefix + ".pdmodel", prefix + ".pdiparams")
    cfg.disable_gpu()
    pred = paddle.inference.create_predictor(cfg)
    out, = pred.run([x])
    np.testing.assert_allclose(out.astype("float32").numpy(), ref.astype("float32").numpy(), rtol=0, atol=0)
