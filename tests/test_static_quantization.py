"""paddle.static.quantization on this framework's Programs: post-training quantization of a saved inference
model (calibration -> int8 weights + activation quant-dequant nodes -> saved, reloadable), weight-only
quantization, and static QAT (quant_aware trains through fake-quant nodes; convert freezes them). CPU."""
import numpy as np
import pytest

import paddlepaddle_amd as paddle
from paddlepaddle_amd.static import quantization as SQ


def _build_and_save(tmp_path):
    paddle.enable_static()
    try:
        main, start = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, start):
            paddle.seed(4)
            x = paddle.static.data("x", [8, 3, 6, 6], "float32")
            conv = paddle.nn.Conv2D(3, 4, 3, padding=1)
            lin = paddle.nn.Linear(4 * 6 * 6, 5)
            h = paddle.nn.functional.relu(conv(x))
            y = lin(h.reshape([8, -1]))
        exe = paddle.static.Executor(paddle.CPUPlace())
        feed = np.random.RandomState(0).rand(8, 3, 6, 6).astype("float32")
        ref = exe.run(main, feed={"x": feed}, fetch_list=[y])[0]
        paddle.static.save_inference_model(str(tmp_path / "fp32" / "model"), [x], [y], exe, program=main)
        return exe, feed, ref
    finally:
        paddle.disable_static()


@pytest.mark.parametrize("algo", ["KL", "abs_max", "hist", "avg"])
def test_post_training_quantization_roundtrip(tmp_path, algo):
    exe, feed, ref = _build_and_save(tmp_path)
    rng = np.random.RandomState(1)

    def batches():
        for _ in range(4):
            yield [rng.rand(8, 3, 6, 6).astype("float32")]
    paddle.enable_static()
    try:
        ptq = SQ.PostTrainingQuantization(exe, str(tmp_path / "fp32"), batch_generator=batches, algo=algo,
                                          quantizable_op_type=["conv2d", "mul"])
        prog = ptq.quantize()
        names = [n.name for n in prog.nodes]
        assert sum(n.endswith(":fake_quant_act") for n in names) == 2
        out = exe.run(prog, feed={"x": feed}, fetch_list=ptq._fetch_list)[0]
        ptq.save_quantized_model(str(tmp_path / "int8"))
        prog2, feeds, fetch = paddle.static.load_inference_model(str(tmp_path / "int8" / "model"), exe)
        out2 = exe.run(prog2, feed={"x": feed}, fetch_list=fetch)[0]
    finally:
        paddle.disable_static()
    np.testing.assert_allclose(out2, out, rtol=1e-5, atol=1e-5)
    assert np.abs(out - ref).max() < 0.1 * np.abs(ref).max() + 1e-3


def test_weight_quantization_keeps_outputs_close(tmp_path):
    exe, feed, ref = _build_and_save(tmp_path)
    paddle.enable_static()
    try:
        SQ.WeightQuantization(str(tmp_path / "fp32")).quantize_weight_to_int(str(tmp_path / "wq"), weight_bits=8)
        prog, feeds, fetch = paddle.static.load_inference_model(str(tmp_path / "wq" / "model"), exe)
        out = exe.run(prog, feed={"x": feed}, fetch_list=fetch)[0]
    finally:
        paddle.disable_static()
    assert np.abs(out - ref).max() < 0.05 * np.abs(ref).max() + 1e-3


def test_static_quant_aware_trains_and_converts():
    paddle.enable_static()
    try:
        main, start = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, start):
            paddle.seed(7)
            x = paddle.static.data("x", [16, 4], "float32")
            t = paddle.static.data("t", [16, 1], "float32")
            lin = paddle.nn.Linear(4, 8)
            lin2 = paddle.nn.Linear(8, 1)
            y = lin2(paddle.nn.functional.relu(lin(x)))
            loss = ((y - t) ** 2).mean()
            paddle.optimizer.Adam(0.02).minimize(loss)
        qprog = SQ.quant_aware(main, paddle.CPUPlace(), {"quantize_op_types": ["mul"]})
        assert sum(n.name.endswith(":qat_fake_quant_act") for n in qprog.nodes) == 2
        exe = paddle.static.Executor(paddle.CPUPlace())
        rng = np.random.RandomState(0)
        xs = rng.rand(16, 4).astype("float32")
        ts = (xs.sum(1, keepdims=True) * 0.5).astype("float32")
        losses = [float(exe.run(qprog, feed={"x": xs, "t": ts}, fetch_list=[loss])[0]) for _ in range(40)]
        assert losses[-1] < 0.5 * losses[0]
        frozen = SQ.convert(qprog, paddle.CPUPlace())
        names = [n.name for n in frozen.nodes]
        assert not any(n.endswith(":qat_fake_quant_act") for n in names)
        assert sum(n.endswith(":fake_quant_act") for n in names) >= 2
    finally:
        paddle.disable_static()
