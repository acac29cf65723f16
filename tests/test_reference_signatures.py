"""Constructor / function signatures that reference-style positional and keyword calls rely on (checked against
the reference's definitions: tensor/logic.py, nn/layer/rnn.py, nn/initializer/*.py, amp/grad_scaler.py,
optimizer/nadam.py, audio/features/layers.py, quantization/observers, device/__init__.py)."""
import inspect

import numpy as np

import paddlepaddle_amd as paddle
from paddlepaddle_amd.nn import initializer as I


def _params(f):
    return list(inspect.signature(f).parameters)


def test_logic_ops_take_out():
    for n in ("bitwise_and", "bitwise_or", "bitwise_xor", "logical_and", "logical_or", "logical_xor"):
        assert _params(getattr(paddle, n)) == ["x", "y", "out", "name"], n
    for n in ("bitwise_not", "logical_not", "bitwise_invert"):
        assert _params(getattr(paddle, n)) == ["x", "out", "name"], n
    a, b = paddle.to_tensor([True, False, True]), paddle.to_tensor([True, True, False])
    out = paddle.zeros([3], dtype="bool")
    assert paddle.logical_xor(a, b, out) is out
    np.testing.assert_array_equal(out.numpy(), [False, True, True])
    assert _params(paddle.trunc) == ["input", "name"] and _params(paddle.seed) == ["seed"]


def test_layer_positional_orders():
    assert _params(paddle.nn.LSTM.__init__)[11:13] == ["proj_size", "name"]
    assert _params(paddle.nn.SimpleRNN.__init__)[7] == "activation"
    rnn = paddle.nn.SimpleRNN(4, 8, 1, "forward", False, 0.0, "relu")
    y, _ = rnn(paddle.randn([2, 3, 4]))
    assert list(y.shape) == [2, 3, 8] and float(y._t.min()) >= 0.0
    assert _params(paddle.nn.AdaptiveLogSoftmaxWithLoss.__init__)[4:7] == ["weight_attr", "bias_attr", "div_value"]
    assert _params(paddle.nn.Softmax2D.__init__) == ["self", "name"]
    assert _params(paddle.nn.functional.interpolate)[7] == "name"


def test_defaults_match_reference():
    assert inspect.signature(paddle.optimizer.NAdam).parameters["learning_rate"].default == 0.002
    assert inspect.signature(paddle.amp.AmpScaler).parameters["decr_every_n_nan_or_inf"].default == 1
    assert inspect.signature(paddle.amp.GradScaler).parameters["decr_every_n_nan_or_inf"].default == 1
    sp = inspect.signature(paddle.audio.features.Spectrogram).parameters
    assert sp["hop_length"].default == 512 and sp["power"].default == 1.0
    for cls in (paddle.audio.features.LogMelSpectrogram, paddle.audio.features.MFCC):
        p = inspect.signature(cls).parameters
        assert p["n_fft"].default == 512 and p["hop_length"].default is None


def test_legacy_initializers():
    assert _params(I.XavierInitializer.__init__)[1:] == ["uniform", "fan_in", "fan_out", "seed", "gain"]
    assert _params(I.MSRAInitializer.__init__)[1:] == ["uniform", "fan_in", "seed", "negative_slope", "nonlinearity"]
    assert _params(I.NormalInitializer.__init__)[1:] == ["loc", "scale", "seed"]
    w = paddle.zeros([3, 3])
    I.UniformInitializer(0.0, 0.0, 0, diag_num=3, diag_step=3, diag_val=2.0)(w)
    np.testing.assert_array_equal(w.numpy(), 2.0 * np.eye(3))


def test_quant_layers_take_the_layer_first():
    from paddlepaddle_amd.quantization import GroupWiseWeightObserver, GroupWiseWeightObserverLayer
    assert _params(GroupWiseWeightObserverLayer.__init__)[1:3] == ["layer", "quant_bits"]
    lin = paddle.nn.Linear(4, 4)
    obs = GroupWiseWeightObserver(group_size=4)._instance(lin)
    assert obs._layer is lin and obs._bits == 8


def test_places_and_streams():
    assert paddle.XPUPlace(2).get_device_id() == 2
    assert paddle.CustomPlace("npu", 1).get_device_type() == "npu"
    assert "stream_base" in _params(paddle.device.cuda.Stream.__init__)
