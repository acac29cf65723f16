"""paddle.onnx.export (reference python/paddle/onnx/export.py; paddle2onnx there): exported ModelProto bytes read
back by the in-tree protobuf reader and executed by the numpy ONNX executor (onnx/runtime.py) must reproduce eager
outputs. No onnx / onnxruntime package in this image: parity with a real ONNX runtime is unpinned."""
import numpy as np
import pytest

import paddlepaddle_amd as paddle
from paddlepaddle_amd.onnx import proto as PB
from paddlepaddle_amd.onnx import runtime as RT
from paddlepaddle_amd.static import InputSpec


class CNN(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.conv = paddle.nn.Conv2D(3, 8, 3, padding=1)
        self.bn = paddle.nn.BatchNorm2D(8)
        self.conv2 = paddle.nn.Conv2D(8, 8, 3, stride=2, padding=1, groups=2)
        self.pool = paddle.nn.AdaptiveAvgPool2D(1)
        self.fc = paddle.nn.Linear(8, 4)
        self.ln = paddle.nn.LayerNorm(4)

    def forward(self, x):
        h = paddle.nn.functional.relu(self.bn(self.conv(x)))
        h = paddle.nn.functional.max_pool2d(h, 2)
        h = paddle.nn.functional.avg_pool2d(paddle.tanh(self.conv2(h)), 1)
        h = self.pool(h).flatten(1)
        y = self.ln(self.fc(h))
        return paddle.nn.functional.softmax(paddle.nn.functional.gelu(y) * 2 + 1, -1)


class Attn(paddle.nn.Layer):
    def __init__(self, d=16, h=2):
        super().__init__()
        self.h = h
        self.qkv = paddle.nn.Linear(d, 3 * d)
        self.out = paddle.nn.Linear(d, d)
        self.norm = paddle.nn.LayerNorm(d)
        self.emb = paddle.nn.Embedding(50, d)

    def forward(self, ids):
        x = self.emb(ids)
        B, S, D = x.shape
        q, k, v = paddle.split(self.qkv(self.norm(x)), 3, axis=-1)
        q = q.reshape([B, S, self.h, D // self.h]).transpose([0, 2, 1, 3])
        k = k.reshape([B, S, self.h, D // self.h]).transpose([0, 2, 1, 3])
        v = v.reshape([B, S, self.h, D // self.h]).transpose([0, 2, 1, 3])
        a = paddle.nn.functional.softmax(paddle.matmul(q, k, transpose_y=True) / (D // self.h) ** 0.5, -1)
        o = paddle.matmul(a, v).transpose([0, 2, 1, 3]).reshape([B, S, D])
        return x + self.out(o)[:, 0:1, :].squeeze(1).unsqueeze(1)


def _check(layer, specs, feeds, tmp_path, rtol=1e-4):
    layer.eval()
    ref = layer(*[paddle.to_tensor(f) for f in feeds]).numpy()
    path = paddle.onnx.export(layer, str(tmp_path / "m"), input_spec=specs)
    data = open(path, "rb").read()
    m = PB.read_model(data)
    assert m["opset"] == 17 and m["nodes"] and len(m["outputs"]) == 1
    got = RT.run(data, {s.name: f for s, f in zip(specs, feeds)})[0]
    np.testing.assert_allclose(got, ref, rtol=rtol, atol=1e-5)
    return m


def test_cnn_export_matches_eager(tmp_path):
    paddle.seed(0)
    x = np.random.RandomState(0).randn(2, 3, 8, 8).astype("float32")
    m = _check(CNN(), [InputSpec([2, 3, 8, 8], "float32", "image")], [x], tmp_path)
    ops = {n[0] for n in m["nodes"]}
    assert {"Conv", "BatchNormalization", "MaxPool", "AveragePool", "ReduceMean", "LayerNormalization", "Softmax"} <= ops
    assert any(n[0] == "Conv" and n[3].get("group") == 2 for n in m["nodes"])


def test_attention_block_export_dynamic_batch(tmp_path):
    paddle.seed(1)
    layer = Attn()
    ids = np.random.RandomState(1).randint(0, 50, (3, 5)).astype("int64")
    layer.eval()
    path = paddle.onnx.export(layer, str(tmp_path / "attn"), input_spec=[InputSpec([None, 5], "int64", "ids")])
    data = open(path, "rb").read()
    for b in (2, 3):  # the symbolic batch dimension is honoured by the exported Reshapes
        got = RT.run(data, {"ids": ids[:b]})[0]
        np.testing.assert_allclose(got, layer(paddle.to_tensor(ids[:b])).numpy(), rtol=1e-4, atol=1e-5)


def test_proto_roundtrip_and_unsupported_op(tmp_path):
    t = PB.tensor("w", np.arange(6, dtype="float32").reshape(2, 3))
    name, arr = PB.read_tensor(t)
    assert name == "w" and arr.shape == (2, 3) and arr[1, 2] == 5

    class Bad(paddle.nn.Layer):
        def forward(self, x):
            return paddle.cumsum(x, 0)
    with pytest.raises(NotImplementedError):
        paddle.onnx.export(Bad(), str(tmp_path / "bad"), input_spec=[InputSpec([2, 2], "float32", "x")])
