"""Reference-format .pdmodel (ProgramDesc protobuf, framework.proto) decode / encode and execution over this
framework's ops. No reference-exported .pdmodel ships with the reference tree, so programs are assembled with
ProgramDescBuilder against the framework.proto field numbers and operator attribute names of the reference
(paddle/fluid/framework/framework.proto, paddle/phi/ops/yaml/op_compat.yaml); results are compared with
independent torch fp32 computations (parity with the reference's own executor unpinned)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as TF

import paddlepaddle_amd as paddle
from paddlepaddle_amd.framework import program_desc as pd


def test_codec_roundtrip_and_packed():
    msg = {"blocks": [{"idx": 0, "parent_idx": -1, "vars": [
        {"name": "x", "type": {"type": 7, "dense_tensor": {"tensor": {"data_type": 5, "dims": [-1, 3, 224]}}},
         "persistable": 0}],
        "ops": [{"type": "scale", "inputs": [{"parameter": "X", "arguments": ["x"]}],
                 "outputs": [{"parameter": "Out", "arguments": ["y"]}],
                 "attrs": [{"name": "scale", "type": pd.FLOAT, "f": 0.5},
                           {"name": "axes", "type": pd.INTS, "ints": [-1, 0, 7]},
                           {"name": "alpha", "type": pd.FLOAT64, "float64": 1e-300},
                           {"name": "s", "type": pd.STRING, "s": "héllo"}]}]}],
        "version": {"version": 3}}
    back = pd.decode(pd.encode(msg))
    assert back == msg
    # packed repeated int64 (what proto3-style writers emit): TensorDesc dims = [2, -1]
    packed = b"\x08\x05" + b"\x12" + bytes([11]) + b"\x02" + b"\xff" * 9 + b"\x01"
    assert pd.decode(packed, "TensorDesc") == {"data_type": 5, "dims": [2, -1]}
    attrs = pd.op_attrs(msg["blocks"][0]["ops"][0])
    assert attrs["axes"] == [-1, 0, 7] and attrs["s"] == "héllo" and abs(attrs["scale"] - 0.5) < 1e-7


def _mlp(tmp_path):
    rng = np.random.RandomState(0)
    w1, b1 = rng.randn(8, 16).astype("float32"), rng.randn(16).astype("float32")
    w2 = rng.randn(4, 16).astype("float32")
    b = pd.ProgramDescBuilder()
    b.feed("x", [-1, 8])
    b.param("fc_0.w_0", w1), b.param("fc_0.b_0", b1), b.param("fc_1.w_0", w2)
    b.op("matmul_v2", {"X": ["x"], "Y": ["fc_0.w_0"]}, {"Out": ["h0"]}, trans_x=False, trans_y=False)
    b.op("elementwise_add", {"X": ["h0"], "Y": ["fc_0.b_0"]}, {"Out": ["h1"]}, axis=1)
    b.op("relu", {"X": ["h1"]}, {"Out": ["h2"]})
    b.op("matmul_v2", {"X": ["h2"], "Y": ["fc_1.w_0"]}, {"Out": ["h3"]}, trans_x=False, trans_y=True)
    b.op("softmax", {"X": ["h3"]}, {"Out": ["prob"]}, axis=-1)
    b.fetch("prob")
    prefix = str(tmp_path / "mlp" / "inference")
    b.save(prefix)
    x = rng.randn(5, 8).astype("float32")
    ref = TF.softmax(torch.relu(torch.from_numpy(x) @ torch.from_numpy(w1) + torch.from_numpy(b1))
                     @ torch.from_numpy(w2).T, -1).numpy()
    return prefix, x, ref


def test_mlp_static_and_predictor(tmp_path):
    prefix, x, ref = _mlp(tmp_path)
    assert pd.is_program_desc(prefix + ".pdmodel")
    paddle.enable_static()
    try:
        exe = paddle.static.Executor(paddle.CPUPlace())
        prog, feeds, fetches = paddle.static.load_inference_model(prefix, exe)
        assert feeds == ["x"] and fetches == ["prob"]
        (out,) = exe.run(prog, feed={"x": x}, fetch_list=fetches)
    finally:
        paddle.disable_static()
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-6)
    from paddlepaddle_amd import inference
    cfg = inference.Config(prefix + ".pdmodel", prefix + ".pdiparams")
    pred = inference.create_predictor(cfg)
    h = pred.get_input_handle(pred.get_input_names()[0])
    h.copy_from_cpu(x)
    pred.run()
    np.testing.assert_allclose(pred.get_output_handle(pred.get_output_names()[0]).copy_to_cpu(), ref, rtol=1e-5,
                               atol=1e-6)


def test_cnn_ops(tmp_path):
    rng = np.random.RandomState(1)
    w = rng.randn(6, 3, 3, 3).astype("float32") * 0.3
    g, beta = rng.rand(6).astype("float32") + 0.5, rng.randn(6).astype("float32")
    mean, var = rng.randn(6).astype("float32"), rng.rand(6).astype("float32") + 0.5
    fw, fb = rng.randn(6 * 4 * 4, 10).astype("float32"), rng.randn(10).astype("float32")
    b = pd.ProgramDescBuilder()
    b.feed("img", [-1, 3, 8, 8])
    for n, v in [("conv.w", w), ("bn.scale", g), ("bn.bias", beta), ("bn.mean", mean), ("bn.var", var),
                 ("fc.w", fw), ("fc.b", fb)]:
        b.param(n, v)
    b.op("conv2d", {"Input": ["img"], "Filter": ["conv.w"]}, {"Output": ["c"]}, strides=[1, 1], paddings=[1, 1],
         dilations=[1, 1], groups=1, padding_algorithm="EXPLICIT", data_format="NCHW")
    b.op("batch_norm", {"X": ["c"], "Scale": ["bn.scale"], "Bias": ["bn.bias"], "Mean": ["bn.mean"],
                        "Variance": ["bn.var"]}, {"Y": ["bn"], "MeanOut": ["bn.mean"], "VarianceOut": ["bn.var"]},
         epsilon=1e-5, is_test=True, data_layout="NCHW")
    b.op("relu", {"X": ["bn"]}, {"Out": ["r"]})
    b.op("pool2d", {"X": ["r"]}, {"Out": ["p"]}, pooling_type="max", ksize=[2, 2], strides=[2, 2],
         paddings=[0, 0], global_pooling=False, adaptive=False, ceil_mode=False, exclusive=True, data_format="NCHW",
         padding_algorithm="EXPLICIT")
    b.op("flatten_contiguous_range", {"X": ["p"]}, {"Out": ["f"], "XShape": ["f.xshape"]}, start_axis=1, stop_axis=-1)
    b.op("matmul_v2", {"X": ["f"], "Y": ["fc.w"]}, {"Out": ["m"]}, trans_x=False, trans_y=False)
    b.op("elementwise_add", {"X": ["m"], "Y": ["fc.b"]}, {"Out": ["logits"]}, axis=-1)
    b.op("pool2d", {"X": ["r"]}, {"Out": ["gap"]}, pooling_type="avg", ksize=[1, 1], global_pooling=True,
         adaptive=False, data_format="NCHW")
    b.fetch("logits")
    b.fetch("gap")
    prefix = str(tmp_path / "cnn")
    b.save(prefix)
    runner = pd.load(prefix, torch.device("cpu"))
    x = rng.randn(2, 3, 8, 8).astype("float32")
    logits, gap = runner.run({"img": paddle.to_tensor(x)})
    T = torch.from_numpy
    c = TF.conv2d(T(x), T(w), padding=1)
    r = torch.relu(TF.batch_norm(c, T(mean), T(var), T(g), T(beta), False, 0.0, 1e-5))
    ref = TF.max_pool2d(r, 2, 2).flatten(1) @ T(fw) + T(fb)
    np.testing.assert_allclose(logits.numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(gap.numpy(), r.mean((2, 3), keepdim=True).numpy(), rtol=1e-5, atol=1e-5)


def test_transformer_ops(tmp_path):
    rng = np.random.RandomState(2)
    B, S, H, NH = 2, 5, 8, 2
    emb = rng.randn(11, H).astype("float32")
    lw, lb = rng.rand(H).astype("float32") + 0.5, rng.randn(H).astype("float32")
    wq = rng.randn(H, 3 * H).astype("float32") * 0.3
    b = pd.ProgramDescBuilder()
    b.feed("ids", [-1, S], torch.int64)
    for n, v in [("emb", emb), ("ln.w", lw), ("ln.b", lb), ("wqkv", wq)]:
        b.param(n, v)
    b.op("lookup_table_v2", {"Ids": ["ids"], "W": ["emb"]}, {"Out": ["e"]}, padding_idx=-1)
    b.op("layer_norm", {"X": ["e"], "Scale": ["ln.w"], "Bias": ["ln.b"]}, {"Y": ["ln"], "Mean": ["m"],
                                                                           "Variance": ["v"]},
         epsilon=1e-5, begin_norm_axis=2)
    b.op("matmul_v2", {"X": ["ln"], "Y": ["wqkv"]}, {"Out": ["qkv"]}, trans_x=False, trans_y=False)
    b.op("split", {"X": ["qkv"]}, {"Out": ["q", "k", "v"]}, num=3, axis=-1, sections=[])
    for t in ("q", "k", "v"):
        b.op("reshape2", {"X": [t]}, {"Out": [t + "r"], "XShape": [t + "x"]}, shape=[0, 0, NH, H // NH])
        b.op("transpose2", {"X": [t + "r"]}, {"Out": [t + "t"], "XShape": [t + "tx"]}, axis=[0, 2, 1, 3])
    b.op("matmul_v2", {"X": ["qt"], "Y": ["kt"]}, {"Out": ["s"]}, trans_x=False, trans_y=True)
    b.op("scale", {"X": ["s"]}, {"Out": ["ss"]}, scale=float((H // NH) ** -0.5), bias=0.0, bias_after_scale=True)
    b.op("softmax", {"X": ["ss"]}, {"Out": ["a"]}, axis=-1)
    b.op("dropout", {"X": ["a"]}, {"Out": ["ad"], "Mask": ["mask"]}, dropout_prob=0.1, is_test=True,
         dropout_implementation="upscale_in_train")
    b.op("matmul_v2", {"X": ["ad"], "Y": ["vt"]}, {"Out": ["o"]}, trans_x=False, trans_y=False)
    b.op("transpose2", {"X": ["o"]}, {"Out": ["ot"], "XShape": ["otx"]}, axis=[0, 2, 1, 3])
    b.op("reshape2", {"X": ["ot"]}, {"Out": ["or"], "XShape": ["orx"]}, shape=[0, 0, -1])
    b.op("gelu", {"X": ["or"]}, {"Out": ["g"]}, approximate=False)
    b.op("slice", {"Input": ["g"]}, {"Out": ["first"]}, axes=[1], starts=[0], ends=[1], decrease_axis=[1])
    b.op("reduce_mean", {"X": ["g"]}, {"Out": ["pool"]}, dim=[1], keep_dim=False, reduce_all=False)
    b.op("concat", {"X": ["first", "pool"]}, {"Out": ["cat"]}, axis=-1)
    b.op("cast", {"X": ["cat"]}, {"Out": ["out"]}, in_dtype=5, out_dtype=6)
    b.fetch("out")
    prefix = str(tmp_path / "tfm")
    b.save(prefix)
    runner = pd.load(prefix, torch.device("cpu"))
    ids = rng.randint(0, 11, (B, S)).astype("int64")
    (out,) = runner.run([paddle.to_tensor(ids)])
    T = torch.from_numpy
    e = T(emb)[T(ids)]
    ln = TF.layer_norm(e, (H,), T(lw), T(lb), 1e-5)
    q, k, v = (ln @ T(wq)).split(H, -1)
    sh = lambda t: t.reshape(B, S, NH, H // NH).permute(0, 2, 1, 3)  # noqa: E731
    a = torch.softmax(sh(q) @ sh(k).transpose(-1, -2) * (H // NH) ** -0.5, -1)
    g = TF.gelu((a @ sh(v)).permute(0, 2, 1, 3).reshape(B, S, H))
    ref = torch.cat([g[:, 0], g.mean(1)], -1).double()
    assert out.dtype == paddle.float64
    np.testing.assert_allclose(out.numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)


def test_unmapped_operator_is_reported(tmp_path):
    b = pd.ProgramDescBuilder()
    b.feed("x", [2])
    b.op("some_custom_op", {"X": ["x"]}, {"Out": ["y"]})
    b.fetch("y")
    b.save(str(tmp_path / "bad"))
    with pytest.raises(NotImplementedError, match="some_custom_op"):
        pd.load(str(tmp_path / "bad"), torch.device("cpu"))


def _static_models():
    paddle.seed(4)
    x = paddle.static.data("x", [-1, 8], "float32")
    lin, ln = paddle.nn.Linear(8, 6), paddle.nn.LayerNorm(6)
    y = paddle.nn.functional.gelu(ln(lin(x)))
    y = paddle.nn.functional.sigmoid(y) * 2.0 - paddle.tanh(y) / 3.0
    y = paddle.reshape(paddle.transpose(paddle.unsqueeze(y, 1), [0, 2, 1]), [-1, 6])
    y = paddle.concat([y, y + 1.0], axis=1)
    y = paddle.nn.functional.softmax(paddle.matmul(y, y, transpose_y=True), axis=-1)
    im = paddle.static.data("im", [-1, 3, 8, 8], "float32")
    conv = paddle.nn.Conv2D(3, 4, 3, padding=1)
    bn = paddle.nn.BatchNorm2D(4)
    bn.eval()
    h = paddle.nn.functional.relu(bn(conv(im)))
    h = paddle.nn.functional.max_pool2d(h, 2, 2)
    h = paddle.nn.functional.avg_pool2d(h, 2)
    q = paddle.flatten(h, 1)
    return (x, im), (y, q)


def test_static_program_exports_to_reference_format(tmp_path):
    rng = np.random.RandomState(5)
    xs = {"x": rng.randn(3, 8).astype("float32"), "im": rng.randn(2, 3, 8, 8).astype("float32")}
    paddle.enable_static()
    try:
        main, startup = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, startup):
            feeds, fetches = _static_models()
        exe = paddle.static.Executor(paddle.CPUPlace())
        exe.run(startup)
        ref = exe.run(main, feed=xs, fetch_list=list(fetches))
        prefix = str(tmp_path / "exported")
        paddle.static.save_inference_model(prefix, list(feeds), list(fetches), exe, program=main,
                                           program_format="protobuf")
        assert pd.is_program_desc(prefix + ".pdmodel")
        prog, feed_names, fetch_names = paddle.static.load_inference_model(prefix, exe)
        assert feed_names == ["x", "im"]
        got = exe.run(prog, feed=xs, fetch_list=fetch_names)
    finally:
        paddle.disable_static()
    types = {o["type"] for o in prog.program.ops}
    assert {"matmul_v2", "layer_norm", "gelu", "conv2d", "batch_norm", "pool2d", "transpose2", "reshape2",
            "concat", "softmax", "scale", "flatten_contiguous_range"} <= types
    for a, b in zip(ref, got):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_reference_program_runs_on_gpu(tmp_path):
    prefix, x, ref = _mlp(tmp_path)
    runner = pd.load(prefix, torch.device("cuda:0"))
    (out,) = runner.run({"x": paddle.Tensor(torch.from_numpy(x).cuda())})
    assert out._t.is_cuda
    np.testing.assert_allclose(out.numpy(), ref, rtol=1e-4, atol=1e-5)
