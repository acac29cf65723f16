"""PIR program JSON (Paddle 3.x model format): a static program saved by save_inference_model is written in the
reference schema (paddle/fluid/pir/serialize_deserialize: base_code / regions / blocks / ops, compressed dialect
ids, "p" parameter ops, t_dtensor types, a_* attributes, mutable attributes as full / full_int_array operands)
and loads back through the PIR runner with the same outputs. Parity with the reference's own reader is unpinned:
no reference-exported .json model ships in the reference tree; the schema checks below follow schema.h /
ir_serialize.cc / serialize_utils.h key for key."""
import json
import os

import numpy as np
import pytest

import paddlepaddle_amd as paddle
from paddlepaddle_amd.framework import pir_json as pir

from test_program_desc import _static_models


def _save(tmp_path, fmt="json"):
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
        prefix = str(tmp_path / "m")
        paddle.static.save_inference_model(prefix, list(feeds), list(fetches), exe, program=main,
                                           program_format=fmt)
    finally:
        paddle.disable_static()
    return prefix, xs, ref


def test_default_save_writes_reference_pir_json(tmp_path):
    prefix, xs, ref = _save(tmp_path)
    assert os.path.exists(prefix + ".pdmodel") and os.path.exists(prefix + ".json")
    with open(prefix + ".json") as f:
        d = json.load(f)
    assert d["base_code"] == {"magic": "pir", "version": 1, "trainable": False}
    region = d["program"]["regions"][0]
    assert region["#"] == "region_0" and region["blocks"][0]["#"] == "block_0"
    ops = region["blocks"][0]["ops"]
    names = [o["#"] for o in ops]
    # dialect-compressed op names, parameter ops, feeds first, fetches last
    assert "p" in names and "1.data" in names and names[-1] == "1.fetch"
    assert {"1.matmul", "1.layer_norm", "1.gelu", "1.conv2d", "1.batch_norm_", "1.pool2d", "1.reshape",
            "1.transpose", "1.concat", "1.softmax", "1.scale", "1.flatten", "1.full_int_array", "0.combine"} <= set(names)
    # value ids: results count up from 1 and every operand refers to an earlier result
    seen = set()
    for o in ops:
        for i in o.get("I", []):
            assert i["%"] in seen
        outs = [o["O"]] if isinstance(o["O"], dict) else o["O"]
        for r in outs:
            assert r["%"] not in seen and r["%"] >= 1
            seen.add(r["%"])
            assert r["TT"]["#"] in ("0.t_dtensor", "0.t_vec")
    p = next(o for o in ops if o["#"] == "p")
    assert len(p["A"]) == 4 and isinstance(p["A"][3], str)
    data = next(o for o in ops if o["#"] == "1.data")
    attrs = {a["N"]: a["AT"] for a in data["A"]}
    assert attrs["name"] == {"#": "0.a_str", "D": "x"} and attrs["dtype"] == {"#": "1.a_dtype", "D": "float32"}
    assert attrs["shape"]["#"] == "1.a_intarray" and attrs["place"]["#"] == "1.a_place"
    # mutable attributes are operands: reshape (x, shape), pool2d (x, kernel_size), concat (combine, axis)
    for op, n in (("1.reshape", 2), ("1.pool2d", 2), ("1.concat", 2), ("1.scale", 2)):
        assert all(len(o["I"]) == n for o in ops if o["#"] == op), op
    mm = next(o for o in ops if o["#"] == "1.matmul")
    assert {a["N"] for a in mm["A"]} == {"transpose_x", "transpose_y"}


def test_pir_json_round_trip_runs(tmp_path):
    prefix, xs, ref = _save(tmp_path, fmt="pir")
    assert not os.path.exists(prefix + ".pdmodel") and pir.is_pir_json(prefix + ".json")
    paddle.enable_static()
    try:
        exe = paddle.static.Executor(paddle.CPUPlace())
        prog, feed_names, fetch_names = paddle.static.load_inference_model(prefix, exe)
        from paddlepaddle_amd.framework.native_interp import NativeRunner
        assert isinstance(prog, (pir.PirRunner, NativeRunner)) and feed_names == ["x", "im"]
        got = exe.run(prog, feed=xs, fetch_list=fetch_names)
    finally:
        paddle.disable_static()
    for a, b in zip(ref, got):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-5)


def test_predictor_reads_pir_json(tmp_path):
    prefix, xs, ref = _save(tmp_path, fmt="pir")
    from paddlepaddle_amd import inference
    cfg = inference.Config(prefix + ".json", prefix + ".pdiparams")
    pred = inference.create_predictor(cfg)
    for n in pred.get_input_names():
        pred.get_input_handle(n).copy_from_cpu(xs[n])
    pred.run()
    outs = [pred.get_output_handle(n).copy_to_cpu() for n in pred.get_output_names()]
    for a, b in zip(ref, outs):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-5)


def test_attribute_and_type_codec():
    assert pir.a_f32(float("nan")) == {"#": "0.a_f32", "VD": "NaN"}
    assert pir.a_f64(float("-inf")) == {"#": "0.a_f64", "VD": "-INF"}
    for a in (pir.a_bool(True), pir.a_i32(3), pir.a_i64(1 << 40), pir.a_str("s"), pir.a_intarray([1, -1]),
              pir.a_array([pir.a_i32(1), pir.a_i32(2)]), pir.a_dtype("bfloat16")):
        pir.decode_attr(a)
    assert pir.decode_attr(pir.a_array([pir.a_i32(1), pir.a_i32(2)])) == [1, 2]
    assert pir.decode_attr({"#": "1.a_scalar", "D": ["float32", 2.5]}) == 2.5
    assert pir.decode_type(pir.dtensor("bfloat16", [2, -1])) == ("bfloat16", [2, -1])
    with pytest.raises(ValueError):
        pir.PirProgram({"program": {}})


def test_native_interpreter_matches_python_replay(tmp_path):
    """The C++ interpreter (csrc/interpreter, instruction list + last-use release) runs the saved PIR program
    with the Python replay's outputs; mutable attributes are folded, intermediates are released."""
    from paddlepaddle_amd.framework import native_interp as ni
    if not ni.available():
        pytest.skip("_C_interp not built")
    prefix, xs, ref = _save(tmp_path, fmt="pir")
    paddle.set_flags({"FLAGS_pir_native_interpreter": True})
    native = pir.load(prefix)
    assert isinstance(native, ni.NativeRunner)
    paddle.set_flags({"FLAGS_pir_native_interpreter": False})
    try:
        py = pir.load(prefix)
    finally:
        paddle.set_flags({"FLAGS_pir_native_interpreter": True})
    assert isinstance(py, pir.PirRunner)
    feeds = {k: paddle.to_tensor(v) for k, v in xs.items()}
    a = [t.numpy() for t in native.run(feeds)]
    b = [t.numpy() for t in py.run(feeds)]
    for x, y, r in zip(a, b, ref):
        np.testing.assert_allclose(x, y, rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(x, r, rtol=1e-5, atol=1e-5)
    it = native.interp
    assert it.num_instructions > 10 and it.releases > 0 and it.peak_live < it.num_instructions


def test_pir_flash_attn_with_attn_mask_replays():
    """pd_op.flash_attn with its attn_mask input (5th operand) replays through the masked attention kernel."""
    import torch
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.framework import pir_json as PJ
    g = torch.Generator().manual_seed(0)
    q, k, v = (torch.randn(2, 5, 2, 8, generator=g) for _ in range(3))
    m = torch.randn(2, 1, 5, 5, generator=g)
    out = PJ._flash_attn([paddle.to_tensor(q), paddle.to_tensor(k), paddle.to_tensor(v), None, paddle.to_tensor(m)],
                         {"causal": False})[0]
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) / 8 ** 0.5 + m
    ref = torch.einsum("bhqk,bkhd->bqhd", torch.softmax(s, -1), v)
    assert (out._t - ref).abs().max().item() < 1e-5


def _cf_program(tmp_path):
    """y = x; i = 0; while i < n: y = y * 2 + 1 (per step), i += 1; out = (sum(y) > 0) ? y - 1 : y * 3
    written with the reference's control-flow ops (pd_op.while / pd_op.if with sub-blocks ending in cf.yield)."""
    w = pir.PirWriter()
    x = w.data("x", [4], "float32")
    n = w.data("n", [1], "int64")
    i0 = w.full([1], 0, "int64")
    c0 = w.op("less_than", [i0, n], {}, [pir.dtensor("bool", [1])])[0]
    one = w.full([1], 1.0)  # defined outside the loop, read inside it and after it
    i_arg, y_arg = w.block([w.types[i0], w.types[x]])
    two = w.full([1], 2.0)
    y2 = w.op("multiply", [y_arg, two], {}, [w.types[x]])[0]
    y3 = w.op("add", [y2, one], {}, [w.types[x]])[0]
    i1 = w.op("increment_", [i_arg], {"value": pir.a_f32(1.0)}, [w.types[i0]])[0]
    c1 = w.op("less_than", [i1, n], {}, [pir.dtensor("bool", [1])])[0]
    body = w.end_block([c1, i1, y3])
    i_out, y_out = w.while_(c0, [i0, x], body)
    s = w.op("sum", [y_out], {"axis": pir.a_intarray([]), "keepdim": pir.a_bool(False),
                              "dtype": pir.a_dtype("float32")}, [pir.dtensor("float32", [])])[0]
    zero = w.full([], 0.0)
    pos = w.op("greater_than", [s, zero], {}, [pir.dtensor("bool", [])])[0]
    w.block()
    t = w.op("subtract", [y_out, one], {}, [w.types[x]])[0]
    tb = w.end_block([t])
    w.block()
    three = w.full([1], 3.0)
    f = w.op("multiply", [y_out, three], {}, [w.types[x]])[0]
    fb = w.end_block([f])
    out = w.if_(pos, tb, fb, [w.types[x]])[0]
    w.fetch(out, "out", 0)
    w.fetch(i_out, "steps", 1)
    prefix = str(tmp_path / "cf")
    w.save(prefix)
    return prefix


def _cf_expect(x, n):
    y = x.copy()
    for _ in range(n):
        y = y * 2 + 1
    return (y - 1 if y.sum() > 0 else y * 3), n


@pytest.mark.parametrize("native", [True, False])
def test_pir_control_flow_if_while(tmp_path, native):
    """pd_op.while / pd_op.if with sub-blocks (reference control_flow_op.cc IfOp / WhileOp, serialized as op
    regions): the Python replay and the native interpreter (branches + block-argument moves in C++, loop-aware
    last-use release) give the same results as numpy, for loops that run 0, 1 and 3 times and both branches."""
    from paddlepaddle_amd.framework import native_interp
    prefix = _cf_program(tmp_path)
    paddle.set_flags({"FLAGS_pir_native_interpreter": native})
    try:
        runner = pir.load(prefix, device="cpu")
    finally:
        paddle.set_flags({"FLAGS_pir_native_interpreter": True})
    assert isinstance(runner, native_interp.NativeRunner) == (native and native_interp.available())
    for xs, n in (([1.0, -2.0, 3.0, 0.5], 3), ([-5.0, -1.0, 0.0, 1.0], 0), ([-5.0, -1.0, 0.0, 1.0], 1)):
        x = np.array(xs, "float32")
        out, steps = runner.run({"x": x, "n": np.array([n], "int64")})
        ey, en = _cf_expect(x, n)
        np.testing.assert_allclose(np.asarray(out.numpy()), ey, rtol=1e-6)
        assert int(np.asarray(steps.numpy()).reshape(-1)[0]) == en


@pytest.mark.gpu
def test_pir_control_flow_native_interpreter_gpu(tmp_path):
    """The same while / if program on the GPU through the native interpreter (device-resident loop state; the
    branch conditions are read back per iteration, as the reference's WhileInstruction does)."""
    from paddlepaddle_amd.framework import native_interp
    import torch
    prefix = _cf_program(tmp_path)
    runner = pir.load(prefix, device=torch.device("cuda:0"))
    assert isinstance(runner, native_interp.NativeRunner)
    for xs, n in (([1.0, -2.0, 3.0, 0.5], 3), ([-5.0, -1.0, 0.0, 1.0], 1)):
        x = np.array(xs, "float32")
        out, steps = runner.run({"x": x, "n": np.array([n], "int64")})
        assert out._t.is_cuda
        ey, en = _cf_expect(x, n)
        np.testing.assert_allclose(out._t.cpu().numpy(), ey, rtol=1e-6)
        assert int(steps._t.cpu().reshape(-1)[0]) == en
