"""The native program interpreter (csrc/interpreter/interpreter.cpp) runs a saved PIR program on this
framework's hand-written kernels: a GPT program exported with save_inference_model(program_format="pir") and
loaded by the inference Predictor executes its matmuls / fused linears on the MFMA GEMM, layer norms on the row
kernel and attention on the flash-attention forward (reference: new_executor/program_interpreter.cc:142,231)."""
import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle
from paddlepaddle_amd.framework import native_interp as NI

pytestmark = pytest.mark.skipif(not NI.available(), reason="_C_interp not built")


def _export_gpt(tmp_path, cfg, ids, dtype="float32"):
    from paddlepaddle_amd.models.gpt import GPTForPretraining
    paddle.seed(3)
    paddle.set_default_dtype(dtype)
    try:
        m = GPTForPretraining(cfg)
    finally:
        paddle.set_default_dtype("float32")
    m.eval()
    ref = m(paddle.to_tensor(ids)).astype("float32").numpy()
    paddle.enable_static()
    try:
        main, start = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, start):
            x = paddle.static.data("ids", list(ids.shape), "int64")
            logits = m(x)
        exe = paddle.static.Executor(paddle.CPUPlace())
        prefix = str(tmp_path / "gpt")
        paddle.static.save_inference_model(prefix, [x], [logits], exe, program=main, program_format="pir")
    finally:
        paddle.disable_static()
    return prefix, ref


def test_gpt_pir_program_runs_on_the_native_interpreter_with_fused_linears(tmp_path):
    from paddlepaddle_amd.models.gpt import GPTConfig
    from paddlepaddle_amd.framework import pir_json
    cfg = GPTConfig.tiny(hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    ids = np.random.RandomState(0).randint(0, cfg.vocab_size, (2, 16)).astype("int64")
    prefix, ref = _export_gpt(tmp_path, cfg, ids)
    cfgi = paddle.inference.Config(prefix + ".json", prefix + ".pdiparams")
    cfgi.disable_gpu()
    pred = paddle.inference.create_predictor(cfgi)
    assert type(pred._runner).__name__ == "NativeRunner"
    np.testing.assert_allclose(pred.run([ids])[0].numpy(), ref, rtol=1e-4, atol=1e-4)
    # matmul + bias (+ GELU) pairs of every block became one fused_linear instruction
    prog = pir_json.PirProgram(__import__("json").load(open(prefix + ".json")))
    names = [o[0] for o in NI._fuse_linear(prog.ops)]
    assert names.count("pd_op.fused_linear") == 4 * cfg.num_hidden_layers
    assert "pd_op.flash_attn_qkvpacked" in names and "pd_op.gelu" not in names


@pytest.mark.gpu
def test_gpt_pir_predictor_launches_the_hip_kernels(tmp_path):
    from paddlepaddle_amd.models.gpt import GPTConfig
    paddle.set_device("gpu:0")
    cfg = GPTConfig.tiny(hidden_size=256, num_attention_heads=2, intermediate_size=1024, hidden_dropout_prob=0.0,
                         attention_probs_dropout_prob=0.0)
    ids = np.random.RandomState(1).randint(0, cfg.vocab_size, (2, 128)).astype("int64")
    prefix, ref = _export_gpt(tmp_path, cfg, ids, dtype="bfloat16")
    cfgi = paddle.inference.Config(prefix + ".json", prefix + ".pdiparams")
    cfgi.enable_use_gpu(100, 0)
    pred = paddle.inference.create_predictor(cfgi)
    assert type(pred._runner).__name__ == "NativeRunner"
    NI.reset_kernel_calls()
    out = pred.run([ids])[0].astype("float32").numpy()
    torch.cuda.synchronize()
    calls = NI.kernel_calls()
    L = cfg.num_hidden_layers
    assert calls.get("gemm", 0) >= 4 * L + 1, calls        # QKV / out-proj / FFN x2 per block + tied LM head
    assert calls.get("layer_norm", 0) == 2 * L + 1, calls
    assert calls.get("flash_attn", 0) == L, calls
    scale = np.abs(ref).max()
    assert np.abs(out - ref).max() / scale < 3e-2


def _one_op_interp(op, attrs, device):
    m = NI._module()
    it = m.Interpreter(2, str(device))
    it.add(op, [0], [1], attrs)
    it.finalize([], [1])
    return it


@pytest.mark.gpu
@pytest.mark.parametrize("cols", [10, 77, 64, 1000])
def test_interp_softmax_guards_rows_the_kernel_cannot_take(cols):
    # softmax.hip needs cols % 8 == 0 and 16-byte rows: 10 / 77 / 1000-wide rows must fall back to
    # ATen, multiples of 8 run the HIP kernel; every row is checked against the fp32 softmax
    dev = torch.device("cuda:0")
    x = torch.randn(33, cols, device=dev, dtype=torch.float32) * 3
    it = _one_op_interp("softmax", {"axis": -1}, dev)
    NI.reset_kernel_calls()
    y = it.run([(0, x)])[0]
    torch.cuda.synchronize()
    ref = torch.softmax(x.double(), -1).float()
    assert torch.allclose(y, ref, atol=1e-5, rtol=1e-4)
    launched = NI.kernel_calls().get("softmax", 0)
    assert launched == (1 if cols % 8 == 0 else 0)


@pytest.mark.gpu
def test_interp_softmax_misaligned_view_falls_back():
    dev = torch.device("cuda:0")
    base = torch.randn(17 * 64 + 2, device=dev)
    x = base[2:].view(17, 64)  # fp32 start 8 bytes past a 16-byte boundary
    it = _one_op_interp("softmax", {"axis": -1}, dev)
    NI.reset_kernel_calls()
    y = it.run([(0, x)])[0]
    torch.cuda.synchronize()
    assert torch.allclose(y, torch.softmax(x, -1), atol=1e-6)
    assert NI.kernel_calls().get("softmax", 0) == 0
