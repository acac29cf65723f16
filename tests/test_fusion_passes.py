"""Fusion / auto-parallel program passes of distributed/passes/fusion_passes.py on traced static programs:
each rewrite is checked for the node it produces and for unchanged results (forward outputs, trained parameters)
against the unrewritten program. Reference: distributed/passes/cpp_pass.py:76-141,
auto_parallel_master_grad.py:84, auto_parallel_quantization.py:48, framework/ir.py:56 (build strategy)."""
import os

import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle  # noqa: E402
from paddlepaddle_amd.distributed.passes import new_pass  # noqa: E402


@pytest.fixture(autouse=True)
def _static(monkeypatch):
    # set per test, not at import: a module-level setting leaks into every process a later GPU test starts
    monkeypatch.setenv("PADDLE_AMD_FORCE_CPU", "1")
    paddle.enable_static()
    yield
    paddle.disable_static()


def _names(prog):
    return [n.name.rsplit(":", 1)[-1] for n in prog.nodes]


def _run(prog, feed, fetch):
    exe = paddle.static.Executor(paddle.CPUPlace())
    return [np.array(v) for v in exe.run(prog, feed=feed, fetch_list=fetch)]


def _ffn_program(fold_first):
    main, start = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, start):
        paddle.seed(3)
        x = paddle.static.data("x", [4, 8, 16], "float32")
        l1, l2 = paddle.nn.Linear(16, 64), paddle.nn.Linear(64, 16)
        y = l2(paddle.nn.functional.gelu(l1(x), approximate=True))
        out = y + x
    if fold_first:
        new_pass("fuse_gemm_epilogue").apply(main, None)
    return main, out


@pytest.mark.parametrize("fold_first", [True, False])
def test_fused_feedforward_rewrites_fc_gelu_fc(fold_first):
    main, out = _ffn_program(fold_first)
    feed = {"x": np.random.RandomState(0).randn(4, 8, 16).astype("float32")}
    ref, = _run(main, feed, [out])
    ctx = new_pass("fused_feedforward").apply(main, None)
    assert ctx.get_attr("fused_feedforward.fused") == 1
    assert "ffn_gelu" in _names(main) and "gelu" not in _names(main)
    got, = _run(main, feed, [out])
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)


def test_fused_attention_folds_residual_into_out_projection():
    main, out = _ffn_program(True)
    feed = {"x": np.random.RandomState(1).randn(4, 8, 16).astype("float32")}
    ref, = _run(main, feed, [out])
    ctx = new_pass("fused_attention").apply(main, None)
    assert ctx.get_attr("fused_attention.fused") == 1 and "add" not in _names(main)
    lin = [n for n in main.nodes if n.name.endswith("fused_linear")][-1]
    assert len(lin.args) == 6 and lin.args[5] is not None  # residual= operand
    got, = _run(main, feed, [out])
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("with_mask", [False, True])
def test_fuse_dot_product_attention(with_mask):
    main, start = paddle.static.Program(), paddle.static.Program()
    B, H, S, D = 2, 4, 16, 8
    with paddle.static.program_guard(main, start):
        q = paddle.static.data("q", [B, H, S, D], "float32")
        k = paddle.static.data("k", [B, H, S, D], "float32")
        v = paddle.static.data("v", [B, H, S, D], "float32")
        s = paddle.matmul(q, k, transpose_y=True) * (D ** -0.5)
        if with_mask:
            m = paddle.static.data("m", [B, 1, S, S], "float32")
            s = s + m
        o = paddle.matmul(paddle.nn.functional.softmax(s, axis=-1), v)
    rs = np.random.RandomState(2)
    feed = {n: rs.randn(B, H, S, D).astype("float32") for n in "qkv"}
    if with_mask:
        feed["m"] = np.where(rs.rand(B, 1, S, S) > 0.2, 0.0, -1e4).astype("float32")
    ref, = _run(main, feed, [o])
    ctx = new_pass("fuse_dot_product_attention").apply(main, None)
    assert ctx.get_attr("fuse_dot_product_attention.fused") == 1
    assert _names(main) == ["attention_bhsd"]
    got, = _run(main, feed, [o])
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)


def _train_program(opt_fn, dtype="float32", groups=False):
    main, start = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, start):
        paddle.seed(5)
        x = paddle.static.data("x", [8, 16], dtype)
        y = paddle.static.data("y", [8, 4], dtype)
        l1, l2 = paddle.nn.Linear(16, 32), paddle.nn.Linear(32, 4)
        if dtype != "float32":
            for p in list(l1.parameters()) + list(l2.parameters()):
                p._t.data = p._t.data.to(torch.bfloat16)
        loss = paddle.mean((l2(paddle.nn.functional.relu(l1(x))) - y) ** 2)
        params = [{"params": l1.parameters()}, {"params": l2.parameters()}] if groups else None
        opt = opt_fn(params)
        opt.minimize(loss)
    return main, loss


def _data(dtype="float32"):
    rs = np.random.RandomState(7)
    x, y = rs.randn(8, 16), rs.randn(8, 4)
    if dtype == "float32":
        return {"x": x.astype("float32"), "y": y.astype("float32")}
    return {"x": torch.tensor(x).bfloat16(), "y": torch.tensor(y).bfloat16()}


@pytest.mark.parametrize("name", ["fuse_adamw", "fuse_optimizer"])
def test_fuse_optimizer_merges_equal_groups(name):
    res = []
    for apply in (False, True):
        main, loss = _train_program(lambda ps: paddle.optimizer.AdamW(0.01, parameters=ps), groups=True)
        if apply:
            ctx = new_pass(name).apply(main, None)
            assert ctx.get_attr(f"{name}.merged_groups") == 1
            assert len(main._optimize[0]._param_groups) == 1
        res.append([float(_run(main, _data(), [loss])[0]) for _ in range(3)])
    np.testing.assert_allclose(res[1], res[0], rtol=1e-6)


def test_master_grad_accumulates_fp32_across_gradient_merge():
    main, loss = _train_program(lambda ps: paddle.optimizer.SGD(0.5), dtype="bfloat16")
    new_pass("auto_parallel_gradient_merge", {"k_steps": 2, "avg": False}).apply(main, None)
    new_pass("auto_parallel_master_grad_pass").apply(main, None)
    params = main.all_parameters()
    w0 = [p._t.detach().float().clone() for p in params]
    _run(main, _data("bf16"), [loss])
    assert all(p._t.grad is None for p in params)  # released into the fp32 main gradients
    assert all(g.dtype == torch.float32 for g in main._pa_main_grads.values()) and main._pa_main_grads
    mg = {k: v.clone() for k, v in main._pa_main_grads.items()}
    _run(main, _data("bf16"), [loss])
    # the update used 2 x the fp32 per-micro-step gradient, rounded once to bf16
    for p, w in zip(params, w0):
        g = (2 * mg[id(p)]).to(torch.bfloat16).float()
        np.testing.assert_allclose(p._t.detach().float().numpy(), (w - 0.5 * g).to(torch.bfloat16).float().numpy(),
                                   rtol=1e-2, atol=1e-2)


def test_quantization_pass_inserts_fake_quant():
    main, loss = _train_program(lambda ps: paddle.optimizer.SGD(0.1))
    ctx = new_pass("auto_parallel_quantization", {"weight_bits": 8, "activation_bits": 8}).apply(main, None)
    assert ctx.get_attr("auto_parallel_quantization.quantized") == 2
    names = _names(main)
    assert names.count("qat_fake_quant_act") == 2 and names.count("qat_fake_quant_weight") == 2
    losses = [float(_run(main, _data(), [loss])[0]) for _ in range(4)]
    assert losses[-1] < losses[0]


def test_build_strategy_applies_fusion_passes_on_first_run():
    main, out = _ffn_program(False)
    feed = {"x": np.random.RandomState(4).randn(4, 8, 16).astype("float32")}
    ref, = _run(main, feed, [out])
    bs = paddle.static.BuildStrategy()
    bs.fuse_gemm_epilogue = True
    bs.fused_feedforward = True
    bs.fused_attention = True
    cp = paddle.static.CompiledProgram(main, build_strategy=bs)
    got, = _run(cp, feed, [out])
    assert set(cp._applied) == {"fuse_gemm_epilogue", "fused_feedforward", "fused_attention"}
    assert "ffn_gelu" in _names(main)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)


def _conv_program(kind):
    main, start = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, start):
        paddle.seed(7)
        x = paddle.static.data("x", [2, 6, 6, 8], "float32")
        if kind == "dw":  # relu -> depthwise conv on a channels-last layer, and on an NCHW one
            y = paddle.nn.Conv2D(8, 8, 3, padding=1, groups=8, data_format="NHWC")(paddle.nn.functional.relu(x))
            z = paddle.transpose(y, [0, 3, 1, 2])
            out = paddle.nn.Conv2D(8, 8, 3, padding=1, groups=8, bias_attr=False)(paddle.nn.functional.relu(z))
        else:  # conv -> BN -> + x -> relu, then conv -> BN -> relu (the two ResNet unit forms)
            c1 = paddle.nn.Conv2D(8, 8, 3, padding=1, data_format="NHWC", bias_attr=False)
            b1 = paddle.nn.BatchNorm2D(8, data_format="NHWC")
            h = paddle.nn.functional.relu(b1(c1(x)) + x)
            c2 = paddle.nn.Conv2D(8, 8, 1, data_format="NHWC", bias_attr=False)
            b2 = paddle.nn.BatchNorm2D(8, data_format="NHWC")
            out = paddle.nn.functional.relu(b2(c2(h)))
        loss = (out * out).mean()
        opt = paddle.optimizer.SGD(0.1)
        opt.minimize(loss)
    return main, loss


@pytest.mark.parametrize("kind", ["dw", "resunit"])
def test_conv_fusion_passes_match_unfused(kind):
    """fuse_relu_depthwise_conv (relu folded into the depthwise conv) and fuse_resunit (conv -> BN (+ add) (+ relu)
    as one conv_bn_unit node, after fuse_bn_act / fuse_bn_add_act): same losses over training steps as the
    unrewritten program (reference cpp_pass.py:63 / :171)."""
    feed = {"x": np.random.RandomState(3).randn(2, 6, 6, 8).astype("float32")}
    losses = []
    for fuse in (False, True):
        main, loss = _conv_program(kind)
        if fuse:
            if kind == "dw":
                ctx = new_pass("fuse_relu_depthwise_conv").apply(main, None)
                assert ctx.get_attr("fuse_relu_depthwise_conv.fused") == 2
                assert _names(main).count("relu_depthwise_conv2d") == 2 and "relu" not in _names(main)
            else:
                new_pass("fuse_bn_add_act").apply(main, None)
                new_pass("fuse_bn_act").apply(main, None)
                ctx = new_pass("fuse_resunit").apply(main, None)
                assert ctx.get_attr("fuse_resunit.fused") == 2
                assert _names(main).count("conv_bn_unit") == 2
                assert "conv2d" not in _names(main) and "batch_norm_act_nhwc" not in _names(main)
        losses.append([float(_run(main, feed, [loss])[0]) for _ in range(3)])
    np.testing.assert_allclose(losses[1], losses[0], rtol=1e-5, atol=1e-6)
    assert losses[0][-1] < losses[0][0]


def _promo_worker(rank, world, port, q):
    import sys
    from test_distributed_cpu import _setup
    pd = _setup(rank, world, port)
    from paddlepaddle_amd.distributed.passes import new_pass as np_
    out = []
    for promote in (False, True):
        pd.enable_static()
        main, start = pd.static.Program(), pd.static.Program()
        with pd.static.program_guard(main, start):
            pd.seed(11 + rank)  # row-parallel: each rank its own slice of W
            x = pd.static.data("x", [8, 16], "float32")
            w = pd.create_parameter([16, 8], "float32")
            pd.seed(5)  # the bias is replicated
            b = pd.create_parameter([8], "float32", is_bias=True,
                                    default_initializer=pd.nn.initializer.Normal(0.0, 1.0))
            h = pd.matmul(x, w)
            pd.distributed.all_reduce(h)
            y = h + b
            loss = (y * y).mean()
            pd.optimizer.SGD(0.05).minimize(loss)
        if promote:
            ctx = np_("auto_parallel_fused_linear_promotion").apply(main, None)
            names = [n.name.rsplit(":", 1)[-1] for n in main.nodes]
            assert ctx.get_attr("auto_parallel_fused_linear_promotion.promoted") == 1
            assert ("fused_linear" in names) == (rank == 0) and "add" not in names, names
        exe = pd.static.Executor(pd.CPUPlace())
        xs = np.random.RandomState(rank).randn(8, 16).astype("float32")
        out.append([float(exe.run(main, feed={"x": xs}, fetch_list=[loss])[0]) for _ in range(3)])
        pd.disable_static()
    q.put((rank, out))


def test_fused_linear_promotion_row_parallel_gloo(monkeypatch):
    """auto_parallel_fused_linear_promotion (reference auto_parallel_fused_linear_promotion.py:130): matmul ->
    all_reduce -> + bias becomes fused_linear(x, W, b) on the group's first rank (the plain matmul elsewhere) with
    the add removed; 2 gloo ranks train with the same losses as the unpromoted program."""
    from test_distributed_cpu import _spawn
    for rank, (ref, got) in _spawn(_promo_worker, world=2):
        np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)
        assert ref[-1] < ref[0]


def test_supplement_explicit_dependencies_orders_collectives():
    """auto_parallel_supplement_explicit_dependencies: the collectives are chained in program order for the
    scheduler (static/program.py build_plan honours the chain; a reversed chain reverses their issue order)."""
    from paddlepaddle_amd.distributed.collective import _static_comm
    from paddlepaddle_amd.static import program as P
    main, start = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, start):
        x = paddle.static.data("x", [4, 4], "float32")
        ts = [x * float(i + 2) for i in range(3)]
        for t in ts:
            assert _static_comm(t, "all_reduce", lambda v: None)
        out = ts[0] + ts[1] + ts[2]
    ctx = new_pass("auto_parallel_supplement_explicit_dependencies").apply(main, None)
    assert ctx.get_attr("auto_parallel_supplement_explicit_dependencies.chained") == 2
    comm = [n for n in main.nodes if n.kind == "comm"]
    slot = main._slot_of[id(out._t)]
    order = [main.nodes[i] for i in P.build_plan(main, [slot]).order if main.nodes[i].kind == "comm"]
    assert order == comm
    main._pa_comm_chain = main._pa_comm_chain[::-1]
    order = [main.nodes[i] for i in P.build_plan(main, [slot]).order if main.nodes[i].kind == "comm"]
    assert order == comm[::-1]


def test_auto_parallel_registry_passes():
    """auto_parallel_gradient_merge_pass (the reference's name), auto_parallel_sequence_parallel_optimization (marks
    the program for the engine's reduce-scatter reshards) and auto_parallel_pipeline (the job list of the
    configured schedule, VPP chunks included)."""
    from paddlepaddle_amd.distributed.passes.pipeline_scheduler import job_pairs
    main, out = _ffn_program(False)
    with paddle.static.program_guard(main):
        paddle.optimizer.SGD(0.1).minimize(out.mean())
    new_pass("auto_parallel_gradient_merge_pass", {"k_steps": 4, "avg": True}).apply(main, None)
    assert main._grad_merge == (4, True)
    ctx = new_pass("auto_parallel_sequence_parallel_optimization").apply(main, None)
    assert main._pa_sp_opt and ctx.get_attr("auto_parallel_sequence_parallel_optimization.enabled")
    ctx = new_pass("auto_parallel_pipeline", {"schedule_mode": "1F1B", "num_micro_batches": 4, "pp_stage": 0,
                                              "pp_degree": 2}).apply(main, None)
    assert ctx.get_attr("auto_parallel_pipeline.mode") == "1F1B"
    assert job_pairs(ctx.get_attr("auto_parallel_pipeline.job_list")) == [
        ("F", 0), ("F", 1), ("B", 0), ("F", 2), ("B", 1), ("F", 3), ("B", 2), ("B", 3)]
    ctx = new_pass("auto_parallel_pipeline", {"schedule_mode": "VPP", "num_micro_batches": 4, "pp_stage": 1,
                                              "pp_degree": 2, "vpp_degree": 2}).apply(main, None)
    jobs = ctx.get_attr("auto_parallel_pipeline.job_list")
    assert {j.chunk_id() for j in jobs if j.type() == "forward"} == {0, 1}
