"""CPU tests of the API-completion additions: static control flow, EMA, auc, distributed/fleet helpers,
fp8 gemm fallback, forward_grad, block_diag, module aliases, reference __all__ coverage."""
import ast
import importlib
import os

import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle

REF = "/root/reference/python/paddle"


def test_static_control_flow_dygraph():
    from paddlepaddle_amd.static import nn as snn
    x = paddle.to_tensor([3.0])
    assert float(snn.cond(x > 2, lambda: x * 2, lambda: x - 1)) == 6.0
    assert int(snn.while_loop(lambda i: i < 5, lambda i: [i + 2], [paddle.to_tensor(0)])[0]) == 6
    assert float(snn.switch_case(paddle.to_tensor(1), {0: lambda: x, 1: lambda: x * 10})) == 30.0
    assert float(snn.case([(x < 0, lambda: x), (x > 1, lambda: x + 100)], default=lambda: x * 0)) == 103.0


def test_static_cond_select_in_meta_mode():
    from paddlepaddle_amd.static import control_flow as cf
    from paddlepaddle_amd.framework.tensor import _wrap
    pred = _wrap(torch.empty((), dtype=torch.bool, device="meta"))
    a = _wrap(torch.empty(3, device="meta"))
    out = cf.cond(pred, lambda: a * 2, lambda: a + 1)
    assert out._t.device.type == "meta" and list(out._t.shape) == [3]


def test_ema_apply_restore():
    lin = paddle.nn.Linear(2, 2)
    w0 = lin.weight.numpy().copy()
    ema = paddle.static.ExponentialMovingAverage(0.5, parameters=[lin.weight])
    ema.update()
    with torch.no_grad():
        lin.weight._t.add_(1.0)
    ema.update()
    with ema.apply():
        np.testing.assert_allclose(lin.weight.numpy(), w0 + 0.5, rtol=1e-6)
    np.testing.assert_allclose(lin.weight.numpy(), w0 + 1.0, rtol=1e-6)


def test_auc_matches_sklearn():
    from sklearn.metrics import roc_auc_score
    rng = np.random.default_rng(0)
    p = rng.random(200)
    y = (rng.random(200) < p).astype("int64")
    prob = np.stack([1 - p, p], 1).astype("float32")
    a, _, _ = paddle.static.auc(paddle.to_tensor(prob), paddle.to_tensor(y))
    assert abs(float(a) - roc_auc_score(y, p)) < 2e-3


def test_forward_grad_is_jvp():
    from paddlepaddle_amd.incubate.autograd import forward_grad
    x = paddle.to_tensor([1.0, 2.0, 3.0])
    x.stop_gradient = False
    y = x * x * x
    v = paddle.to_tensor([1.0, 0.5, 2.0])
    jv = forward_grad(y, x, v)
    np.testing.assert_allclose(jv.numpy(), 3 * np.array([1.0, 4.0, 9.0]) * v.numpy(), rtol=1e-6)


def test_fp8_gemm_fallback_cpu():
    x = torch.randn(16, 32).to(torch.float8_e4m3fn)
    y = torch.randn(32, 8).to(torch.float8_e4m3fn)
    out = paddle.linalg.fp8_fp8_half_gemm_fused(paddle.Tensor(x), paddle.Tensor(y), scale=0.5,
                                                output_dtype="bfloat16")
    ref = 0.5 * (x.float() @ y.float())
    np.testing.assert_allclose(out._t.float().numpy(), ref.numpy(), rtol=2e-2, atol=2e-2)


def test_block_diag_and_misc():
    out = paddle.block_diag([paddle.to_tensor([[1, 2]]), paddle.to_tensor([3])])
    np.testing.assert_array_equal(out.numpy(), [[1, 2, 0], [0, 0, 3]])
    assert os.path.isdir(paddle.sysconfig.get_lib())
    paddle.utils.require_version("2.0.0")
    with pytest.raises(Exception):
        paddle.utils.require_version("99.0")
    assert paddle.distributed.ProbabilityEntry(0.2)._to_attr() == "probability_entry:0.2"
    fs = paddle.distributed.fleet.utils.LocalFS()
    assert fs.is_exist("/")
    import paddlepaddle_amd.sparse.nn.functional as SF  # noqa: F401
    import paddlepaddle_amd.audio.features as AF  # noqa: F401


def _ref_all(mod):
    p = os.path.join(REF, *mod.split("."))
    f = p + ".py" if os.path.exists(p + ".py") else os.path.join(p, "__init__.py")
    if not os.path.exists(f):
        return None
    for node in ast.parse(open(f).read()).body:
        if isinstance(node, ast.Assign) and any(getattr(t, "id", None) == "__all__" for t in node.targets):
            try:
                return [e.value for e in node.value.elts]
            except AttributeError:
                return None
    return []


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not mounted")
@pytest.mark.parametrize("mod", ["", "nn", "nn.functional", "optimizer", "optimizer.lr", "amp", "io", "static",
                                 "static.nn", "jit", "distributed", "distributed.fleet", "vision.models", "vision.ops",
                                 "vision.transforms", "metric", "linalg", "fft", "signal", "sparse", "distribution",
                                 "profiler", "autograd", "incubate", "incubate.nn.functional", "quantization",
                                 "text", "geometric", "nn.initializer", "utils", "device", "inference"])
def test_reference_all_coverage(mod):
    names = _ref_all(mod) if mod else _ref_all("")
    if mod == "":
        names = None
        for node in ast.parse(open(os.path.join(REF, "__init__.py")).read()).body:
            if isinstance(node, ast.Assign) and any(getattr(t, "id", None) == "__all__" for t in node.targets):
                names = [e.value for e in node.value.elts]
    if not names:
        pytest.skip("no __all__")
    m = importlib.import_module("paddlepaddle_amd" + ("." + mod if mod else ""))
    missing = [n for n in names if not hasattr(m, n)]
    assert not missing, f"paddle.{mod} missing {missing}"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not mounted")
def test_reference_tensor_methods_coverage():
    names = None
    for node in ast.parse(open(os.path.join(REF, "tensor", "__init__.py")).read()).body:
        if isinstance(node, ast.Assign) and any(getattr(t, "id", None) == "tensor_method_func" for t in node.targets):
            names = [e.value for e in node.value.elts]
    missing = [n for n in names if not hasattr(paddle.Tensor, n)]
    assert not missing, missing


def test_top_p_sampling_respects_nucleus():
    x = paddle.to_tensor([[0.05, 0.6, 0.3, 0.05]] * 64)
    _, ids = paddle.top_p_sampling(x, paddle.to_tensor([0.5] * 64), seed=3)
    assert set(ids.numpy().ravel().tolist()) == {1}
    _, ids = paddle.top_p_sampling(x, paddle.to_tensor([0.85] * 64), seed=3)
    assert set(ids.numpy().ravel().tolist()) <= {1, 2}


def test_legacy_reader_decorators():
    r = paddle.reader.compose(lambda: iter([1, 2, 3]), lambda: iter([(4,), (5,), (6,)]))
    assert list(r()) == [(1, 4), (2, 5), (3, 6)]
    assert list(paddle.reader.chain(lambda: iter([1]), lambda: iter([2, 3]))()) == [1, 2, 3]
    assert sorted(paddle.reader.buffered(lambda: iter(range(5)), 2)()) == list(range(5))
    assert list(paddle.reader.xmap_readers(lambda x: x + 1, lambda: iter(range(8)), 3, 4, order=True)()) == \
        list(range(1, 9))
    c = paddle.reader.cache(lambda: iter([7, 8]))
    assert list(c()) == [7, 8] and list(c()) == [7, 8]


def test_hub_local(tmp_path):
    (tmp_path / "hubconf.py").write_text("def tiny(scale=1):\n    '''tiny model'''\n    return scale * 3\n")
    assert "tiny" in paddle.hub.list(str(tmp_path), source="local")
    assert paddle.hub.help(str(tmp_path), "tiny", source="local") == "tiny model"
    assert paddle.hub.load(str(tmp_path), "tiny", source="local", scale=2) == 6


def test_c_ops_and_base_namespaces():
    out = paddle._C_ops.add(paddle.ones([2]), paddle.ones([2]))
    np.testing.assert_array_equal(out.numpy(), [2, 2])
    x = paddle.ones([2])
    paddle._C_ops.scale_(x, 3.0)
    np.testing.assert_array_equal(x.numpy(), [3, 3])
    assert paddle.base.framework.in_dygraph_mode()
    assert paddle.base.Program is paddle.static.Program
