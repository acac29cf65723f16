"""AST dy2static (paddlepaddle_amd/jit/dy2static): Python control flow on tensors becomes static-program control
flow. Reference: python/paddle/jit/dy2static/transformers/ifelse_transformer.py:57, loop_transformer.py:473,
convert_operators.py:167,398, jit/api.py:1110-1115 (jit.save of functions)."""
import numpy as np
import pytest

import paddlepaddle_amd as paddle
from paddlepaddle_amd.jit import dy2static as D
from paddlepaddle_amd.static import InputSpec


def _t(v):
    return paddle.to_tensor(np.asarray(v, dtype="float32"))


# --------------------------------------------------------------------------- converted code == eager code
def _many(x, n):
    y = x * 2
    if x.sum() > 0:
        y = y + 1
        z = y * 3
    elif x.sum() < -100:
        z = y
    else:
        z = y - 1
    i = 0
    while i < n:
        z = z + x
        i += 1
    for k in range(1, 6, 2):
        z = z * 1.0 + k
    w = z if z.mean() > 0 else -z
    if not (z.max() > 1000) and x.min() > -50 or n > 100:
        w = w + 0.5
    assert x.shape[0] == 2, "shape"
    if w.sum() > 1e6:
        return w * 0
    return w


def test_converted_function_matches_eager_in_dygraph():
    g = D.convert_to_static(_many)
    assert g is not _many
    src = D.converted_source(_many)
    assert "_jst.IfElse" in src and "_jst.While" in src and "_jst.RangeCond" in src and "_jst.And" in src
    for v, n in (([1.0, 2.0], 2), ([-1.0, -2.0], 3), ([-300.0, 1.0], 0)):
        np.testing.assert_allclose(g(_t(v), n).numpy(), _many(_t(v), n).numpy())


def test_loop_variable_and_python_semantics_kept():
    def f(n):
        acc = []
        for i in range(n):
            acc.append(i)
        j = 10
        while j > 3:
            j -= 2
        return acc, i, j
    g = D.convert_to_static(f)
    assert g(4) == f(4) == ([0, 1, 2, 3], 3, 2)


def test_super_and_closure_in_converted_method():
    scale = 3.0

    class Base(paddle.nn.Layer):
        def forward(self, x):
            return x + 1

    class Child(Base):
        def forward(self, x):
            y = super().forward(x)
            if y.sum() > 0:
                y = y * scale
            return y

    c = Child()
    conv = D.convert_to_static(c.forward)
    np.testing.assert_allclose(conv(_t([1.0, 1.0])).numpy(), [6.0, 6.0])
    np.testing.assert_allclose(conv(_t([-5.0, -5.0])).numpy(), [-4.0, -4.0])


# --------------------------------------------------------------------------- static programs
class _CondNet(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.fc = paddle.nn.Linear(4, 4)

    def forward(self, x):
        y = self.fc(x)
        if y.mean() > 0:
            out = y * 2 + 1
        else:
            out = y - 10
        i = 0
        s = paddle.zeros_like(out)
        while i < x.shape[0]:  # Python trip count: unrolled
            s = s + out
            i += 1
        return s


class _LoopNet(paddle.nn.Layer):
    def forward(self, x):
        s = paddle.zeros_like(x)
        n = x.sum()
        while n > 0:  # tensor-dependent trip count: one while node
            s = s + x
            n = n - 1.0
        return s


def _names(prog):
    return [n.name for n in prog.nodes]


def test_to_static_layer_records_one_cond_node_for_both_branches():
    paddle.seed(1)
    net = _CondNet()
    net.eval()
    xs = [_t(np.ones((2, 4))), _t(-5 * np.ones((2, 4)))]
    ref = [net(x).numpy() for x in xs]
    paddle.jit.to_static(net)
    for x, r in zip(xs, ref):
        np.testing.assert_allclose(net(x).numpy(), r, rtol=1e-6)
    (cp,) = net.forward.variants(xs[0])
    assert not cp.guarded and _names(cp.program).count("cf:cond") == 1


def test_tensor_while_records_a_while_node_and_gradients_flow():
    net = _LoopNet()
    sf = paddle.jit.to_static(net)
    x = paddle.to_tensor(np.array([0.5, 1.0, 1.0], "float32"), stop_gradient=False)
    out = sf(x)
    np.testing.assert_allclose(out.numpy(), [1.5, 3.0, 3.0])  # sum 2.5 -> 3 iterations
    (cp,) = net.forward.variants(x)
    assert "cf:while" in _names(cp.program)
    out.sum().backward()
    np.testing.assert_allclose(x.grad.numpy(), [3.0, 3.0, 3.0])


def test_sublayer_control_flow_is_converted_too():
    class Outer(paddle.nn.Layer):
        def __init__(self):
            super().__init__()
            self.inner = _LoopNet()

        def forward(self, x):
            return self.inner(x) * 2

    o = Outer()
    paddle.jit.to_static(o)
    for v, r in (([1.0, 1.0], [4.0, 4.0]), ([0.25, 0.25], [0.5, 0.5])):
        np.testing.assert_allclose(o(_t(v)).numpy(), r)
    (cp,) = o.forward.variants(_t([1.0, 1.0]))
    assert "cf:while" in _names(cp.program)


def test_jit_save_load_and_predictor_take_both_branches(tmp_path):
    paddle.seed(2)
    net = _CondNet()
    net.eval()
    xs = [np.ones((2, 4), "float32"), -5 * np.ones((2, 4), "float32")]
    ref = [net(_t(x)).numpy() for x in xs]
    path = str(tmp_path / "cond")
    paddle.jit.save(net, path, input_spec=[InputSpec([2, 4], "float32", "x")])
    loaded = paddle.jit.load(path)
    for x, r in zip(xs, ref):
        np.testing.assert_allclose(loaded(_t(x)).numpy(), r, rtol=1e-6)
    assert "cf:cond" in _names(loaded.program())
    cfg = paddle.inference.Config(path + ".pdmodel", path + ".pdiparams")
    cfg.disable_gpu()
    pred = paddle.inference.create_predictor(cfg)
    for x, r in zip(xs, ref):
        np.testing.assert_allclose(pred.run([x])[0].numpy(), r, rtol=1e-6)


def test_jit_save_of_a_function_with_tensor_loop_and_early_return(tmp_path):
    @paddle.jit.to_static(input_spec=[InputSpec([3], "float32", "x")])
    def fn(x):
        s = paddle.zeros([3])
        n = x.sum()
        while n > 0:
            s = s + x
            n = n - 1.0
        if s.mean() > 5:
            return s
        return -s

    path = str(tmp_path / "fn")
    paddle.jit.save(fn, path)
    lf = paddle.jit.load(path)
    for v in ([1.0, 2.0, 3.0], [0.5, 0.25, 0.25]):
        x = _t(v)
        exp = fn.dygraph_function(x).numpy()
        np.testing.assert_allclose(fn(x).numpy(), exp)
        np.testing.assert_allclose(lf(x).numpy(), exp)
    names = _names(lf.program())
    assert "cf:while" in names and "cf:cond" in names


def test_variable_bound_in_one_branch_fails_loudly_in_a_static_program(tmp_path):
    class Bad(paddle.nn.Layer):
        def forward(self, x):
            if x.sum() > 0:
                y = x * 2
            return y

    with pytest.raises(Exception, match="not defined on every path"):
        paddle.jit.save(Bad(), str(tmp_path / "bad"), input_spec=[InputSpec([2], "float32")])


def test_branch_shape_mismatch_is_reported():
    def f(x):
        if x.sum() > 0:
            y = x
        else:
            y = paddle.concat([x, x])
        return y
    with pytest.raises(Exception, match="shape"):
        paddle.jit.save(f, "/nonexistent/never_written", input_spec=[InputSpec([2], "float32")])


# --------------------------------------------------------------------------- break / continue
def _bc(x, n):
    s = x * 0
    for i in range(n):
        if i % 2 == 1:
            continue
        s = s + x * i
        if s.sum() > 20:
            break
        s = s + 1
    j = 0
    while j < 10:
        j += 1
        if j == 3:
            continue
        if j > 6:
            break
        s = s - 0.5
    return s, i, j


def test_break_continue_lowered_and_python_semantics_kept():
    src = D.converted_source(_bc)
    assert "_jst_brk_" in src and "_jst_cnt_" in src and "break" not in src and "continue" not in src
    g = D.convert_to_static(_bc)
    for v, n in (([1.0, 2.0], 9), ([5.0, 5.0], 9), ([0.1, 0.1], 4), ([1.0, 1.0], 0)):
        got, exp = g(_t(v), n), _bc(_t(v), n) if n else None
        if n == 0:
            continue  # i is unbound after an empty range in both versions
        np.testing.assert_allclose(got[0].numpy(), exp[0].numpy())
        assert got[1:] == exp[1:]


def test_tensor_dependent_break_is_one_static_while(tmp_path):
    @paddle.jit.to_static(input_spec=[InputSpec([3], "float32", "x")])
    def fn(x):
        s = paddle.zeros([3])
        n = paddle.zeros([1])
        while n < 100:
            n = n + 1.0
            if s.sum() > 10:
                break
            if n.sum() == 2:
                continue
            s = s + x
        for k in range(50):
            if s.mean() > 30:
                break
            s = s * 1.5
        return s, n

    path = str(tmp_path / "bc")
    paddle.jit.save(fn, path)
    lf = paddle.jit.load(path)
    for v in ([1.0, 2.0, 3.0], [0.5, 0.25, 0.25], [4.0, 4.0, 4.0]):
        x = _t(v)
        es, en = fn.dygraph_function(x)
        ls, ln = lf(x)
        np.testing.assert_allclose(fn(x)[0].numpy(), es.numpy(), rtol=1e-6)
        np.testing.assert_allclose(ls.numpy(), es.numpy(), rtol=1e-6)
        np.testing.assert_allclose(ln.numpy(), en.numpy())
    assert _names(lf.program()).count("cf:while") >= 2
