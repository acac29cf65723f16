"""jit.to_static graph breaks: a Python conversion of tensor data (bool / item / tolist / numpy) makes the
trace guarded — one replayed program per observed data-dependent path, re-selected by its guards
(reference: python/paddle/jit/sot/translate.py:31 graph breaks + guards)."""
import warnings

import numpy as np
import pytest

import paddlepaddle_amd as paddle
from paddlepaddle_amd import jit as J


def _count_traces(monkeypatch):
    calls = []
    orig = J.trace_program

    def counting(*a, **k):
        calls.append(k.get("guarded", False))
        return orig(*a, **k)
    monkeypatch.setattr(J, "trace_program", counting)
    return calls


def test_branch_on_tensor_value_records_one_variant_per_path(monkeypatch):
    calls = _count_traces(monkeypatch)

    def f(x):
        if x.sum() > 0:
            return x * 2 + 1
        return x - 3

    sf = paddle.jit.to_static(f)
    pos = paddle.to_tensor(np.ones([4], "float32"))
    neg = paddle.to_tensor(-np.ones([4], "float32"))
    np.testing.assert_allclose(sf(pos).numpy(), f(pos).numpy())
    np.testing.assert_allclose(sf(neg).numpy(), f(neg).numpy())   # guard fails -> second variant
    np.testing.assert_allclose(sf(pos * 5).numpy(), f(pos * 5).numpy())
    np.testing.assert_allclose(sf(neg * 2).numpy(), f(neg * 2).numpy())
    vs = sf.variants(pos)
    # the AST conversion (jit/dy2static) turns the tensor-dependent if into one control-flow node: a single
    # unguarded program serves both paths, recorded once
    assert len(vs) == 1 and not vs[0].guarded
    assert [n.name for n in vs[0].program.nodes].count("cf:cond") == 1
    assert calls == [False]


def test_branch_on_host_value_records_one_variant_per_path(monkeypatch):
    """A branch on a host conversion (.numpy()) cannot be a program node: guarded variants, one per path."""
    calls = _count_traces(monkeypatch)

    def f(x):
        if (x.sum() > 0).numpy():
            return x * 2 + 1
        return x - 3

    sf = paddle.jit.to_static(f)
    pos = paddle.to_tensor(np.ones([4], "float32"))
    neg = paddle.to_tensor(-np.ones([4], "float32"))
    for v in (pos, neg, pos * 5, neg * 2):
        np.testing.assert_allclose(sf(v).numpy(), f(v).numpy())
    vs = sf.variants(pos)
    assert len(vs) == 2 and all(cp.guarded for cp in vs)
    assert [g.expected for g in vs[0].guards] in ([True], [False])
    # converted and plain meta traces fail once, then exactly two guarded traces (one per path)
    assert calls == [False, False, True, True]


def test_item_as_loop_trip_count_and_tolist():
    def g(x, y):
        n = int(x.max().item())
        for _ in range(n):
            y = y + 1.0
        shift = y.sum().tolist()
        return y * 0.5, shift

    sf = paddle.jit.to_static(g)
    for v in (2.0, 3.0, 2.0):
        x = paddle.to_tensor(np.array([1.0, v], "float32"))
        y = paddle.to_tensor(np.zeros([3], "float32"))
        out, shift = sf(x, y)
        ref, rshift = g(x, y)
        np.testing.assert_allclose(out.numpy(), ref.numpy())
        assert shift == rshift
    assert len(sf.variants(x, y)) == 2


def test_guarded_layer_trains_like_eager():
    class Net(paddle.nn.Layer):
        def __init__(self):
            super().__init__()
            self.a = paddle.nn.Linear(4, 4)
            self.b = paddle.nn.Linear(4, 4)

        def forward(self, x):
            h = self.a(x)
            if (h.mean() > 0).numpy():
                return self.b(h).sum()
            return (h * h).sum()

    paddle.seed(3)
    net = Net()
    ref = Net()
    ref.set_state_dict(net.state_dict())
    snet = paddle.jit.to_static(net)
    rs = np.random.RandomState(0)
    for _ in range(4):
        x = paddle.to_tensor(rs.randn(3, 4).astype("float32"))
        l1 = snet(x)
        l1.backward()
        l2 = ref(x)
        l2.backward()
        np.testing.assert_allclose(l1.numpy(), l2.numpy(), rtol=1e-6)
        for p, q in zip(net.parameters(), ref.parameters()):
            assert (p.grad is None) == (q.grad is None)  # the untaken branch's layer gets no gradient
            if p.grad is not None:
                np.testing.assert_allclose(p.grad.numpy(), q.grad.numpy(), rtol=1e-5, atol=1e-6)
            p.clear_gradient(set_to_zero=False)
            q.clear_gradient(set_to_zero=False)


def test_too_many_paths_fall_back_to_eager():
    def h(x):
        return x * int(x.sum().item())

    sf = paddle.jit.to_static(h)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        for k in range(J._MAX_VARIANTS + 2):
            x = paddle.to_tensor(np.full([2], float(k), "float32"))
            np.testing.assert_allclose(sf(x).numpy(), h(x).numpy())
    assert any("data-dependent paths" in str(m.message) for m in w)


def test_guarded_program_cannot_be_saved(tmp_path):
    def f(x):
        return x * 2 if bool(x.sum() > 0) else x

    sf = paddle.jit.to_static(f)
    x = paddle.to_tensor(np.ones([2], "float32"))
    sf(x)
    cp = sf.variants(x)[0]
    with pytest.raises(ValueError, match="guards"):
        cp.program.to_dict(cp.fetch_slots, {})
