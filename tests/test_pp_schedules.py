"""Pipeline job lists (parallel/pp_schedules.py; reference pipeline_scheduler_pass/) and the weight-gradient
deferral the zero-bubble schedule runs on (ops/linear.py defer_weight_grads / apply_weight_grads)."""
import numpy as np
import pytest
import torch

from paddlepaddle_amd.parallel import pp_schedules as S


@pytest.mark.parametrize("p,n", [(1, 1), (2, 2), (4, 4), (4, 8), (8, 16), (4, 2)])
def test_job_lists_are_valid(p, n):
    for s in range(p):
        S.check(S.fthenb(p, s, n), n, False)
        S.check(S.one_f_one_b(p, s, n), n, False)
        jobs = S.zbh1(p, s, n)
        S.check(jobs, n, True)
        # F/B order is exactly 1F1B's; at most warm + 1 weight gradients are ever pending
        assert [j for j in jobs if j[0] != "W"] == S.one_f_one_b(p, s, n)
        warm, pend, peak = min(p - s - 1, n), set(), 0
        for k, mb in jobs:
            if k == "B":
                pend.add(mb)
            elif k == "W":
                pend.discard(mb)
            peak = max(peak, len(pend))
        assert peak <= warm + 1
    with pytest.raises(ValueError):
        S.schedule("nope", 2, 0, 2)


def test_deferred_weight_grads_equal_fused_backward():
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.ops import linear as LIN
    paddle.seed(0)
    net = paddle.nn.Sequential(paddle.nn.Linear(8, 16), paddle.nn.GELU(), paddle.nn.Linear(16, 4))
    x = paddle.randn([5, 8])
    x.stop_gradient = False
    net(x).sum().backward()
    ref = {n: p.grad.numpy().copy() for n, p in net.named_parameters()}
    ref_dx = x.grad.numpy().copy()
    net.clear_gradients()
    x.clear_gradient()
    q = []
    with LIN.zero_bubble_forward():
        y = net(x)
    with LIN.defer_weight_grads(q):
        y.sum().backward()
    assert len(q) == 2
    np.testing.assert_allclose(x.grad.numpy(), ref_dx, rtol=1e-6)
    for w in (net[0].weight, net[2].weight):  # B only: dW pending (clear_gradients left zeros)
        assert w.grad is None or not w.grad.numpy().any()
    assert net[0].bias.grad.numpy().any()  # bias gradients are not deferred
    seen = []
    net[0].weight._t.register_post_accumulate_grad_hook(lambda t: seen.append(t))
    LIN.apply_weight_grads(q)
    assert q == [] and len(seen) == 1
    for n, p in net.named_parameters():
        np.testing.assert_allclose(p.grad.numpy(), ref[n], rtol=1e-5, atol=1e-6, err_msg=n)


@pytest.mark.gpu
def test_deferred_weight_grads_on_hip_linears():
    """The zero-bubble B/W split on the HIP linear path (bf16 _LinearFn / _LinearBiasGeluFn): dX from B, dW from
    the deferred W GEMMs, equal to the fused backward."""
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.ops import linear as LIN
    from paddlepaddle_amd.ops import _loader as L
    paddle.seed(0)
    x = torch.randn(256, 512, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w1 = (torch.randn(512, 1024, device="cuda") * 0.03).to(torch.bfloat16).requires_grad_(True)
    b1 = torch.zeros(1024, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w2 = (torch.randn(1024, 512, device="cuda") * 0.03).to(torch.bfloat16).requires_grad_(True)

    def f():
        return LIN.fused_linear(LIN.fused_linear(x, w1, b1, act="gelu"), w2).float().square().mean()
    f().backward()
    ref = [t.grad.clone() for t in (x, w1, b1, w2)]
    for t in (x, w1, b1, w2):
        t.grad = None
    q = []
    L.CALLS.clear()
    with LIN.zero_bubble_forward():
        y = f()
    with LIN.defer_weight_grads(q):
        y.backward()
    assert len(q) == 2 and w1.grad is None and w2.grad is None and x.grad is not None
    LIN.apply_weight_grads(q)
    assert sum(L.CALLS.values()) > 0
    for got, exp in zip((x.grad, w1.grad, b1.grad, w2.grad), ref):
        torch.testing.assert_close(got.float(), exp.float(), rtol=2e-2, atol=2e-3)
