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
        eager = S.eager_1f1b(p, s, n)
        S.check(eager, n, False)
        # 2 (p - s) - 1 forwards before the first backward (capped by the micro-batch count)
        assert [k for k, _ in eager[:min(2 * (p - s) - 1, n)]] == ["F"] * min(2 * (p - s) - 1, n)
    with pytest.raises(ValueError):
        S.schedule("nope", 2, 0, 2)


@pytest.mark.parametrize("p,n,v", [(2, 2, 2), (2, 4, 2), (4, 8, 2), (4, 4, 3)])
def test_vpp_job_lists_cover_every_chunk(p, n, v):
    for s in range(p):
        jobs = S.vpp(p, s, n, v)
        fw = [(S.vpp_mb(k, p, v), S.vpp_chunk(k, p, v, True)) for kind, k in jobs if kind == "F"]
        bw = [(S.vpp_mb(k, p, v), S.vpp_chunk(k, p, v, False)) for kind, k in jobs if kind == "B"]
        assert sorted(fw) == sorted(bw) == sorted((m, c) for m in range(n) for c in range(v))
        for m in range(n):  # chunks of a micro-batch run forward in order and backward in reverse order
            assert [c for mb, c in fw if mb == m] == list(range(v))
            assert [c for mb, c in bw if mb == m] == list(range(v))[::-1]
    with pytest.raises(ValueError):
        S.vpp(4, 0, 6, 2)


def test_pipeline_scheduler_passes_build_job_lists():
    """pipeline_scheduler_<mode> passes (reference pipeline_scheduler_pass/): the stage's job list, optimizer job
    last, on the program and in the pass context."""
    from paddlepaddle_amd.distributed.passes import new_pass
    from paddlepaddle_amd.distributed.passes.pipeline_scheduler import OPT, job_pairs
    from paddlepaddle_amd.static import program as P
    fns = {"FThenB": S.fthenb, "1F1B": S.one_f_one_b, "Eager1F1B": S.eager_1f1b, "ZBH1": S.zbh1}
    for name, fn in fns.items():
        prog = P.Program()
        ctx = new_pass(f"pipeline_scheduler_{name}", {"num_micro_batches": 8, "pp_stage": 1,
                                                      "pp_degree": 4}).apply(prog, None)
        jobs = ctx.get_attr("pipeline_scheduler.job_list")
        assert jobs is prog._pa_jobs and jobs[-1].type() == OPT
        assert job_pairs(jobs) == fn(4, 1, 8)
    prog = P.Program()
    ctx = new_pass("pipeline_scheduler_VPP", {"num_micro_batches": 4, "pp_stage": 0, "pp_degree": 2,
                                              "vpp_degree": 2}).apply(prog, None)
    jobs = ctx.get_attr("pipeline_scheduler.job_list")
    assert len(jobs) == 2 * 4 * 2 + 1 and {j.chunk_id() for j in jobs[:-1]} == {0, 1}
    ctx = new_pass("pipeline_scheduler_ZBVPP", {"num_micro_batches": 4, "pp_stage": 0, "pp_degree": 2,
                                                "vpp_degree": 2}).apply(P.Program(), None)
    jobs = ctx.get_attr("pipeline_scheduler.job_list")
    assert len(jobs) == 3 * 4 * 2 + 1 and sum(j.type() == "backward_w" for j in jobs) == 8
    # missing attributes: the pass does not apply
    assert new_pass("pipeline_scheduler_1F1B").apply(P.Program(), None).get_attr(
        "pipeline_scheduler.job_list") is None


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
