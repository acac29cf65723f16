"""Forward-weight layout cache of ops.fused_linear (TN-form forward GEMM): results must track in-place
weight updates (version counter), optimizer steps (epoch bump) and stay numerically identical to the
plain NN-form product."""
import pytest
import torch

import paddlepaddle_amd as paddle
from paddlepaddle_amd import ops
from paddlepaddle_amd.ops import linear as LN


@pytest.mark.gpu
def test_fused_linear_weight_cache_tracks_updates():
    paddle.set_flags({"FLAGS_linear_wt_cache_mb": 1024})
    try:
        _check()
    finally:
        paddle.set_flags({"FLAGS_linear_wt_cache_mb": 0})


def _check():
    dev = torch.device("cuda")
    x = torch.randn(64, 256, device=dev, dtype=torch.bfloat16)
    w = torch.randn(256, 512, device=dev, dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(512, device=dev, dtype=torch.bfloat16, requires_grad=True)
    ref = (x.float() @ w.float() + b.float())
    y = ops.fused_linear(x, w, b)
    assert (y.float() - ref).abs().max() < 0.5
    assert id(w) in LN._WT  # the TN copy is in use
    with torch.no_grad():
        w.mul_(0.5)  # in-place update bumps the version counter -> cache refresh
    y2 = ops.fused_linear(x, w, b)
    ref2 = x.float() @ w.float() + b.float()
    assert (y2.float() - ref2).abs().max() < 0.5
    # a real optimizer step drops the cache
    lin = paddle.nn.Linear(256, 512)
    lin.to(device="gpu", dtype="bfloat16")
    opt = paddle.optimizer.SGD(0.1, parameters=lin.parameters())
    xt = paddle.Tensor(x)
    out = lin(xt)
    out.astype("float32").sum().backward()
    opt.step()
    assert len(LN._WT) == 0
    out2 = lin(xt)
    exp = x.float() @ lin.weight._t.float() + lin.bias._t.float()
    assert (out2._t.float() - exp).abs().max() < 0.5
