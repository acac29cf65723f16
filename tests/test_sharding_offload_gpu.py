"""Sharding optimizer-state offload on the GPU: same losses as the resident run, less HBM held between steps.
Reference: python/paddle/distributed/fleet/meta_parallel/sharding/group_sharded_stage3.py:98-127 (offload)."""
import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle

pytestmark = pytest.mark.gpu


class _Net(paddle.nn.Layer):
    def __init__(self, d=512, n=4):
        super().__init__()
        self.blocks = paddle.nn.LayerList([paddle.nn.Linear(d, d) for _ in range(n)])
        self.head = paddle.nn.Linear(d, 1)

    def forward(self, x):
        for b in self.blocks:
            x = paddle.nn.functional.gelu(b(x))
        return self.head(x)


def _run(offload):
    import gc
    gc.collect()
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    paddle.seed(7)
    net = _Net()
    opt = paddle.optimizer.AdamW(1e-3, parameters=net.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    from paddlepaddle_amd.distributed.sharding import group_sharded_parallel
    model, opt, _ = group_sharded_parallel(net, opt, level="os_g", offload=offload)
    rng = np.random.RandomState(0)
    x = paddle.to_tensor(rng.randn(64, 512).astype("float32"))
    y = paddle.to_tensor(rng.randn(64, 1).astype("float32"))
    losses = []
    for _ in range(4):
        loss = ((model(x) - y) ** 2).mean()
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    torch.cuda.synchronize()
    torch.empty(1, device="cuda")  # lets the allocator retire blocks freed behind the copy stream
    mem = torch.cuda.memory_allocated() - base  # what this run keeps resident between steps
    eng = model._engine
    return losses, mem, eng.offloaded_bytes(), (model, opt)


def test_offload_matches_and_frees_hbm():
    ref, mem_ref, off_ref, keep = _run(False)
    del keep
    got, mem_off, off_bytes, keep2 = _run(True)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)
    assert off_ref == 0
    n_params = sum(int(np.prod(p.shape)) for p in keep2[0].parameters())
    assert off_bytes >= 8 * n_params  # two fp32 moments per parameter live on the host
    # the moments are not resident in HBM any more (allow slack for the allocator's rounding)
    assert mem_ref - mem_off >= 0.8 * 8 * n_params, (mem_ref, mem_off, n_params)
    d = keep2[1]._inner._accumulators["moment1"]
    assert all(t.device.type == "cpu" and t.is_pinned() for t in d.values())
