"""Weight-gradient pairing across accumulation micro-batches (ops/linear.py pair_weight_grads) and the two-segment
K GEMM under it (ops.gemm.gemm_seg, csrc/kernels/gemm.hip pa_gemm_bf16_pp_seg): the merged product against an
fp32 reference, and sharded GPT training with pairing == without."""
import numpy as np
import pytest
import torch

import paddlepaddle_amd as paddle
from paddlepaddle_amd.ops import _loader as L
from paddlepaddle_amd.ops import gemm as G
from paddlepaddle_amd.ops import linear as LIN

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K1,K2,out_dt", [(1024, 2048, 4096, 4096, torch.bfloat16),
                                            (768, 1280, 256, 448, torch.float32),
                                            (5120, 5120, 4096, 4096, torch.bfloat16)])
def test_gemm_seg_matches_fp32(M, N, K1, K2, out_dt):
    assert L.has("pa_gemm_bf16_pp_segs")
    torch.manual_seed(0)
    xa = torch.randn(K1, M, device="cuda", dtype=torch.bfloat16)
    xb = torch.randn(K2, M, device="cuda", dtype=torch.bfloat16)
    da = torch.randn(K1, N, device="cuda", dtype=torch.bfloat16)
    db = torch.randn(K2, N, device="cuda", dtype=torch.bfloat16)
    acc0 = torch.randn(M, N, device="cuda").to(out_dt)
    acc = acc0.clone()
    assert G.gemm_seg_supported(xa.t(), xb.t(), da, db)
    G.gemm_seg(xa.t(), xb.t(), da, db, out=acc, accumulate=True)
    ref = acc0.float() + xa.t().float() @ da.float() + xb.t().float() @ db.float()
    err = (acc.float() - ref).abs().max() / ref.abs().max()
    assert err < (1e-2 if out_dt == torch.bfloat16 else 1e-3), err


def _run(pair, steps=2, accum=4):
    from paddlepaddle_amd.distributed.sharding import group_sharded_parallel
    from paddlepaddle_amd.models.gpt import GPTConfig, GPTForPretraining, GPTPretrainingCriterion
    paddle.set_device("gpu:0")
    paddle.seed(5)
    paddle.set_default_dtype("bfloat16")
    try:
        cfg = GPTConfig.tiny(hidden_size=256, num_attention_heads=4, intermediate_size=1024, num_hidden_layers=2,
                             hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
        model = GPTForPretraining(cfg)
    finally:
        paddle.set_default_dtype("float32")
    crit = GPTPretrainingCriterion(cfg)
    opt = paddle.optimizer.AdamW(1e-3, parameters=model.parameters(), multi_precision=True)
    model, opt, _ = group_sharded_parallel(model, opt, level="p_g_os")
    g = torch.Generator(device="cuda").manual_seed(1)
    data = torch.randint(0, cfg.vocab_size, (accum, 2, 129), device="cuda", generator=g)
    merges = 0
    for _ in range(steps):
        for a in range(accum):
            mode = ("defer" if a % 2 == 0 and a + 1 < accum else "merge") if pair else None
            with LIN.pair_weight_grads(mode):
                loss = crit(model(paddle.Tensor(data[a, :, :-1])), paddle.Tensor(data[a, :, 1:])) * (1.0 / accum)
                loss.backward()
                if mode == "defer":
                    merges += LIN.pending_weight_grads()
        assert LIN.pending_weight_grads() == 0
        opt.step()
        opt.clear_grad()
    return {k: v.astype("float32").numpy() for k, v in model.state_dict().items()}, merges


def test_paired_weight_grads_train_like_unpaired():
    ref, _ = _run(False)
    got, merges = _run(True)
    assert merges > 0  # linears' dW GEMMs really were queued and paired
    for k in ref:
        np.testing.assert_allclose(got[k], ref[k], rtol=2e-2, atol=2e-3, err_msg=k)
