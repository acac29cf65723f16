"""Fused gradient accumulation (ops/linear.py fuse_grad_accumulation, used by the fleet pipeline engine and the
bench's accumulation loop; reference: paddle/phi/kernels/fusion/gpu/fused_linear_param_grad_add_kernel.cu): the
weight-gradient GEMM of every micro-batch adds into the parameter's .grad buffer in its epilogue (norm weights: the
norm backward kernels add their column sums) instead of autograd adding a fresh dW. Training must match autograd
accumulation; the gradient buffers stay the same storage across steps."""
import pytest
import torch

import paddlepaddle_amd as paddle
from paddlepaddle_amd.ops import linear as LIN

pytestmark = pytest.mark.gpu


def _train(fused, steps=3, accum=4):
    from paddlepaddle_amd.models.llama import LlamaConfig, LlamaForCausalLM
    paddle.set_device("gpu:0")
    paddle.set_flags({"FLAGS_fused_grad_accumulation": fused})
    paddle.set_default_dtype("bfloat16")
    paddle.seed(7)
    cfg = LlamaConfig.tiny(num_hidden_layers=2)
    model = LlamaForCausalLM(cfg)
    paddle.set_default_dtype("float32")
    opt = paddle.optimizer.AdamW(1e-3, parameters=model.parameters(), multi_precision=True)
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, cfg.vocab_size, (8, 65), generator=g).cuda()
    mbs = [(paddle.Tensor(a), paddle.Tensor(b)) for a, b in zip(ids[:, :-1].chunk(accum), ids[:, 1:].chunk(accum))]
    losses, ptrs, params = [], [], None
    for _ in range(steps):
        params = LIN.fuse_grad_accumulation(model, params)
        tot = 0.0
        for x, y in mbs:
            logits = model(x)
            loss = paddle.nn.functional.cross_entropy(logits.astype("float32").reshape([-1, cfg.vocab_size]),
                                                      y.reshape([-1])) * (1.0 / accum)
            loss.backward()
            tot += float(loss)
        opt.step()
        opt.clear_grad()
        losses.append(tot)
        ptrs.append(tuple(p._t.grad.data_ptr() for p in params))
    return losses, params, ptrs


def test_fused_grad_accumulation_matches_autograd():
    try:
        fused, params, ptrs = _train(True)
        assert len(params) >= 10  # the linear / norm weights of the two layers
        assert len(set(ptrs)) == 1  # the same gradient storage every step
        ref, pr, _ = _train(False)
        assert pr == []
        torch.testing.assert_close(torch.tensor(fused), torch.tensor(ref), rtol=2e-2, atol=2e-2)
    finally:
        paddle.set_flags({"FLAGS_fused_grad_accumulation": True})
