"""Fused gradient accumulation in the fleet pipeline engine (parallel/pipeline.py _fuse_grad_accumulation;
reference: paddle/phi/kernels/fusion/gpu/fused_linear_param_grad_add_kernel.cu): the weight-gradient GEMM of every
micro-batch adds into the parameter's .grad buffer in its epilogue instead of autograd adding a fresh dW. Training
must match autograd accumulation; the gradient buffers stay the same storage across steps."""
import os
import socket
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _train(paddle, fused, steps=3):
    from paddlepaddle_amd.distributed import fleet
    from paddlepaddle_amd.models.llama import LlamaConfig, LlamaForCausalLMPipe
    paddle.set_flags({"FLAGS_fused_grad_accumulation": fused})
    paddle.set_default_dtype("bfloat16")
    paddle.seed(7)
    cfg = LlamaConfig.tiny(num_hidden_layers=2)
    pipe = LlamaForCausalLMPipe(cfg)
    paddle.set_default_dtype("float32")
    opt = paddle.optimizer.AdamW(1e-3, parameters=pipe.parameters(), multi_precision=True)
    model = fleet.distributed_model(pipe)
    opt = fleet.distributed_optimizer(opt)
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, cfg.vocab_size, (8, 33), generator=g).cuda()
    x, y = paddle.Tensor(ids[:, :-1].contiguous()), paddle.Tensor(ids[:, 1:].contiguous())
    losses, ptrs = [], []
    for _ in range(steps):
        losses.append(float(model.train_batch([x, y], opt)))
        regs = getattr(model, "_mg_params", None) or []
        ptrs.append(tuple(p._t.grad.data_ptr() for p in regs))
    return losses, model, ptrs


def test_fused_grad_accumulation_matches_autograd():
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import paddlepaddle_amd as paddle
    from paddlepaddle_amd.distributed import fleet
    paddle.set_device("gpu:0")
    s = fleet.DistributedStrategy()
    s.hybrid_configs = dict(dp_degree=1, mp_degree=1, pp_degree=1)
    s.pipeline_configs = {"accumulate_steps": 4, "micro_batch_size": 2}
    fleet.init(is_collective=True, strategy=s)
    try:
        fused, model, ptrs = _train(paddle, True)
        assert len(model._mg_params) >= 10  # every linear / norm weight of the two layers (+ head)
        assert len(set(ptrs)) == 1  # the same gradient storage every step
        ref, _, _ = _train(paddle, False)
        torch.testing.assert_close(torch.tensor(fused), torch.tensor(ref), rtol=2e-2, atol=2e-2)
    finally:
        paddle.set_flags({"FLAGS_fused_grad_accumulation": True})
