"""One LLaMA-2 70B decoder layer (h 8192, 64 query / 8 KV heads, ffn 28672), bf16, forward + backward at
B x S tokens on one GPU: ms per layer step and achieved TFLOP/s (6 * layer params * tokens + causal attention).
The per-layer view of the BASELINE's LLaMA-2 70B PP4 x TP2 path (tp 1 here: the full layer on one GPU)."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import paddlepaddle_amd as paddle
from paddlepaddle_amd.models.llama import LlamaConfig, LlamaDecoderLayer


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    paddle.set_device("gpu:0")
    paddle.seed(0)
    cfg = LlamaConfig.llama2_70b()
    layer = LlamaDecoderLayer(cfg)
    layer.to(dtype="bfloat16")
    B, S, h = a.batch, a.seq, cfg.hidden_size
    x = paddle.Tensor(torch.randn(B, S, h, device="cuda", dtype=torch.bfloat16).requires_grad_(True))
    x.stop_gradient = False
    gy = paddle.Tensor(torch.randn(B, S, h, device="cuda", dtype=torch.bfloat16))

    params = [p._t for p in layer.parameters()]

    def step():
        # fresh gradients each step (a training step's optimizer consumes them): autograd hands the new gradient
        # over instead of accumulating into the previous step's (no bf16 grad += kernels in the profile)
        for t in params + [x._t]:
            t.grad = None
        y = layer(x)
        y.backward(gy)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / a.steps
    n = sum(p._t.numel() for p in layer.parameters())
    flops = 6 * n * B * S + 6 * h * S * B * S  # causal attention: half of 12 h S^2 per sequence
    print(json.dumps({"layer": "llama2-70b", "batch": B, "seq": S, "ms": round(ms, 3),
                      "tflops": round(flops / ms / 1e9, 1), "params": n}))


if __name__ == "__main__":
    main()
